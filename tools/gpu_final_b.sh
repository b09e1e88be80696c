#!/bin/bash
# round-end evidence, part B: the MFMA counter pass (C4 and a 129-token prefill), the throughput sweeps, the
# loopback per-rank TP steps.   tools/gpu_final_b.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r4}
mkdir -p gpurun_out
bash tools/pmc_mfma.sh $tag llama3-8b/f16/tp1/b8 --preset llama3-8b --ctx 4096 --batch 8 --prefill-tokens 129 || exit 1
bash tools/sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/${tag}_sweep.txt
bash tools/gpu_tp_final.sh $tag || exit 1
echo part B done
