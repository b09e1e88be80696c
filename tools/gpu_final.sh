#!/bin/bash
# GPU box, end of round: PMC traffic passes (C1, C3, C4) first so the bench lines carry roofline.traffic,
# then the gpu test suite, the three bench lines, and a rocprofv3 kernel trace of the C1 step.
#   tools/gpu_final.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r04}
mkdir -p gpurun_out
KEY=llama2-7b/f16/tp1 ./tools/pmc_traffic.sh $tag || exit 1
KEY=llama2-7b/i8/tp1 ./tools/pmc_traffic.sh $tag --w-dtype i8 || exit 1
KEY=llama3-8b/f16/tp1/b8 ./tools/pmc_traffic.sh $tag --preset llama3-8b --ctx 4096 --batch 8 || exit 1
cp gpurun_out/pmc/${tag}_gemv_traffic.json profiles/${tag}_gemv_traffic.json || exit 1
./tools/gpu_round.sh $tag || exit 1
./tools/prof_step.sh ${tag}_c1 || exit 1
./tools/prof_step.sh ${tag}_c3 --w-dtype i8 || exit 1
./tools/prof_step.sh ${tag}_c4 --preset llama3-8b --ctx 4096 --batch 8 || exit 1
for c in c1 c3 c4; do
  python3 tools/step_trace.py $(find gpurun_out/prof -name "${tag}_${c}_kernel_trace.csv" | head -1) > gpurun_out/prof/${tag}_${c}_step_trace.txt
  tail -1 gpurun_out/prof/${tag}_${c}_step_trace.txt
done
# keep the summaries (kernel stats, step traces) within gpurun's 64 MiB copy-back: drop the raw traces
find gpurun_out/prof -name '*_kernel_trace.csv' -delete
find gpurun_out/prof -name '*agent_info*' -delete
echo final done
