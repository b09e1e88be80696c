#!/bin/bash
# round-end evidence, part A: FETCH_SIZE passes (C1, C3, C4) -> profiles/<tag>_gemv_traffic.json, then rocprofv3
# kernel stats + one-step traces of C1, C3, C4.   tools/gpu_final_a.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r3}
mkdir -p gpurun_out
KEY=llama2-7b/f16/tp1 ./tools/pmc_traffic.sh $tag || exit 1
KEY=llama2-7b/i8/tp1 ./tools/pmc_traffic.sh $tag --w-dtype i8 || exit 1
KEY=llama3-8b/f16/tp1/b8 ./tools/pmc_traffic.sh $tag --preset llama3-8b --ctx 4096 --batch 8 || exit 1
./tools/prof_step.sh ${tag}_c1 || exit 1
./tools/prof_step.sh ${tag}_c3 --w-dtype i8 || exit 1
./tools/prof_step.sh ${tag}_c4 --preset llama3-8b --ctx 4096 --batch 8 || exit 1
for c in c1 c3 c4; do
  python3 tools/step_trace.py $(find gpurun_out/prof -name "${tag}_${c}_kernel_trace.csv" | head -1) > gpurun_out/prof/${tag}_${c}_step_trace.txt
  tail -1 gpurun_out/prof/${tag}_${c}_step_trace.txt
done
find gpurun_out/prof -name '*_kernel_trace.csv' -delete
find gpurun_out/prof -name '*agent_info*' -delete
echo part A done
