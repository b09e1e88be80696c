#!/bin/bash
# GPU box: rocprofv3 kernel traces of the C4 (batch 8) and C3 (int8) benches + their step traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r03}
./tools/prof_step.sh ${tag}_c4 --preset llama3-8b --ctx 4096 --batch 8 || exit 1
./tools/prof_step.sh ${tag}_c3 --w-dtype i8 || exit 1
for w in c4 c3; do
  tr=$(find gpurun_out/prof -name "${tag}_${w}_kernel_trace.csv" | head -1)
  python3 tools/step_trace.py "$tr" > gpurun_out/prof/${tag}_${w}_step_trace.txt
  cat gpurun_out/prof/${tag}_${w}_step_trace.txt
done
