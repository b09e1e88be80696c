#!/bin/bash
# Round 6 evidence passes on one box: FETCH_SIZE traffic per family (C1, C3, C4; each its own --pmc pass) into
# gpurun_out/pmc/<tag>_gemv_traffic.json, then rocprofv3 kernel-trace stats + one-step traces of C1 / C3 / C4.
#   tools/gpu_r6_profiles.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6}
mkdir -p gpurun_out
(while sleep 30; do date >> gpurun_out/heartbeat.txt; done) &  # counter passes print nothing for minutes
hb=$!
trap 'kill $hb' EXIT
KEY=llama2-7b/f16/tp1 ./tools/pmc_traffic.sh $tag --prefill-tokens 0 || exit 1
KEY=llama2-7b/i8/tp1 ./tools/pmc_traffic.sh $tag --w-dtype i8 --prefill-tokens 0 || exit 1
KEY=llama3-8b/f16/tp1/b8 ./tools/pmc_traffic.sh $tag --preset llama3-8b --ctx 4096 --batch 8 || exit 1
./tools/prof_step.sh ${tag}_c1 --prefill-tokens 0 || exit 1
./tools/prof_step.sh ${tag}_c3 --w-dtype i8 --prefill-tokens 0 || exit 1
./tools/prof_step.sh ${tag}_c4 --preset llama3-8b --ctx 4096 --batch 8 || exit 1
for c in c1 c3 c4; do
  python3 tools/step_trace.py $(find gpurun_out/prof -name "${tag}_${c}_kernel_trace.csv" | head -1) > gpurun_out/prof/${tag}_${c}_step_trace.txt || exit 1
  tail -1 gpurun_out/prof/${tag}_${c}_step_trace.txt
done
echo profiles done
