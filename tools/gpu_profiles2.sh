#!/bin/bash
# GPU box: the second half of tools/gpu_profiles.sh (the prefill MFMA pass and the kernel-trace stats),
# for when the first half's results are already in.   tools/gpu_profiles2.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r2}
mkdir -p gpurun_out
(while sleep 30; do date >> gpurun_out/heartbeat.txt; done) &
hb=$!
trap 'kill $hb' EXIT
./tools/pmc_mfma.sh $tag llama2-7b/f16/tp1/prefill129 --prefill-tokens 129 --prefill-reps 1 || exit 1
./tools/prof_step.sh ${tag}_c1 --prefill-tokens 0 || exit 1
./tools/prof_step.sh ${tag}_c3 --w-dtype i8 --prefill-tokens 0 || exit 1
./tools/prof_step.sh ${tag}_c4 --preset llama3-8b --ctx 4096 --batch 8 || exit 1
for c in c1 c3 c4; do
  python3 tools/step_trace.py $(find gpurun_out/prof -name "${tag}_${c}_kernel_trace.csv" | head -1) > gpurun_out/prof/${tag}_${c}_step_trace.txt || exit 1
  tail -1 gpurun_out/prof/${tag}_${c}_step_trace.txt
done
echo profiles done
