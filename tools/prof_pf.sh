#!/bin/bash
# rocprofv3 kernel trace + stats of a 512-token prefill (fp16, 4 timed prompts); writes gpurun_out/prof/<tag>_*.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-pf}; shift
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o "$tag" --output-format csv -- python3 tools/prefill_time.py --tokens 512 --reps 4 "$@" > gpurun_out/prof/${tag}_run.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof/${tag}_run.log; exit 1; }
tail -1 gpurun_out/prof/${tag}_run.log
f=$(ls gpurun_out/prof/*${tag}*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/kstats.py "$f" 14
