#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run; writes gpurun_out/prof/<tag>_*.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-step}; shift
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o "$tag" --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --prefill-tokens 0 "$@" > gpurun_out/prof/${tag}_bench.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/prof/${tag}_bench.log | cut -c1-200
