#!/bin/bash
# A/B the decode bench over environment settings: tools/ab_bench.sh "ENV=a" "ENV=b" ...
# (each setting runs bench.py once under its own time limit; prints tokens/s per setting)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for setting in "$@"; do
    env $setting timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 60 --warmup 10 > gpurun_out/ab.log 2>&1 || { echo "FAILED: $setting"; tail -5 gpurun_out/ab.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('%-40s %8.2f tok/s  %.4f ms  gemv %.1f GB/s' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['achieved']))" "$setting"
done
