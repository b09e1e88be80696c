#!/bin/bash
# Interleaved A/B of env-knob variants of the C1 bench (one process per run):
#   tools/ab_env.sh <rounds> "<env a>" "<env b>" ... [-- bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1; shift
vars=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
[ "$1" == "--" ] && shift
for r in $(seq 1 $rounds); do
  for v in "${vars[@]}"; do
    out=$(env $v timeout -k 10 240 python3 bench.py --no-cpu-baseline --prefill-tokens 0 --greedy-steps 2 --steps 100 --warmup 20 "$@" 2>gpurun_out/ab_err.log) || { echo "FAILED: $v"; tail -5 gpurun_out/ab_err.log; exit 1; }
    echo "$out" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['roofline']['families']
print('%-34s %8.1f tok/s %7.4f ms  ' % ('$v' or 'base', d['value'], d['ms_per_step']) + ' '.join('%s %.2f' % (k, v['avg_launch_us']) for k, v in f.items()), flush=True)"
  done
done
