#!/bin/bash
# A/B two prebuilt libsli.so variants (exp/libsli_a.so, exp/libsli_b.so; exp/ is git-ignored) on one bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in a b a b; do
  cp exp/libsli_$v.so simplellminference_amd/libsli.so
  timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_us'])")"
done
