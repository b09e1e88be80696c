#!/bin/bash
# A/B/... prebuilt libsli.so variants (exp/libsli_<v>.so; exp/ is git-ignored) on one bench line each,
# interleaved twice.   tools/ab3.sh "a b c" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
vs=$1; shift
cp simplellminference_amd/libsli.so exp/libsli_orig.so
for rep in 1 2; do
  for v in $vs; do
    cp exp/libsli_$v.so simplellminference_amd/libsli.so
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --prefill-tokens 0 "$@" > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; cp exp/libsli_orig.so simplellminference_amd/libsli.so; exit 1; }
    echo "$v $(grep '^{' gpurun_out/ab.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['families'].items()})")"
  done
done
cp exp/libsli_orig.so simplellminference_amd/libsli.so
