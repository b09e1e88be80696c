#!/bin/bash
# A/B/... variant builds (python -m simplellminference_amd.build --variant <v> -D ...: libsli_<v>.so beside
# libsli.so; "base" = libsli.so itself) on one bench line each, interleaved over two rounds in one call.
#   tools/ab_variants.sh "base v1 v2" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
vs=$1; shift
for rep in 1 2; do
  for v in $vs; do
    if [ "$v" = base ]; then unset SLI_LIB_VARIANT; else export SLI_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --prefill-tokens 0 "$@" > gpurun_out/ab_$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/ab_$v.log; exit 1; }
    echo "$v $(grep '^{' gpurun_out/ab_$v.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['families'].items()})")"
  done
done
