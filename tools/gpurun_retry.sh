#!/bin/bash
# Local helper (this container, not the GPU box): run one gpurun call, re-submitting it only when gpurun
# reports an INFRASTRUCTURE transient (box lost while being prepared, back-off, no box free) — never
# when the command itself ran and failed.   tools/gpurun_retry.sh <out-file> <timeout-s> '<command>'
out=$1; to=$2; cmd=$3
for i in $(seq 1 16); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" "$out" && ! grep -q "status=ok" "$out"; }; then
    wait_s=$(grep -o "retry in [0-9]*s" "$out" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${wait_s:-60} > 600 ? 600 : ${wait_s:-60} + 5 ))
    continue
  fi
  exit $rc
done
exit $rc
