#!/bin/bash
# Local helper (this container, not the GPU box): run one gpurun call, re-submitting it only when gpurun
# reports an INFRASTRUCTURE transient (box lost while being prepared, back-off, no box free) — never
# when the command itself ran and failed.   tools/gpurun_retry.sh <out-file> <timeout-s> '<command>'
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|no box\|rc=3" "$out" && ! grep -q "status=ok" "$out"; then
    sleep 45
    continue
  fi
  exit $rc
done
exit $rc
