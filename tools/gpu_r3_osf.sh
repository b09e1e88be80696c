#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tp.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/osf_tests.log 2>&1 || { tail -30 gpurun_out/osf_tests.log; exit 1; }
tail -1 gpurun_out/osf_tests.log
for v in base osf; do
  if [ $v = base ]; then unset SLI_LIB_VARIANT; else export SLI_LIB_VARIANT=$v; fi
  for ar in oneshot fused; do TP_AR=$ar timeout -k 10 300 python3 tools/tp_rank_time.py 8 2>&1 | sed "s/^/$v /" || exit 1; done
done
