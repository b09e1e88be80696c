#!/bin/bash
# per-rank TP step on one GPU (Llama-2-7B fp16 ctx 2048, last rank): no exchange, then the one-shot and fused
# exchanges (launch-level and per workgroup) in loopback (tools/tp_rank_time.py) -> gpurun_out/<tag>_tp_rank_time_loopback.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r4}
mkdir -p gpurun_out
out=gpurun_out/${tag}_tp_rank_time_loopback.txt
timeout -k 10 300 python3 tools/tp_rank_time.py 1 2 4 8 > $out 2>&1 || { tail -20 $out; exit 1; }
TP_AR=oneshot timeout -k 10 300 python3 tools/tp_rank_time.py 2 4 8 >> $out 2>&1 || { tail -20 $out; exit 1; }
TP_AR=fused timeout -k 10 300 python3 tools/tp_rank_time.py 2 4 8 >> $out 2>&1 || { tail -20 $out; exit 1; }
TP_AR=fused_wg timeout -k 10 300 python3 tools/tp_rank_time.py 2 4 8 >> $out 2>&1 || { tail -20 $out; exit 1; }
cat $out
