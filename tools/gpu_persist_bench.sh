#!/bin/bash
# bench.py's N>1 persistent-layer selection rehearsed on ONE GPU: 2 rank processes, no RCCL communicator
# (SLI_DEBUG_NOCOMM), each grid capped to 64 workgroups, the persist step held to the fused_wg launch graph.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r6_persist_bench}
SLI_DEBUG_NOCOMM=1 SLI_DEBUG_GEMV_MAX_BLOCKS=64 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 \
  --preset small-h128 --ctx 1024 --tp-allreduce fused_wg > gpurun_out/${tag}.json 2> gpurun_out/${tag}.log
rc=$?
tail -5 gpurun_out/${tag}.log
cat gpurun_out/${tag}.json
exit $rc
