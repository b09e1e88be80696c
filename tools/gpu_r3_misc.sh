#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SLI_DEBUG_NOCOMM=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --prefill-tokens 0 > gpurun_out/bench_tp2_fused.log 2>&1 || { tail -20 gpurun_out/bench_tp2_fused.log; exit 1; }
grep '^{' gpurun_out/bench_tp2_fused.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tp2 nocomm', d['value'], d['tp_allreduce'], d['ms_per_step'])"
tools/ab_variants.sh "base attnnt" --greedy-steps 2 || exit 1
tools/ab_variants.sh "base attnnt" --greedy-steps 2 --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10
