#!/bin/bash
# GPU box: decode throughput sweeps on one GPU — Llama-2-7B fp16 batch 1 over the context length, and
# Llama-3-8B fp16 ctx 4096 over the batch — one bench line each, summarised to gpurun_out/sweep.txt.
#   tools/sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sweep.txt
: > $out
run() {
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --prefill-tokens 0 --steps 40 --warmup 8 "$@" > gpurun_out/sweep_run.log 2>&1 || { echo "FAILED: $*"; tail -5 gpurun_out/sweep_run.log; exit 1; }
  grep '^{' gpurun_out/sweep_run.log | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); r = d['roofline']; c = d['config']
fam = ' '.join(f\"{k}={v['avg_launch_us']:.1f}\" for k, v in r['families'].items())
print(f\"{c['workload']:60s} {d['value']:9.1f} tok/s  {d['ms_per_step']:7.3f} ms  step/HBM {c['step_frac_of_hbm_peak']:.3f}  | {fam}\")" | tee -a $out
}
for ctx in 128 512 1024 2048 4096; do run --ctx $ctx; done
for b in 1 2 4 8; do run --preset llama3-8b --ctx 4096 --batch $b; done
run --w-dtype i8 --ctx 4096
echo sweep done
