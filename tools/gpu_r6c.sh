#!/bin/bash
# Round 6 (second session) final tree: the GPU suite, smoke, then the driver's default bench command, C3 and C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6c}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench_c1.log 2>&1 || { echo BENCH C1 FAILED; tail -20 gpurun_out/${tag}_bench_c1.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['value'], d['step_ms']['p50'], d['roofline']['frac'], d['prefill']['tokens_per_s'])"
timeout -k 10 300 python3 bench.py --w-dtype i8 --no-cpu-baseline > gpurun_out/${tag}_bench_c3.log 2>&1 || { echo BENCH C3 FAILED; tail -20 gpurun_out/${tag}_bench_c3.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['step_ms']['p50'], d['prefill']['tokens_per_s'])"
timeout -k 10 400 python3 bench.py --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 > gpurun_out/${tag}_bench_c4.log 2>&1 || { echo BENCH C4 FAILED; tail -20 gpurun_out/${tag}_bench_c4.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['step_ms']['p50'])"
echo done
