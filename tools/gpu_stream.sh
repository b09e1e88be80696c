#!/bin/bash
# GPU box: the stream-engine parity tests, then (only if no test crashed) a short stream-mode bench.
# Usage (from the repo root): bash tools/gpu_stream.sh [pytest -k expr] [bench args...]
set -u
mkdir -p gpurun_out
K=${1:-}
shift || true
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_gpu_stream.py "${KARG[@]}" \
    > gpurun_out/stream_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
grep -E "passed|failed|PASSED|FAILED|ERROR|Error" gpurun_out/stream_tests.log | tail -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests did not finish cleanly: stop"; exit $rc; fi
timeout -k 10 400 python -u bench.py --exec stream --prefill-tokens 0 --no-cpu-baseline --greedy-steps 8 "$@" \
    > gpurun_out/bench_stream.json 2> gpurun_out/bench_stream.err
brc=$?
echo "bench rc=$brc"
tail -3 gpurun_out/bench_stream.err
python - <<'PY'
import json
try:
    d = json.loads(open("gpurun_out/bench_stream.json").read().strip().splitlines()[-1])
    print("value", d["value"], "ms", d["ms_per_step"], "greedy", d["greedy_64"])
    print("roofline", {k: d["roofline"][k] for k in ("kernel", "achieved", "frac", "avg_launch_us")})
except Exception as e:
    print("no bench line:", e)
PY
exit $brc
