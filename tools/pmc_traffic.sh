#!/bin/bash
# GPU box: one rocprofv3 FETCH_SIZE pass over a short bench run, then the per-GEMV-launch traffic
# into profiles/<round>_gemv_traffic.json (read by bench.py as roofline.traffic).
#   tools/pmc_traffic.sh r02 [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r02}; shift
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 420 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gemv-iters 1 --greedy-steps 2 --prefill-tokens 0 "$@" > gpurun_out/pmc/bench.log 2>&1 || { echo PMC FAILED; tail -20 gpurun_out/pmc/bench.log; exit 1; }
csvf=$(find gpurun_out/pmc -name 'fetch_counter_collection.csv' | head -1)  # rocprofv3 may or may not add a subdirectory
[ -n "$csvf" ] || { echo "PMC: no counter csv"; exit 1; }
read alg dom < <(grep '^{' gpurun_out/pmc/bench.log | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read())['roofline']; print(r['algorithmic_bytes_per_launch'], r['kernel'].split(':')[0])")
python3 tools/pmc_traffic.py "$csvf" "$alg" "gpurun_out/pmc/${tag}_gemv_traffic.json" "${KEY:-llama2-7b/f16/tp1}" "$dom" gpurun_out/pmc/bench.log || exit 1
mv "$csvf" "gpurun_out/pmc/${tag}_${KEY//\//_}_fetch_counter_collection.csv"
rm -rf gpurun_out/pmc/*/ gpurun_out/pmc/fetch_*.csv  # the raw per-run files: the next pass must not find them
