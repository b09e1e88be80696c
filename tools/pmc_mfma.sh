#!/bin/bash
# GPU box: one rocprofv3 MFMA counter pass over a short bench run (C4 batch-8 by default; the prefill leg
# runs too when the bench args leave it on), summarised per bgemm family into
# gpurun_out/pmc/<tag>_mfma.json.   tools/pmc_mfma.sh <tag> <key> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r2}; key=${2:-llama3-8b/f16/tp1/b8}; shift 2
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 420 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_F16 GRBM_GUI_ACTIVE -d gpurun_out/pmc -o mfma --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gemv-iters 1 --greedy-steps 2 "$@" > gpurun_out/pmc/mfma_bench.log 2>&1 || { echo PMC MFMA FAILED; tail -20 gpurun_out/pmc/mfma_bench.log; exit 1; }
csvf=$(find gpurun_out/pmc -name 'mfma_counter_collection.csv' | head -1)
[ -n "$csvf" ] || { echo "PMC: no counter csv"; exit 1; }
python3 tools/pmc_mfma.py "$csvf" "gpurun_out/pmc/${tag}_mfma.json" "$key" || exit 1
mv "$csvf" "gpurun_out/pmc/${tag}_${key//\//_}_mfma_counter_collection.csv"
rm -rf gpurun_out/pmc/*/ gpurun_out/pmc/mfma_*.csv
