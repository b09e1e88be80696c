#!/bin/bash
# SQ counters of the prefill GEMM (tools/pgemm_lab LAB_QUICK: the engine's fp16 tilings at M = 256), one pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$PWD
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$root"
export LAB_QUICK=1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc -o pg_sq --output-format csv -- ./tools/pgemm_lab 256 > gpurun_out/pmc/pg_sq_run.log 2>&1
rc=$?
tail -3 gpurun_out/pmc/pg_sq_run.log
ls gpurun_out/pmc
exit $rc
