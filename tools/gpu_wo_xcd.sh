#!/bin/bash
# K-split wo with its K blocks XCD-aligned (gemv.h GemvIn::kx): the wo / model parity tests, then an interleaved
# A/B against the dispatch-order variant (libsli_noxcd.so) at C3 and C1.   tools/gpu_wo_xcd.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6b}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wo_ksplit.py tests/test_gpu_model.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_wo_xcd_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${tag}_wo_xcd_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_wo_xcd_tests.log
echo "## C3" ; tools/ab_variants.sh "base noxcd" --w-dtype i8 || exit 1
echo "## C1" ; tools/ab_variants.sh "base noxcd" || exit 1
