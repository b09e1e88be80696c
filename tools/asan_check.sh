#!/bin/bash
# AddressSanitizer + UBSan over the CPU side, in this container (no GPU):
#   1. oracle/Makefile `asan`: the C oracle, the reference's CPU path (+ our harness) and the C++ drop-in layer's host
#      files, each built with -fsanitize=address,undefined;
#   2. tests/cpp/asan_host.cpp (the host layer on the CPU device: allocators, Buffer, Tensor, the flat-file reader;
#      leak detection on) and its stub mode (the CPU kernel stubs' LOG-exit, expected status 1);
#   3. the CPU suite's oracle and C-ABI tests with the sanitized oracle / reference builds preloaded into Python
#      (SLI_ORACLE_LIB / SLI_REF_LIB; leak detection off: CPython's own allocations are not ours).
# Usage: tools/asan_check.sh [log]   (default profiles/r6_asan.txt)
set -o pipefail
cd "$(dirname "$0")/.."
log=${1:-profiles/r6_asan.txt}
make -s -C oracle asan -j8 || exit 1
{
echo "# tools/asan_check.sh $(date -u +%Y-%m-%dT%H:%MZ), gcc $(gcc -dumpversion), -fsanitize=address,undefined -fno-sanitize-recover=undefined"
echo "## asan_host (detect_leaks=1)"
ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 oracle/_ref/asan/asan_host || { echo "asan_host FAILED"; exit 1; }
echo "## asan_host stub (expects the reference's LOG-exit, status 1, and no sanitizer report)"
ASAN_OPTIONS=detect_leaks=0 oracle/_ref/asan/asan_host stub > /tmp/asan_stub.out 2>&1
rc=$?
cat /tmp/asan_stub.out
if [ $rc -ne 1 ] || grep -q "Sanitizer" /tmp/asan_stub.out; then echo "stub FAILED (rc $rc)"; exit 1; fi
echo "## pytest tests/test_oracle.py tests/test_capi.py tests/test_comm_wait.py with the sanitized oracle / reference"
LD_PRELOAD="$(gcc -print-file-name=libasan.so)" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 \
    UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    SLI_ORACLE_LIB="$PWD/oracle/_ref/asan/liboracle.so" SLI_REF_LIB="$PWD/oracle/_ref/asan/libref.so" \
    timeout -k 10 1200 python3 -m pytest tests/test_oracle.py tests/test_capi.py tests/test_comm_wait.py -q -m "not gpu" \
    -p no:cacheprovider 2>&1 | grep -v "^$" | tail -15
rc=$?
echo "## the sanitized builds were the ones loaded:"
LD_PRELOAD="$(gcc -print-file-name=libasan.so)" ASAN_OPTIONS=detect_leaks=0 \
    SLI_ORACLE_LIB="$PWD/oracle/_ref/asan/liboracle.so" SLI_REF_LIB="$PWD/oracle/_ref/asan/libref.so" \
    python3 -c "import oracle, oracle.ref as r; oracle.lib(); r.lib(); print(*sorted({l.split()[-1] for l in open('/proc/self/maps') if '_ref/asan' in l or 'libasan' in l}), sep='\n')"
echo "## result: pytest exit $rc"
exit $rc
} 2>&1 | tee "$log"
