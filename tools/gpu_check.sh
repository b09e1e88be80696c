set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r01 --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof/bench.log 2>&1 || { echo PROF FAILED; exit 1; }
echo done
