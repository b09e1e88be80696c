set -o pipefail
cd $GRAFT_REPO_ROOT
SLI_PF_KB=2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
tools/ab_env.sh 2 "SLI_PF_KB=0" "SLI_PF_KB=1" "SLI_PF_KB=2" "SLI_PF_KB=4" "SLI_PF_KB=2 SLI_PF_SKIP=4" "SLI_PF_KB=8 SLI_PF_SKIP=4"
