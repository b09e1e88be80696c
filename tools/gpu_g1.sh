mkdir -p gpurun_out
timeout -k 10 120 ./tools/attn_mfma_lab > gpurun_out/aml1.txt 2>&1; echo lab rc=$?
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_batch.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/g1_tests.log 2>&1; echo tests rc=$?
tail -5 gpurun_out/g1_tests.log
cat gpurun_out/aml1.txt
