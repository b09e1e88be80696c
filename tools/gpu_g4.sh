#!/bin/bash
# MFMA attention merge rework: lab, attention-touching GPU tests, C4 bench
mkdir -p gpurun_out
timeout -k 10 120 ./tools/attn_mfma_lab > gpurun_out/aml4.txt 2>&1; echo lab rc=$?
echo "lab mismatches: $(grep -c MISMATCH gpurun_out/aml4.txt)"
grep -q MISMATCH gpurun_out/aml4.txt && { cat gpurun_out/aml4.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_batch.py tests/test_gpu_model.py -q --timeout 300 --timeout-method thread -m gpu -x > gpurun_out/g4_tests.log 2>&1; echo tests rc=$?
tail -4 gpurun_out/g4_tests.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --prefill-tokens 0 --preset llama3-8b --ctx 4096 --batch 8 > gpurun_out/g4_c4.json 2> gpurun_out/g4_c4.err; echo c4 rc=$?
python3 -c "
import json
d = json.loads(open('gpurun_out/g4_c4.json').read().strip().splitlines()[-1])
print('c4', d['value'], {k: v['avg_launch_us'] for k, v in d['roofline']['families'].items()})"
grep -E "^C4 |C4-pos.*4095|B1-8B|C4-tp8|C2-tp8|G8|C4-rag" gpurun_out/aml4.txt
