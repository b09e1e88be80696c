#!/bin/bash
# round-5 check: MFMA attention lab, then the op / batch / model / qkv_attn tests, then short C1 / C4 benches
mkdir -p gpurun_out
timeout -k 10 120 ./tools/attn_mfma_lab > gpurun_out/aml2.txt 2>&1; echo lab rc=$?
grep -c MISMATCH gpurun_out/aml2.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_batch.py tests/test_gpu_model.py tests/test_gpu_qkv_attn.py -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/g2_tests.log 2>&1; echo tests rc=$?
tail -8 gpurun_out/g2_tests.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --prefill-tokens 0 > gpurun_out/g2_c1.json 2> gpurun_out/g2_c1.err; echo c1 rc=$?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --prefill-tokens 0 --preset llama3-8b --ctx 4096 --batch 8 > gpurun_out/g2_c4.json 2> gpurun_out/g2_c4.err; echo c4 rc=$?
python3 - <<'PY'
import json
for c in ("c1", "c4"):
    try:
        d = json.loads(open(f"gpurun_out/g2_{c}.json").read().strip().splitlines()[-1])
        f = d["roofline"]["families"]
        print(c, d["value"], {k: v["avg_launch_us"] for k, v in f.items()})
    except Exception as e:
        print(c, "no line", e)
PY
cat gpurun_out/aml2.txt
