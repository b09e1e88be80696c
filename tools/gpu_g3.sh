#!/bin/bash
# round-5 check: MFMA attention lab (correctness + timing), the whole GPU suite, C1 / C3 / C4 benches
mkdir -p gpurun_out
timeout -k 10 120 ./tools/attn_mfma_lab > gpurun_out/aml3.txt 2>&1; echo lab rc=$?
echo "lab mismatches: $(grep -c MISMATCH gpurun_out/aml3.txt)"
grep -q MISMATCH gpurun_out/aml3.txt && { cat gpurun_out/aml3.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests/ -q --timeout 300 --timeout-method thread -m gpu -x > gpurun_out/g3_tests.log 2>&1; echo tests rc=$?
tail -8 gpurun_out/g3_tests.log
for c in "c1:" "c3:--w-dtype i8" "c4:--preset llama3-8b --ctx 4096 --batch 8"; do
  n=${c%%:*}; args=${c#*:}
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --prefill-tokens 0 $args > gpurun_out/g3_$n.json 2> gpurun_out/g3_$n.err; echo $n rc=$?
done
python3 - <<'PY'
import json
for c in ("c1", "c3", "c4"):
    try:
        d = json.loads(open(f"gpurun_out/g3_{c}.json").read().strip().splitlines()[-1])
        f = d["roofline"]["families"]
        print(c, d["value"], {k: v["avg_launch_us"] for k, v in f.items()})
    except Exception as e:
        print(c, "no line", e)
PY
cat gpurun_out/aml3.txt
