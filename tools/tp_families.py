"""Per-family launch times of one tensor-parallel shard on ONE GPU (SLI_DEBUG_NOCOMM: the last rank of TP N at its
real Llama-2-7B shard shapes, no communicator; values are not a model), beside each family's stream floor.
    python tools/tp_families.py [N ...]
TP_AR=oneshot|fused: the wo / down launches include the exchange, in loopback (SLI_DEBUG_OS_LOOPBACK, as in
tools/tp_rank_time.py). Prints one line per TP degree: step time, then per family us per launch (floor).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SLI_DEBUG_NOCOMM"] = "1"

from simplellminference_amd.model import LlamaModel, preset  # noqa: E402

# TP_PRESET / TP_BATCH / TP_CTX: another workload (default C2: llama2-7b, batch 1, ctx 2048)
PRESET = os.environ.get("TP_PRESET", "llama2-7b")
BATCH = int(os.environ.get("TP_BATCH", "1"))
CTX = int(os.environ.get("TP_CTX", "2048"))

for world in [int(a) for a in sys.argv[1:]] or [1, 8]:
    m = LlamaModel(config=preset(PRESET, max_length=CTX), w_dtype="f16", kv_dtype="f16", seed=1, tp_rank=world - 1,
                   tp_size=world, batch=BATCH).init()
    m.fill_kv_synthetic(7, CTX - 1)
    ar = os.environ.get("TP_AR")
    if ar and world > 1:
        os.environ["SLI_DEBUG_OS_LOOPBACK"] = "1"
        m.set_allreduce(ar)
    for b in range(BATCH):
        m.set_state_seq(b, 1234 + 17 * b, CTX - 1, advance=False)
    for _ in range(10):
        m.step()
    m.sync()
    step_ms = m.time_steps(50) / 1000.0
    fam = m.time_families(50)
    floor = m.time_stream(50)
    parts = []
    for k, v in fam.items():
        parts.append(f"{k} {v['avg_us']:.2f} ({floor[k]:.2f})")
    what = f"exchange {ar} (loopback)" if ar and world > 1 else "no exchange"
    tag = "" if (PRESET, BATCH, CTX) == ("llama2-7b", 1, 2048) else f"{PRESET} B{BATCH} ctx {CTX} "
    print(f"{tag}tp{world} rank {world - 1} {what}: step {step_ms:.3f} ms | " + " ".join(parts), flush=True)
    m.close()
