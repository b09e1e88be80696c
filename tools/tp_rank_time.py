"""Per-rank decode-step time of one tensor-parallel shard on ONE GPU, without a communicator
(SLI_DEBUG_NOCOMM: the rank's kernels at their real shapes, no RCCL all-reduces; values are not a model).
Estimates the compute part of config C2 (Llama-2-7B at TP N); the collectives come on top.
    python tools/tp_rank_time.py [N ...]
TP_AR=oneshot|fused|fused_wg: the rank's all-reduces included, in loopback (SLI_DEBUG_OS_LOOPBACK: the exchange
kernels run against the rank's own comm buffer, every flag raised locally — everything but the xGMI hop).
TP_EXEC=persist: the layer stack as one persistent launch (csrc/tp_layers.h; with TP_AR=fused_wg its in-launch
granule exchange in loopback).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SLI_DEBUG_NOCOMM"] = "1"

from simplellminference_amd.model import LlamaModel, preset  # noqa: E402

# TP_PRESET / TP_BATCH / TP_CTX: another workload (default C2: llama2-7b, batch 1, ctx 2048)
PRESET = os.environ.get("TP_PRESET", "llama2-7b")
BATCH = int(os.environ.get("TP_BATCH", "1"))
CTX = int(os.environ.get("TP_CTX", "2048"))

for world in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]:
    m = LlamaModel(config=preset(PRESET, max_length=CTX), w_dtype="f16", kv_dtype="f16", seed=1, tp_rank=world - 1,
                   tp_size=world, batch=BATCH).init()
    m.fill_kv_synthetic(7, CTX - 1)
    ar = os.environ.get("TP_AR")
    if ar and world > 1:
        os.environ["SLI_DEBUG_OS_LOOPBACK"] = "1"
        m.set_allreduce(ar)
    if os.environ.get("TP_EXEC"):
        m.set_exec(os.environ["TP_EXEC"])
    for b in range(BATCH):
        m.set_state_seq(b, 1234 + 17 * b, CTX - 1, advance=False)
    for _ in range(10):
        m.step()
    m.sync()
    t0 = time.perf_counter()
    n = 50
    for _ in range(n):
        m.step()
    m.sync()
    ms = 1e3 * (time.perf_counter() - t0) / n
    what = f"all-reduces {ar} (loopback)" if ar and world > 1 else "no all-reduces"
    tag = "" if (PRESET, BATCH, CTX) == ("llama2-7b", 1, 2048) else f"{PRESET} B{BATCH} ctx {CTX} "
    qa = {0: "", 1: " qkv+attn fused", 2: " qkv+attn+wo fused"}[m.fused_qkv_attn()]
    print(f"{tag}tp{world} rank {world - 1} [{m.exec_mode()}{qa}]: {ms:.3f} ms/step compute ({what}); device error "
          f"{m.state()['error']}", flush=True)
    m.close()
