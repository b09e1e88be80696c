#!/usr/bin/env python3
"""Decode-throughput benchmark (BASELINE.json metric): Llama-2-7B fp16, batch 1, ctx 2048, TP = N.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python bench.py --preset llama3-8b --ctx 4096 --batch 8      # BASELINE configs[4] (C4) at TP = N
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step is one full decode step of the 32-layer model at position 2047 (KV rows 0..2046 resident in
HBM), replayed from its captured hipGraph; the step is idempotent (it rewrites the same K/V row), so
K steps time K tokens of a ctx-2048 decode. Weights are seeded synthetic fp16 of the Llama-2-7B
architecture (no checkpoints are reachable); every input is resident in HBM before timing starts.
Under TP each rank holds 1/N of the heads / FFN columns / vocab and the step all-reduces twice per
layer over RCCL; value = tokens/s of the whole job (1 token per step across all ranks).

Rank 0 prints one JSON line. `roofline` prices the dominant kernel family (the weight-streaming GEMVs,
92.5 % of the step's bytes): algorithmic bytes per launch / mean launch time measured with HIP events
on the engine's stream. `cpu_baseline` times the C oracle (single-threaded restatement of the
reference CPU path) on a bounded sample and projects the full model's tokens/s.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decode tokens/sec, Llama-7B fp16 seq=1 ctx=2048, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CTX = 2048


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--w-dtype", default="f16", choices=["f16", "i8", "f32"])
    ap.add_argument("--preset", default="llama2-7b")
    ap.add_argument("--ctx", type=int, default=CTX)
    ap.add_argument("--batch", type=int, default=1, help="sequences decoding in lockstep (MFMA projections if > 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample budget")
    ap.add_argument("--gemv-iters", type=int, default=20)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r04_gemv_traffic.json"))
    return ap.parse_args()


def cpu_baseline(budget_s: float, preset_name: str = "llama2-7b", ctx: int = CTX) -> dict:
    """Oracle (port of the reference CPU path, 1 thread, one sequence at a time): a 2-layer model of the
    workload's shape with its full tied LM head at position ctx-1; full-model time = embed + L * layer + head."""
    import oracle as O
    from simplellminference_amd.model import preset
    pc = preset(preset_name, max_length=ctx)
    cfg = O.Config(pc.vocab_size, pc.hidden_size, pc.num_attention_heads, pc.num_key_value_heads, pc.head_dim,
                   pc.intermediate_size, 2, ctx, pc.rms_norm_eps, pc.rope_theta)
    n_layers = pc.num_hidden_layers
    m = O.Model(cfg, seed=1, wmode=O.W_F32)
    m.fill_kv_synthetic(7, ctx - 1)
    t_lay, t_head, t_emb = [], [], []
    t0 = time.perf_counter()
    while True:
        m.forward(1234, ctx - 1)
        e, l, h = m.last_timing()
        t_emb.append(e)
        t_lay.append(l / cfg.n_layers)
        t_head.append(h)
        if time.perf_counter() - t0 >= budget_s or len(t_lay) >= 50:
            break
    m.close()
    layer, head, emb = statistics.median(t_lay), statistics.median(t_head), statistics.median(t_emb)
    step = emb + n_layers * layer + head
    return {"value": 1.0 / step, "unit": "tokens/s", "cores": 1, "kind": "port",
            "sample": (f"C oracle (oracle/sli_oracle.c, fp32, 1 thread, one sequence per step as the reference) on "
                       f"{len(t_lay)} decode steps of a 2-layer {preset_name}-shape model (+{pc.vocab_size}x"
                       f"{pc.hidden_size} tied head) at pos {ctx - 1}; median layer {layer * 1e3:.1f} ms, head "
                       f"{head * 1e3:.1f} ms; full {n_layers}-layer step projected {step:.2f} s")}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    dist_on = world > 1
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)

    from simplellminference_amd.model import LlamaModel, comm_id, preset

    cid = None
    if dist_on:
        box = [comm_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        cid = box[0]
    cfg = preset(a.preset, max_length=a.ctx)
    B = a.batch
    model = LlamaModel(config=cfg, w_dtype=a.w_dtype, kv_dtype="f16", tp_rank=rank, tp_size=world, comm_id=cid,
                       device=local, seed=1, batch=B).init()
    model.fill_kv_synthetic(7, a.ctx - 1)
    for b in range(B):  # every sequence at position ctx-1 (KV rows 0..ctx-2 resident), its own token
        model.set_state_seq(b, 1234 + 17 * b, a.ctx - 1, advance=False)

    def barrier():
        model.sync()
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()

    for _ in range(a.warmup):
        model.step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        model.step()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    st = model.state()
    if st["error"]:
        raise SystemExit(f"device error flag {st['error']}")
    wbytes, kvbytes = model.step_bytes()
    g = model.time_gemv(a.gemv_iters)
    achieved = g["bytes_per_launch"] / (g["avg_us"] * 1e-6) / 1e9

    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            key = f"{a.preset}/{a.w_dtype}/tp{world}" + (f"/b{B}" if B > 1 else "")
            if key in tj:
                traffic = tj[key]["hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            traffic = None

    ms = 1e3 * elapsed / a.steps
    value = B * a.steps / elapsed  # tokens/s of the whole job (B tokens per step, all ranks on the same tokens)
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": a.w_dtype if a.w_dtype != "f16" else "fp16",
        "data": "synthetic",
        "config": {"workload": f"{a.preset} decode step, batch {B}, ctx {a.ctx}, tensor parallel {world}",
                   "global_batch": B, "seq_len": a.ctx, "parallelism": f"tp{world}", "weights": a.w_dtype,
                   "kv_cache": "fp16", "accumulate": "fp32",
                   "step_bytes_per_gpu": round(wbytes + kvbytes), "hbm_roofline_tokens_per_s":
                       round(HBM_PEAK_GBS * 1e9 / (wbytes + kvbytes), 1),
                   "step_frac_of_hbm_peak": round((wbytes + kvbytes) / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)},
        "roofline": {"bound": "hbm", "kernel": ("gemv_kernel (qkv/wo/gate-up/down/lm-head weight streaming)" if B == 1
                                                else "bgemm_kernel (MFMA 16x16x32 f16, qkv/wo/gate-up/down/lm-head)"),
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "avg_launch_us": round(g["avg_us"], 3), "algorithmic_bytes_per_launch": round(g["bytes_per_launch"]),
                     "launches_per_step": g["launches_per_step"]},
    }
    if B > 1:  # MFMA work of the dominant kernel family: 2 flop per weight per sequence
        tflops = 2.0 * B * (g["bytes_per_launch"] / 2.0) / (g["avg_us"] * 1e-6) / 1e12
        out["roofline"]["mfma"] = {"achieved_tflops": round(tflops, 2), "peak_tflops": 2500.0,
                                   "frac": round(tflops / 2500.0, 5)}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.cpu_seconds, a.preset, a.ctx)
    model.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
