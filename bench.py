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

Rank 0 prints one JSON line. `roofline` prices the DOMINANT kernel (the family with the largest share
of the step's device time, e.g. the fused RMSNorm + gate/up GEMV + SwiGLU at C1): its algorithmic bytes
per launch / its mean launch time, measured live with HIP events on the engine's own stream
(sli_model_time_families); `roofline.families` lists every family the same way, and `roofline.traffic`
is that kernel's HBM bytes per launch from the committed rocprofv3 FETCH_SIZE pass (x2 gfx950
correction). `greedy_64` is a true 64-token greedy decode (positions ctx-64 .. ctx-1, the state advancing
on the device) beside the idempotent-step timing. `cpu_baseline` times the reference's own CPU path
(oracle/_ref/libref.so, compiled from the reference sources in the build container) pinned to one host
core on a bounded 2-layer sample and projects the full model's tokens/s; beside it the oracle port on one
core and on all cores (labelled not reference).
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
FAMILY_KERNELS = {
    False: {"qkv": "gemv_kernel<EpiQKV> (RMSNorm + [wq;wk;wv] GEMV + RoPE + K/V write)",
            "attention": "attn_partial_kernel (split-context flash decode + last-arriver merge)",
            "wo": "gemv_merge_kernel<EpiKPart> (attention split merge while staging + K-split wo GEMV -> 2 partial "
                  "rows; past 8 splits per head: the attention merges and wo is gemv_kernel<EpiStore>)",
            "gate_up": "gemv_sum_kernel<EpiSwiGLU> (residual + wo partials staged, RMSNorm + [gate;up] GEMV + "
                       "sigmoid(g)*u)",
            "down": "gemv_kernel<EpiStoreSum> (down GEMV + residual + wo partials -> x)",
            "lm_head": "gemv_kernel<EpiLogits> (RMSNorm + tied LM head + argmax keys)"},
    True: {"qkv": "bgemm_kernel<BgEpiQKV> (MFMA 16x16x32 f16)", "attention": "attn_mfma_kernel (fp16 cache: LDS-DMA K/V, MFMA 16x16x32 f16, in-launch "
                                                                    "split merge)",
           "wo": "bgemm_kernel<BgEpiStore> (MFMA)", "gate_up": "bgemm_kernel<BgEpiSwiGLU> (MFMA)",
           "down": "bgemm_kernel<BgEpiStore> (MFMA)", "lm_head": "bgemm_kernel<BgEpiLogits> (MFMA)"},
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--w-dtype", default="f16", choices=["f16", "i8", "f32"])
    ap.add_argument("--preset", default="llama2-7b")
    ap.add_argument("--ctx", type=int, default=CTX)
    ap.add_argument("--batch", type=int, default=1, help="sequences decoding in lockstep (MFMA projections if > 1)")
    ap.add_argument("--tp-exec", default="auto", choices=["auto", "launches", "persist"],
                    help="N>1: the layer stack as one persistent launch per rank where it fits and validates (auto), "
                         "or the launch graph")
    ap.add_argument("--tp-allreduce", default="auto", choices=["auto", "rccl", "oneshot", "fused", "fused_wg"],
                    help="TP all-reduce: auto = the one-shot exchange fused into the wo / down launches per "
                         "workgroup when every rank has its own GPU (else batch 1: one summing workgroup per launch, "
                         "batch > 1: the sliced one-shot launch) if a validation step against RCCL agrees on every "
                         "rank, else RCCL")
    ap.add_argument("--prefill-tokens", type=int, default=512,
                    help="after the decode timing: prefill a prompt of this many tokens (0: skip; batch 1 only)")
    ap.add_argument("--prefill-reps", type=int, default=3, help="timed prefill repetitions (after one warm-up)")
    ap.add_argument("--settle-ms", type=float, default=1000.0,
                    help="untimed warm-up before the --warmup steps: replay the step for this much wall time "
                         "(0: one step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--greedy-steps", type=int, default=64, help="the greedy sanity run's length (profiling passes: 2)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample budget")
    ap.add_argument("--gemv-iters", type=int, default=20)
    ap.add_argument("--traffic-json", default=next(
        (p for p in (os.path.join(ROOT, "profiles", f) for f in ("r6_gemv_traffic.json", "r5_gemv_traffic.json", "r4_gemv_traffic.json",
                                                                   "r3_gemv_traffic.json"))
         if os.path.exists(p)), os.path.join(ROOT, "profiles", "r5_gemv_traffic.json")))
    return ap.parse_args()


def _time_steps(fwd, timing, n_layers, budget_s, min_steps=3, max_steps=50):
    """Median embed / per-layer / head seconds of repeated forwards (at least min_steps, then until the budget)."""
    t_emb, t_lay, t_head = [], [], []
    t0 = time.perf_counter()
    while len(t_lay) < max_steps:
        fwd()
        e, l, h = timing()
        t_emb.append(e)
        t_lay.append(l)
        t_head.append(h)
        if len(t_lay) >= min_steps and time.perf_counter() - t0 >= budget_s:
            break
    return statistics.median(t_emb), statistics.median(t_lay) / n_layers, statistics.median(t_head), len(t_lay)


def cpu_baseline(budget_s: float, preset_name: str = "llama2-7b", ctx: int = CTX) -> dict:
    """The host-CPU baseline, timed on this box's cores in this run.

    `value`: the REFERENCE's own CPU path — oracle/_ref/libref.so, its source/kernel/cpu + source/op compiled in
    place from the reference sources in the build container (oracle/Makefile `ref`), the ops wired as
    model.cpp:40-140 (oracle/ref_harness.cpp) — on 1 pinned core, one sequence per step as the reference; a
    2-layer model of the workload's shape with its full tied LM head at position ctx-1 (KV rows 0..ctx-2 filled),
    the full model's step projected as embed + L x layer + head. If libref.so is absent: the oracle port instead
    (kind "port"). Beside it, on the same sample: the port on 1 core (the measured port / reference ratio, no
    factor applied anywhere) and the port with GEMV rows over all cores of this process ("all_cores", labelled
    not reference)."""
    import oracle as O
    from oracle import ref as R
    from simplellminference_amd.model import preset
    pc = preset(preset_name, max_length=ctx)
    cfg = O.Config(pc.vocab_size, pc.hidden_size, pc.num_attention_heads, pc.num_key_value_heads, pc.head_dim,
                   pc.intermediate_size, 2, ctx, pc.rms_norm_eps, pc.rope_theta)
    n_layers = pc.num_hidden_layers
    prev = os.sched_getaffinity(0)
    core = max(prev)
    n_all = max(1, min(len(prev), int(os.environ.get("OMP_NUM_THREADS", len(prev))), 32))
    m = O.Model(cfg, seed=1, wmode=O.W_F32)
    m.fill_kv_synthetic(7, ctx - 1)

    def run(label, fwd, timing, budget):
        e, lay, h, n = _time_steps(fwd, timing, cfg.n_layers, budget)
        step = e + n_layers * lay + h
        return {"tokens_per_s": 1.0 / step, "step_s": step, "sample_step_s": e + cfg.n_layers * lay + h,
                "layer_ms": lay * 1e3, "head_ms": h * 1e3, "steps": n, "label": label}

    os.sched_setaffinity(0, {core})  # the reference CPU path is single-threaded: one pinned core, in-process
    try:
        ref = None
        if os.path.exists(R.LIB_PATH):
            rm = R.Model(cfg, flat=m.flat_image())
            k, v = rm.kv_cache()
            ok, ov = m.kv_cache()
            k[:] = ok
            v[:] = ov
            ref = run("reference", lambda: rm.forward(1234, ctx - 1), rm.last_timing, 0.55 * budget_s)
            rm.close()
        port = run("port", lambda: m.forward(1234, ctx - 1), m.last_timing, (0.2 if ref else 0.75) * budget_s)
    finally:
        os.sched_setaffinity(0, prev)
    m.set_threads(n_all)
    allc = run("all cores", lambda: m.forward(1234, ctx - 1), m.last_timing, 0.2 * budget_s)
    m.close()
    prim = ref or port
    shape = (f"2-layer {preset_name}-shape model (+{pc.vocab_size}x{pc.hidden_size} tied head), fp32, at pos "
             f"{ctx - 1} (KV rows 0..{ctx - 2} filled), one sequence per step; full {n_layers}-layer step "
             f"projected = embed + {n_layers} x layer + head")
    who = ("the reference CPU path (oracle/_ref/libref.so: source/kernel/cpu + source/op compiled from the reference "
           "sources, the model.cpp op wiring)" if ref else "the C oracle port (oracle/sli_oracle.c)")
    out = {"value": prim["tokens_per_s"], "unit": "tokens/s", "cores": 1, "core_id": core,
           "kind": "reference" if ref else "port",
           "sample": (f"{who}, 1 thread pinned to core {core}, {prim['steps']} steps of a {shape}: median "
                      f"{prim['sample_step_s']:.3f} s per sample step (layer {prim['layer_ms']:.1f} ms, head "
                      f"{prim['head_ms']:.1f} ms), full step {prim['step_s']:.2f} s"),
           "port_1core": {"value": port["tokens_per_s"], "step_s": round(port["step_s"], 3),
                          "layer_ms": round(port["layer_ms"], 2), "head_ms": round(port["head_ms"], 2)},
           "all_cores": {"value": allc["tokens_per_s"], "unit": "tokens/s", "cores": n_all, "kind": "port",
                         "label": "NOT the reference (single-threaded): the oracle port with GEMV rows split over "
                                  f"{n_all} host threads, bit-identical results", "step_s": round(allc["step_s"], 3)}}
    if ref:
        out["port_over_reference_step_time"] = round(port["step_s"] / ref["step_s"], 3)
    return out


def _oneshot_opened(model, dist, torch, mode) -> bool:
    """Map every rank's one-shot all-reduce buffer (IPC over the gloo group); True only if it worked on
    EVERY rank (a rank that failed still joins the collective vote, so no rank waits on a peer that is not
    there). Forced --tp-allreduce oneshot re-raises the failure."""
    from simplellminference_amd import tp
    err = None
    try:
        tp.open_oneshot(model)
    except Exception as e:  # noqa: BLE001 - reported, voted on, then RCCL carries the step
        err = e
        progress(f"one-shot buffers unavailable on this rank: {e}")
    flag = torch.tensor([0 if err else 1], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if flag.item() == 0 and mode in ("oneshot", "fused", "fused_wg"):  # forced one-shot: EVERY rank stops (none waits on RCCL alone)
        raise SystemExit(f"one-shot buffers could not be mapped on every rank ({err or 'another rank failed'})")
    return flag.item() == 1


def _own_gpus(dist, torch, local: int, world: int) -> bool:
    """True when every rank drives a DIFFERENT GPU (its PCI domain / bus / device id and uuid all-gathered over
    gloo): only then may the step use the modes whose kernels spin-wait on their own grid or on the peers (the fused
    q/k/v + attention launch, the per-workgroup exchange). Ranks that share a device, or a torch without the PCI
    fields, get the modes that never wait across launches."""
    p = torch.cuda.get_device_properties(local)
    key = ":".join(str(getattr(p, f, "?")) for f in ("pci_domain_id", "pci_bus_id", "pci_device_id", "uuid"))
    keys = [None] * world
    dist.all_gather_object(keys, key)
    return "?" not in key and len(set(keys)) == world


def _try_persist(model, dist, torch, ref, forced: bool, B: int) -> str:
    """The layer stack as one persistent launch per rank (csrc/tp_layers.h, exec "persist"), its residual exchange the
    per-workgroup granule exchange over the mapped peer buffers: taken only if it fits EVERY rank's shard (a rank that
    refuses still votes) and its step agrees with the RCCL reference step on every rank; else the launch graph stays.
    A wait inside the launch is bounded (DevState error kTlErrWait), so a peer that never arrives fails the check."""
    import numpy as np
    from simplellminference_amd import SliError
    fits = 1
    try:
        model.set_exec("persist")
    except SliError as e:
        fits = 0
        progress(f"persistent layers do not fit this rank's shard: {e}")
    flag = torch.tensor([fits], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    all_fit = flag.item() == 1
    if all_fit:
        model.step()
        got = model.logits()[0]
        ok = bool(model.state()["error"] == 0 and np.isfinite(got).all() and np.abs(got - ref).max() <= 1e-3)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if flag.item() == 1:
            return "persist (one launch per rank for the layer stack; validated against rccl on every rank)"
    if forced:
        raise SystemExit("--tp-exec persist: the persistent layer stack does not fit or disagrees with RCCL")
    model.set_exec("launches")
    for b in range(B):  # clears a timed-out wait's device error flag
        model.set_state_seq(b, (1234 + 17 * b) % model.config.vocab_size, model.config.max_length - 1, advance=False)
    return "launches (persistent layers " + ("failed validation)" if all_fit else "do not fit every rank)")


class StepMarks:
    """HIP events recorded on the engine stream between the timed loop's graph replays. Recording is an
    enqueue (no host wait), so the timed loop keeps its host cadence; the durations are read after the
    closing barrier."""

    def __init__(self, torch, model, device, n):
        self.stream = torch.cuda.ExternalStream(model.stream(), device=device)
        self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]

    def start(self):
        self.ev[0].record(self.stream)

    def mark(self, i):
        self.ev[i + 1].record(self.stream)

    def durations_ms(self):
        return [a.elapsed_time(b) for a, b in zip(self.ev[:-1], self.ev[1:])]


def step_stats(ms: list, mean_ms: float) -> dict:
    """p50 / p99 / min / max and the first-5 / last-5 means of the per-step device durations (HIP events),
    beside the host-clock mean of the same window."""
    import numpy as np
    v = np.asarray(ms, np.float64)
    k = min(5, len(v))
    p50 = float(np.percentile(v, 50))
    return {"source": "HIP events between consecutive graph replays on the engine stream (timed window)",
            "n": int(len(v)), "p50": round(p50, 4), "p99": round(float(np.percentile(v, 99)), 4),
            "min": round(float(v.min()), 4), "max": round(float(v.max()), 4), "mean": round(float(v.mean()), 4),
            "first5_mean": round(float(v[:k].mean()), 4), "last5_mean": round(float(v[-k:].mean()), 4),
            "host_clock_mean": round(mean_ms, 4),
            "p50_over_host_mean": round(p50 / mean_ms, 4) if mean_ms > 0 else None}


def settle_device(model, barrier, settle_ms: float, elapsed_max=lambda s: s) -> dict:
    """Warm-up policy, before the --warmup steps: replay the step until the device has run it for settle_ms
    of wall time (at least one step). A fresh box's first few milliseconds of replays run slower than its
    steady state (clock and first-replay effects; round 5's driver window was 2.9 % behind its own greedy run
    at --warmup 5), so a count-only warm-up of a few steps does not reach the state the window is meant to
    time. Untimed, like --warmup; --steps and --warmup keep their meaning."""
    n = 0
    t0 = time.perf_counter()
    while True:
        model.step()
        n += 1
        if n % 8 == 0 or settle_ms <= 0:
            barrier()
            # every rank takes the same decision (the max over ranks), so all replay the same step count
            if elapsed_max((time.perf_counter() - t0) * 1e3) >= settle_ms:
                break
    return {"steps": n, "ms": round((time.perf_counter() - t0) * 1e3, 1)}


def progress(msg):
    """A progress line on stderr (long profiled runs stay visibly alive; stdout keeps the one JSON line)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    a = parse()
    progress("start (the first torch import on a fresh box can take a minute or two)")
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
    local = local % max(1, torch.cuda.device_count())  # (several ranks per GPU only in debug runs)
    torch.cuda.set_device(local)

    from simplellminference_amd.model import LlamaModel, comm_id, preset

    cid = None
    if dist_on:
        box = [comm_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        cid = box[0]
    cfg = preset(a.preset, max_length=a.ctx)
    B = a.batch
    own_gpu = dist_on and _own_gpus(dist, torch, local, world)
    if own_gpu:
        # each rank has a GPU of its own: q/k/v + attention as one launch on the shards where it fits
        # (csrc/qkv_attn.h; its attention workgroups wait inside the launch, so ranks sharing a GPU keep two launches)
        os.environ.setdefault("SLI_QKV_ATTN", "1")
    model = LlamaModel(config=cfg, w_dtype=a.w_dtype, kv_dtype="f16", tp_rank=rank, tp_size=world, comm_id=cid,
                       device=local, seed=1, batch=B).init()
    model.fill_kv_synthetic(7, a.ctx - 1)
    for b in range(B):  # every sequence at position ctx-1 (KV rows 0..ctx-2 resident), its own token
        model.set_state_seq(b, (1234 + 17 * b) % model.config.vocab_size, a.ctx - 1, advance=False)

    def barrier():
        model.sync()
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()

    allreduce = "none"
    exec_mode = "launches"
    if dist_on:
        allreduce = "rccl"
        # auto: the exchange inside wo / down per workgroup (batch 1: the GEMV; batch > 1: per MFMA group) when
        # every rank has a GPU of its own (ranks sharing one would starve each other of CUs), else batch 1 through
        # one summing workgroup per launch, batch > 1 through the sliced one-shot launch
        os_mode = (a.tp_allreduce if a.tp_allreduce in ("oneshot", "fused", "fused_wg")
                   else "fused_wg" if own_gpu else ("fused" if B == 1 else "oneshot"))
        if os.environ.get("SLI_DEBUG_NOCOMM") and a.tp_allreduce != "rccl":
            # debug (several ranks on one GPU, no RCCL communicator): the one-shot kernels are the only exchange
            from simplellminference_amd import tp
            tp.open_oneshot(model)
            model.set_allreduce(os_mode)
            allreduce = f"{os_mode} (SLI_DEBUG_NOCOMM: not validated against rccl)"
            if os_mode == "fused_wg" and a.tp_exec != "launches":  # rehearsal: persist held to the fused_wg step
                model.step()
                exec_mode = _try_persist(model, dist, torch, model.logits()[0].copy(), a.tp_exec == "persist", B)
                exec_mode = exec_mode.replace("against rccl", "against the fused_wg launch graph (SLI_DEBUG_NOCOMM)")
        elif a.tp_allreduce != "rccl" and not _oneshot_opened(model, dist, torch, a.tp_allreduce):
            allreduce = "rccl (one-shot buffers could not be mapped on every rank)"
        elif a.tp_allreduce != "rccl":
            import numpy as np
            model.step()  # RCCL reference step (idempotent: position ctx-1 is recomputed)
            ref = model.logits()[0].copy()
            model.set_allreduce(os_mode)
            model.step()
            got = model.logits()[0]
            ok = bool(model.state()["error"] == 0 and np.isfinite(got).all() and np.abs(got - ref).max() <= 1e-3)
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if flag.item() == 1:
                allreduce = f"{os_mode} (validated against rccl on every rank)"
                if os_mode == "fused_wg" and a.tp_exec != "launches":
                    exec_mode = _try_persist(model, dist, torch, ref, a.tp_exec == "persist", B)
            elif a.tp_allreduce in ("oneshot", "fused", "fused_wg"):
                raise SystemExit("one-shot all-reduce disagrees with RCCL")
            else:
                model.set_allreduce("rccl")
                for b in range(B):  # clears a timed-out one-shot's device error flag
                    model.set_state_seq(b, (1234 + 17 * b) % model.config.vocab_size, a.ctx - 1, advance=False)
                allreduce = "rccl (one-shot validation failed)"
    progress("model ready, timing the step")
    def elapsed_max(v):
        if not dist_on:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    settle = settle_device(model, barrier, a.settle_ms, elapsed_max)
    for _ in range(a.warmup):
        model.step()
    barrier()
    # one HIP event after every graph replay on the engine's own stream (no host sync inside the loop): the
    # per-step device durations behind step_ms (SURVEY §5's p50 / p99; model.cpp:157-185 is the loop timed)
    marks = StepMarks(torch, model, local, a.steps)
    t0 = time.perf_counter()
    marks.start()
    for i in range(a.steps):
        model.step()
        marks.mark(i)
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
    progress("timed; per-family probes")
    fam = model.time_families(a.gemv_iters)
    sfl = model.time_stream(a.gemv_iters)  # the measured streaming-read floor of the same launches
    g = model.time_gemv(a.gemv_iters)
    # the dominant kernel: the family with the largest device time per step
    dom = max(fam, key=lambda f: fam[f]["avg_us"] * fam[f]["launches_per_step"])
    d = fam[dom]
    step_dev_us = sum(f["avg_us"] * f["launches_per_step"] for f in fam.values())
    achieved = d["bytes_per_launch"] / (d["avg_us"] * 1e-6) / 1e9

    # a true greedy decode beside the idempotent-step timing: 64 tokens at positions ctx-64 .. ctx-1, the
    # state (position, next token = greedy argmax) advancing on the device every step
    progress("greedy run")
    g_steps = min(a.greedy_steps, a.ctx - 1)
    for b in range(B):
        model.set_state_seq(b, (1234 + 17 * b) % model.config.vocab_size, a.ctx - 1 - g_steps, advance=True)
    barrier()
    tg = time.perf_counter()
    for _ in range(g_steps):
        model.step()
    barrier()
    tg = time.perf_counter() - tg
    gst = [model.state(b) for b in range(B)]
    greedy = {"tokens": B * g_steps, "tokens_per_s": round(B * g_steps / tg, 2), "ms_per_step": round(1e3 * tg / g_steps, 4),
              "positions": f"{a.ctx - 1 - g_steps}..{a.ctx - 2}",
              "final_pos_ok": all(x["pos"] == a.ctx - 1 for x in gst) and not any(x["error"] for x in gst)}

    traffic, traffic_family = None, {}
    tkey = f"{a.preset}/{a.w_dtype}/tp{world}" + (f"/b{B}" if B > 1 else "")
    traffic_source = {"file": os.path.relpath(a.traffic_json, ROOT), "key": tkey, "family": dom,
                      "field": "per_family_hbm_bytes_per_launch", "found": False,
                      "note": "rocprofv3 --pmc FETCH_SIZE pass (tools/pmc_traffic.sh), KiB x 1024 x 2 (gfx950 correction); "
                              "a committed builder pass, not measured in this run"}
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            if tkey in tj:
                traffic_family = tj[tkey].get("per_family_hbm_bytes_per_launch", {})
                traffic = traffic_family.get(dom)
                traffic_source["found"] = traffic is not None
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
                   "step_bytes_per_gpu": round(wbytes + kvbytes),
                   "hbm_roofline_tokens_per_s": round(B * HBM_PEAK_GBS * 1e9 / (wbytes + kvbytes), 1),
                   "step_frac_of_hbm_peak": round((wbytes + kvbytes) / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)},
        "exec": exec_mode,
        "tp_allreduce": allreduce,
        "qkv_attn_fused": model.fused_qkv_attn(),
        "roofline": {"bound": "hbm", "kernel": f"{dom}: {FAMILY_KERNELS[B > 1][dom]}",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_source,
                     "avg_launch_us": round(d["avg_us"], 3), "algorithmic_bytes_per_launch": round(d["bytes_per_launch"]),
                     "stream_floor_us": round(sfl[dom], 3) if dom in sfl else None,
                     "stream_floor_gbs": (round(d["bytes_per_launch"] / (sfl[dom] * 1e-6) / 1e9, 1)
                                          if dom in sfl else None),
                     "frac_of_stream": round(sfl[dom] / d["avg_us"], 4) if dom in sfl else None,
                     "launches_per_step": d["launches_per_step"],
                     "share_of_step_device_time": round(d["avg_us"] * d["launches_per_step"] / step_dev_us, 4),
                     "families_note": "the step's launches by family",
                     "families": {f: {"avg_launch_us": round(v["avg_us"], 3),
                                      "bytes_per_launch": round(v["bytes_per_launch"]),
                                      "launches_per_step": v["launches_per_step"],
                                      "gbs": round(v["bytes_per_launch"] / (v["avg_us"] * 1e-6) / 1e9, 1),
                                      "frac": round(v["bytes_per_launch"] / (v["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                                      "traffic": traffic_family.get(f),
                                      "stream_floor_us": round(sfl[f], 3),
                                      "frac_of_stream": round(sfl[f] / v["avg_us"], 4)}
                                  for f, v in fam.items()},
                     "weight_streaming_average": {"avg_launch_us": round(g["avg_us"], 3),
                                                  "bytes_per_launch": round(g["bytes_per_launch"]),
                                                  "launches_per_step": g["launches_per_step"],
                                                  "frac": round(g["bytes_per_launch"] / (g["avg_us"] * 1e-6) / 1e9
                                                                / HBM_PEAK_GBS, 4)}},
        "greedy_64": greedy,
        "step_ms": step_stats(marks.durations_ms(), ms),
        "settle": {**settle, "note": "untimed replays before the --warmup steps (--settle-ms)"},
    }
    out["greedy_64"]["timed_mean_over_greedy"] = round(ms / greedy["ms_per_step"], 4)
    if exec_mode.startswith("persist"):
        out["roofline"]["families_note"] = ("the launch graph's kernels by family (sli_model_time_families), probed beside "
                                            "the step: the timed step ran the layer stack as ONE persistent launch per "
                                            "rank (tp_layers_kernel), so these are the fallback path's launches")
    if B > 1:  # MFMA work of the batched projections: 2 flop per weight per sequence
        wb_el = {"f16": 2.0, "i8": 1.0, "f32": 4.0}[a.w_dtype]
        proj = [f for f in fam if f != "attention"]
        flops = sum(2.0 * B * fam[f]["bytes_per_launch"] / wb_el * fam[f]["launches_per_step"] for f in proj)
        t = sum(fam[f]["avg_us"] * fam[f]["launches_per_step"] for f in proj) * 1e-6
        tflops = flops / t / 1e12
        out["roofline"]["mfma"] = {"kernel": "bgemm_kernel (v_mfma_f32_16x16x32_f16), all projections",
                                   "achieved_tflops": round(tflops, 2), "peak_tflops": 2500.0,
                                   "frac": round(tflops / 2500.0, 5)}
    if a.prefill_tokens > 1 and B == 1 and a.prefill_tokens <= a.ctx:
        progress("prefill")
        # prompt prefill: positions 0..n-2 in chunks of up to 256 through the MFMA GEMMs
        # (prefill.h); the last prompt position is the first decode step (not part of this timing)
        n = a.prefill_tokens
        ids = [(1 + 7919 * i) % cfg.vocab_size for i in range(n)]
        model.prefill(ids)  # warm-up: capture + first run
        barrier()
        tp = time.perf_counter()
        reps = a.prefill_reps
        for _ in range(reps):
            model.prefill(ids)
        barrier()
        tp = (time.perf_counter() - tp) / reps
        wb_el = {"f16": 2.0, "i8": 1.0, "f32": 4.0}[a.w_dtype]
        layer_bytes = wbytes - cfg.vocab_size * cfg.hidden_size * wb_el / world  # this rank's layer weights
        params = layer_bytes / wb_el
        mfma = model.prefill_path() == "mfma"  # the path the engine took (sli_model_prefill_path)
        chunks = []  # (valid rows, padded rows) per chunk (engine.hip kPfSizes)
        for p0 in range(0, n - 1, 256):
            nv = min(256, n - 1 - p0)
            chunks.append((nv, next(m for m in (32, 64, 128, 256) if nv <= m)))
        # weight passes: a GEMM workgroup reads its weight rows once per BM chunk rows (engine.hip
        # StepRecorder::pg tilings); the workgroups of one row block share an XCD and run together, so HBM
        # sees ~one pass per chunk and the rest are L2 hits (PMC: profiles/r3_prefill_pmc.txt)
        D, Il, QD = cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads * cfg.head_dim
        KVD = cfg.num_key_value_heads * cfg.head_dim
        role_w = {"qkv": D * (QD + 2 * KVD), "gu": 2 * D * Il, "out": D * QD + D * Il}
        tot_w = float(sum(role_w.values()))

        def bm(role, M):  # chunk rows per workgroup (engine.hip StepRecorder::pg_pick)
            if M == 32:
                return 32
            if role == "out":
                return 64 if M == 256 else 32
            if a.w_dtype == "i8":
                if role == "gu":
                    return 128 if M == 128 else 64
                return 128 if M == 256 else 64
            if M == 64 or (M == 128 and role == "qkv"):
                return 64
            if M == 256 and role == "gu":
                return 64
            return 128
        passes = sum(role_w[r] / tot_w * (M // bm(r, M)) for _, M in chunks for r in role_w)
        useful = 2.0 * params * (n - 1) * world  # whole-job flops of the projections (1 flop per MAC x 2)
        issued = 4.0 * params * sum(M for _, M in chunks) * world  # hi + lo MFMAs over the padded rows
        out["prefill"] = {"prompt_tokens": n, "positions_prefilled": n - 1,
                          "chunks": [{"rows": nv, "padded": M} for nv, M in chunks],
                          "seconds": round(tp, 5), "tokens_per_s": round((n - 1) / tp, 1),
                          "hbm_weight_passes": len(chunks) if mfma else n - 1,
                          "l2_weight_passes": round(passes, 2) if mfma else n - 1,
                          "projection_tflops": round(useful / tp / 1e12, 2),
                          "mfma_issued_tflops": round(issued / tp / 1e12, 2) if mfma else None,
                          "mfma_peak_tflops": 2500.0,
                          "path": ("MFMA pgemm (v_mfma_f32_16x16x32_f16, fp16 hi + lo activations), chunks of "
                                   "<= 256 positions, block-causal attention" if mfma
                                   else "decode step, teacher-forced (sli_model_prefill_path = 0: fp32 weights, an "
                                        "unsupported shard shape, or a TP rank without an RCCL communicator)"),
                          "vs_token_by_token_s": round((n - 1) * ms * 1e-3, 4)}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.cpu_seconds, a.preset, a.ctx)
    model.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


def _comm_fatal(e: BaseException) -> bool:
    """An RCCL error or an expired bounded wait on this rank (sli.h SLI_ERR_COMM / SLI_ERR_TIMEOUT): the engine has
    already aborted its communicator, so the rank ends here with a non-zero status — no retry, no re-exec."""
    from simplellminference_amd._lib import SLI_ERR_COMM, SLI_ERR_TIMEOUT, SliError
    return isinstance(e, SliError) and e.code in (SLI_ERR_COMM, SLI_ERR_TIMEOUT)


if __name__ == "__main__":
    try:
        main()
    except Exception as e:  # noqa: BLE001 - a wedged communicator must not leave the rank (or the node run) hanging
        if not _comm_fatal(e):
            raise
        print(f"[bench] rank {os.environ.get('RANK', '0')}: {e}; exiting", file=sys.stderr, flush=True)
        os._exit(3)  # skip interpreter teardown: destructors of a torch/RCCL stack behind a dead peer can block
