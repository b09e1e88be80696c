"""The engine's RCCL tensor-parallel path on the GPU: two ranks (two processes) built with tp_size=2,
compared with the TP=1 engine on the same synthetic weights. On a one-GPU box both ranks share
device 0 when RCCL allows it; if RCCL refuses duplicate devices the test is skipped (the multi-GPU
bench then exercises the path). Bar: greedy tokens identical, logits within 1e-3 (fp16 weights)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
PROMPT = [1, 17, 42, 99]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    import torch.distributed as dist

    from simplellminference_amd import tp
    from simplellminference_amd.model import LlamaModel, preset
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ndev = torch.cuda.device_count()
        dev = rank % ndev
        cid = tp.broadcast_comm_id(rank)
        m = LlamaModel(config=preset(name), w_dtype="f16", kv_dtype="f16", tp_rank=rank, tp_size=world,
                       comm_id=cid, device=dev, seed=0).init()
        toks, logits = m.predict(PROMPT, 16, want_logits=True)
        parts = [torch.zeros(logits.shape, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(logits))
        m.close()
        if rank == 0:
            q.put(("ok", toks, np.concatenate([p.numpy() for p in parts], axis=1)))
    except Exception as e:  # report to the parent instead of hanging it
        q.put(("err", repr(e), None))
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["tiny", "tiny-gqa"])
def test_rccl_tp2_matches_tp1(gpu, name):
    from simplellminference_amd.model import LlamaModel, preset
    ref = LlamaModel(config=preset(name), w_dtype="f16", kv_dtype="f16", seed=0).init()
    rtoks, rlogits = ref.predict(PROMPT, 16, want_logits=True)
    ref.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    status, toks, logits = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    if status == "err":
        if "Duplicate GPU" in toks or "ncclInvalidUsage" in toks or "invalid usage" in toks.lower():
            pytest.skip(f"RCCL refuses two ranks on one device: {toks}")
        raise AssertionError(toks)
    assert np.array_equal(toks, rtoks)
    assert np.abs(logits - rlogits).max() <= 1e-3


def _oracle_for(oracle, name, wmode, kv_f16):
    c = _preset(name)  # "preset:layers" too
    return oracle.Model(oracle.Config(c.vocab_size, c.hidden_size, c.num_attention_heads, c.num_key_value_heads,
                                      c.head_dim, c.intermediate_size, c.num_hidden_layers, c.max_length,
                                      c.rms_norm_eps, c.rope_theta), seed=0, wmode=wmode, kv_f16=kv_f16)


def test_tp_step_on_one_rank_communicator(gpu, oracle, monkeypatch):
    """SLI_DEBUG_FORCE_COMM: the TP step (partials into xpart, residual on rank 0, RCCL sum all-reduces and
    the uint64 MAX argmax all-reduce, all captured in the hipGraph) on a 1-rank RCCL communicator."""
    from simplellminference_amd.model import LlamaModel, preset
    monkeypatch.setenv("SLI_DEBUG_FORCE_COMM", "1")
    m = LlamaModel(config=preset("tiny-gqa"), w_dtype="f16", kv_dtype="f16", seed=0).init()
    toks, logits = m.predict(PROMPT, 36, want_logits=True)
    m.close()
    otoks, ologits = _oracle_for(oracle, "tiny-gqa", oracle.W_F16, True).predict(PROMPT, 36)
    assert np.array_equal(toks, otoks)
    assert np.abs(logits - ologits).max() <= 1e-3


@pytest.mark.parametrize("w", ["f16", "i8"])
@pytest.mark.parametrize("world", [2, 4])
def test_tp_shard_placement_on_device(gpu, oracle, monkeypatch, w, world):
    """Every rank's device shard equals the plan window of the full (rounded / quantised) weights; int8
    column shards (wo, down) keep the full-row scales."""
    from simplellminference_amd import tp
    from simplellminference_amd.model import LlamaModel, preset
    monkeypatch.setenv("SLI_DEBUG_NOCOMM", "1")
    cfg = preset("tiny")
    om = _oracle_for(oracle, "tiny", oracle.W_F16 if w == "f16" else oracle.W_I8, True)
    kinds = {"wq": oracle.T_WQ, "wk": oracle.T_WK, "wv": oracle.T_WV, "wo": oracle.T_WO, "gate": oracle.T_GATE,
             "up": oracle.T_UP, "down": oracle.T_DOWN}
    for r in range(world):
        m = LlamaModel(config=cfg, w_dtype=w, kv_dtype="f16", tp_rank=r, tp_size=world, seed=0).init()
        for name, kind in kinds.items():
            for layer in range(cfg.num_hidden_layers):
                want = tp.take(om.weight(kind, layer), tp.shard_window(cfg, name, r, world))
                assert np.array_equal(m.weight_shard(kind, layer), want), (r, name, layer)
        assert np.array_equal(m.weight_shard(oracle.T_EMB), om.weight(oracle.T_EMB))
        m.close()


@pytest.mark.parametrize("w", ["f16", "i8"])
@pytest.mark.parametrize("world", [2, 8])
def test_tp_rank_of_c2_shapes_steps_nocomm(gpu, monkeypatch, w, world):
    """One rank of config C2 (Llama-2-7B shapes, 2 layers, ctx 2048, TP 2 / 8): the rank's GEMV shapes
    (TP 8: qkv 1536x4096, wo 4096x512, gate/up 2752x4096, down 4096x1376, LM head 4000x4096, 4 heads of
    attention) plan, allocate and step without a communicator (SLI_DEBUG_NOCOMM: kernel shapes and
    placement only, the values are not a model); the step is deterministic and idempotent."""
    from simplellminference_amd.model import LlamaModel, preset
    monkeypatch.setenv("SLI_DEBUG_NOCOMM", "1")
    cfg = preset("llama2-7b", num_hidden_layers=2)
    m = LlamaModel(config=cfg, w_dtype=w, kv_dtype="f16", seed=1, tp_rank=world - 1, tp_size=world).init()
    m.fill_kv_synthetic(7, 2047)
    a = m.forward(1234, 2047)
    b = m.forward(1234, 2047)
    assert a.shape == (cfg.vocab_size // world,) and np.isfinite(a).all() and np.array_equal(a, b)
    m.close()


LONG_PROMPT = [(7 * i + 3) % 500 for i in range(23)]


def _preset(name):
    """"llama2-7b:2" = the preset cut to 2 layers (full-size shard shapes in a test-sized step)."""
    from simplellminference_amd.model import preset
    base, _, layers = name.partition(":")
    return preset(base, num_hidden_layers=int(layers)) if layers else preset(base)


def _prompts(batch):
    return ([PROMPT, [5, 6, 7]] + [[9 + b, 3, 11, b] for b in range(2, batch)])[:batch]


def _oneshot_rank(rank, world, port, name, batch, q, mode="oneshot", w="f16", prefill=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                      SLI_DEBUG_NOCOMM="1")  # no RCCL communicator: the one-shot kernels are the only exchange
    mode, _, qa = mode.partition("+")  # "+qa": q/k/v + attention as one launch (qkv_attn.h) on the ranks too
    if qa:
        os.environ["SLI_QKV_ATTN"] = "1"
    if mode == "fused_wg":  # every workgroup waits for its peers': the ranks' grids must fit the one GPU together
        os.environ["SLI_DEBUG_GEMV_MAX_BLOCKS"] = str(256 // (2 * world))
    import torch
    import torch.distributed as dist

    from simplellminference_amd import tp
    from simplellminference_amd.model import LlamaModel, preset
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = rank % torch.cuda.device_count()
        m = LlamaModel(config=_preset(name), w_dtype=w, kv_dtype="f16", tp_rank=rank, tp_size=world,
                       device=dev, seed=0, batch=batch).init()
        tp.open_oneshot(m)
        m.set_allreduce(mode)
        if qa and m.fused_qkv_attn() != 1:
            raise AssertionError("+qa: the q/k/v + attention launch was not taken at this shape")
        dist.barrier()
        if prefill:
            path = m.prefill_path()
            toks, logits = m.predict_prefill(LONG_PROMPT, 32, want_logits=True)
        elif batch == 1:
            toks, logits = m.predict(PROMPT, 16, want_logits=True)
        else:
            toks, logits = m.predict_batch(_prompts(batch), 16, want_logits=True)
        err = m.state()["error"]
        parts = [torch.zeros(logits.shape, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(logits)))
        dist.barrier()
        m.close()
        if rank == 0:
            q.put(("ok", toks, np.concatenate([p.numpy() for p in parts], axis=-1), err if not prefill else (err, path)))
    except Exception as e:  # report to the parent instead of hanging it
        q.put(("err", repr(e), None, None))
    dist.destroy_process_group()


@pytest.mark.parametrize("name,batch,mode", [("tiny", 1, "oneshot"), ("tiny-gqa", 1, "oneshot"), ("tiny-gqa", 2, "oneshot"),
                                             ("tiny", 1, "fused"), ("tiny-gqa", 1, "fused"), ("tiny-h8", 1, "fused"),
                                             ("tiny", 1, "fused_wg"), ("tiny-gqa", 1, "fused_wg"),
                                             ("tiny-h8", 1, "fused_wg"), ("tiny-gqa", 2, "fused_wg"),
                                             ("llama3-8b:2", 8, "fused_wg"), ("llama3-8b:2", 8, "oneshot"),
                                             ("tiny", 1, "fused_wg+qa"), ("tiny-gqa", 1, "oneshot+qa"),
                                             ("tiny-gqa", 1, "fused+qa")])
def test_oneshot_allreduce_two_processes(gpu, oracle, name, batch, mode):
    """The one-shot all-reduce (oneshot.h) between two rank PROCESSES through IPC-mapped uncached buffers
    (both on device 0 here; on the 8-GPU node each on its own GPU, over xGMI): greedy tokens identical to
    the TP = 1 engine, logits within 1e-3, no device error (the bounded waits never gave up). mode "fused":
    the exchange runs inside the wo / down GEMV launches (EpiPush: rows pushed from the epilogue, the
    launch's last workgroup waits and sums); "fused_wg": per workgroup (each waits for the same workgroup of
    the peer and sums its own rows; the grids capped so both ranks' launches fit the one GPU together), at batch
    > 1 inside the MFMA wo / down (BgEpiPush, per group). "llama3-8b:2": the C4 shard shapes at TP 2 (2 layers,
    batch 8): the per-group exchange and the sliced one-shot launch."""
    from simplellminference_amd.model import LlamaModel
    ref = LlamaModel(config=_preset(name), w_dtype="f16", kv_dtype="f16", seed=0, batch=batch).init()
    if batch == 1:
        rtoks, rlogits = ref.predict(PROMPT, 16, want_logits=True)
    else:
        rtoks, rlogits = ref.predict_batch(_prompts(batch), 16, want_logits=True)
    ref.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_oneshot_rank, args=(r, 2, port, name, batch, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    status, toks, logits, err = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", toks
    assert err == 0
    assert np.array_equal(toks, rtoks)
    assert np.abs(logits - rlogits).max() <= 1e-3
    if mode.endswith("+qa"):
        otoks, ologits = _oracle_for(oracle, name, oracle.W_F16, True).predict(PROMPT, 16)
        assert np.array_equal(toks, otoks)
        assert np.abs(logits - ologits).max() <= 1e-3


@pytest.mark.parametrize("mode", ["oneshot", "fused"])
def test_oneshot_prefill_two_processes(gpu, mode):
    """Prompt prefill on two rank processes whose only exchange is the one-shot all-reduce (no RCCL
    communicator): the chunked prefill has no exchange for a chunk's residual rows, so the engine takes the
    teacher-forced decode path (sli_model_prefill_path == 0), whose one-shot exchange it does have; tokens equal
    the TP = 1 engine's prefilled predict, logits within 1e-3 (prefill used to copy the unreduced
    partials there)."""
    from simplellminference_amd.model import LlamaModel, preset
    ref = LlamaModel(config=preset("tiny-gqa"), w_dtype="f16", kv_dtype="f16", seed=0).init()
    assert ref.prefill_path() == "mfma"
    rtoks, rlogits = ref.predict_prefill(LONG_PROMPT, 32, want_logits=True)
    ref.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_oneshot_rank, args=(r, 2, port, "tiny-gqa", 1, q, mode, "f16", True))
             for r in range(2)]
    for p in procs:
        p.start()
    status, toks, logits, info = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", toks
    err, path = info
    assert err == 0 and path == "decode"
    assert np.array_equal(toks, rtoks)
    n = len(LONG_PROMPT)
    assert np.abs(logits[n - 1:] - rlogits[n - 1:]).max() <= 1e-3


@pytest.mark.parametrize("name,world,mode,w", [("tiny-h8", 4, "fused", "f16"), ("tiny-h8", 4, "oneshot", "f16"),
                                               ("tiny-gqa", 2, "fused", "i8"), ("tiny-h8", 4, "fused_wg", "f16"),
                                               ("tiny-gqa", 2, "fused_wg", "i8"), ("llama2-7b:2", 2, "fused_wg", "f16"),
                                               ("llama2-7b:2", 2, "fused", "f16"), ("tiny-h8", 4, "fused_wg+qa", "f16"),
                                               ("tiny-gqa", 2, "fused+qa", "i8"), ("tiny-h8", 4, "fused+qa", "f16"),
                                               ("llama2-7b:2", 4, "fused+qa", "f16")])
def test_oneshot_allreduce_more_ranks(gpu, oracle, name, world, mode, w):
    """The one-shot exchange (separate launch or fused into wo / down) between 4 rank processes on one GPU, the
    fused forms with int8 weights, and both fused forms at Llama-2-7B shard shapes (2 layers, TP 2: 64 / 256
    workgroups per wo / down launch): tokens identical to the TP = 1 engine, logits within 1e-3, no device
    error. "+qa": q/k/v + attention as one launch on every rank, also held directly to the oracle, at the tiny
    shapes and at Llama-2-7B's TP-4 shards (2 layers, head_dim 128, 8 heads x 8 splits per rank)."""
    from simplellminference_amd.model import LlamaModel
    ref = LlamaModel(config=_preset(name), w_dtype=w, kv_dtype="f16", seed=0).init()
    rtoks, rlogits = ref.predict(PROMPT, 16, want_logits=True)
    ref.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_oneshot_rank, args=(r, world, port, name, 1, q, mode, w)) for r in range(world)]
    for p in procs:
        p.start()
    status, toks, logits, err = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", toks
    assert err == 0
    assert np.array_equal(toks, rtoks)
    assert np.abs(logits - rlogits).max() <= 1e-3
    if mode.endswith("+qa"):
        otoks, ologits = _oracle_for(oracle, name, oracle.W_F16 if w == "f16" else oracle.W_I8, True).predict(PROMPT, 16)
        assert np.array_equal(toks, otoks)
        assert np.abs(logits - ologits).max() <= 1e-3


def _absent_peer_rank(rank, world, port, q, mode="fused"):
    """Rank 0 steps with the fused exchange while rank 1 never does: rank 0's first wait gives up after the bounded
    spin, every later one at once (oneshot.h os_gave_up)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                      SLI_DEBUG_NOCOMM="1")
    import time

    import torch.distributed as dist

    from simplellminference_amd import SliError, tp
    from simplellminference_amd.model import LlamaModel, preset
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = LlamaModel(config=preset("tiny"), w_dtype="f16", kv_dtype="f16", tp_rank=rank, tp_size=world, seed=0).init()
        tp.open_oneshot(m)
        m.set_allreduce(mode)
        dist.barrier()
        if rank == 0:
            def run(steps):  # steps x (2 layers x the wo / down exchanges + the argmax-key exchange)
                t0 = time.perf_counter()
                msg = ""
                try:
                    m.predict(PROMPT, steps)  # resets the state (and its error bits) first
                except SliError as e:  # the device error check at the end of predict
                    msg = str(e)
                return time.perf_counter() - t0, msg
            t1, msg1 = run(1)
            t3, msg3 = run(3)
            refused = False
            try:
                m.set_allreduce("oneshot")
            except SliError:
                refused = True
            q.put(("ok", (t1, t3), (msg1, msg3), refused))
        dist.barrier()  # rank 1 stays until rank 0 is done with the buffers it mapped
        m.close()
    except Exception as e:  # report to the parent instead of hanging it
        q.put(("err", repr(e), None, None))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["fused", "fused_wg"])
def test_oneshot_absent_peer_gives_up_once(gpu, mode):
    """A peer that never arrives (rank 1 maps the buffers and does not step): rank 0's predict ends with
    DevState::error bit 4 after ONE bounded wait, not one per exchange (oneshot.h os_gave_up: later waits give up
    after 4096 polls): 3 steps take about as long as 1 (measured: 1 step, 5 exchanges, 2.57 s; 3 steps, 15 exchanges,
    2.58 s). predict reports the timeout and the one-shot path is refused afterwards (os_dead), so bench.py falls
    back to RCCL."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_absent_peer_rank, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    status, times, msgs, refused = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", times
    assert all("one-shot all-reduce timed out" in msg for msg in msgs), msgs
    t1, t3 = times
    print(f"absent peer ({mode}): 1 step (5 exchanges) {t1:.2f} s, 3 steps (15 exchanges) {t3:.2f} s")
    assert t3 < 2.0 * t1  # one bounded wait each (3x that without the give-up)
    assert refused
