"""The layer stack as ONE persistent launch (csrc/tp_layers.h, exec mode "persist"): the reference's layer loop
(source/model/model.cpp:50-129) with every dependency edge inside the launch as tagged granules.

* one rank, head_dim-128 shapes small enough for the kernel's per-CU shares (small-h128: MHA; small-h128-gqa: GQA-2):
  40 greedy steps held directly to the oracle and to the launch graph of the same model (tokens bit-exact, logits
  within the north star's 1e-3; measured 1.6e-4 from the oracle, the launch graph's own distance printed beside);
* Llama-2-7B TP-8 / TP-4 rank shards (2 layers, ctx 2048, SLI_DEBUG_NOCOMM: the rank's own step, the exchange a copy
  of the local partial as the launch path's debug mode does) against the launch graph at positions on and around
  the split boundaries (128 keys per split here), each step run twice (idempotent: the launch counter advances the
  tags, the granules are reused);
* two rank PROCESSES on one GPU exchanging through the per-workgroup granule exchange inside the launch (each rank's
  grid capped to 64 workgroups so both fit the chip together), held to the TP = 1 engine and to the oracle;
* the refusals: shapes whose shares do not fit (the unsharded Llama-2-7B) and RCCL-exchanged ranks.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
PROMPT = [1, 17, 42, 99]


def _ocfg(oracle, c):
    return oracle.Config(c.vocab_size, c.hidden_size, c.num_attention_heads, c.num_key_value_heads, c.head_dim,
                         c.intermediate_size, c.num_hidden_layers, c.max_length, c.rms_norm_eps, c.rope_theta)


@pytest.mark.parametrize("name", ["small-h128", "small-h128-gqa"])
def test_persist_one_rank_matches_oracle_and_launches(gpu, oracle, name):
    from simplellminference_amd.model import LlamaModel, preset
    cfg = preset(name)
    m = LlamaModel(config=cfg, w_dtype="f16", kv_dtype="f16", seed=0).init()
    ltoks, llogits = m.predict(PROMPT, 40, want_logits=True)
    m.set_exec("persist")
    assert m.exec_mode() == "persist"
    ptoks, plogits = m.predict(PROMPT, 40, want_logits=True)
    assert m.state()["error"] == 0
    ptoks2, plogits2 = m.predict(PROMPT, 40, want_logits=True)  # again: new tags, reused granules
    m.close()
    om = oracle.Model(_ocfg(oracle, cfg), seed=0, wmode=oracle.W_F16, kv_f16=True)
    otoks, ologits = om.predict(PROMPT, 40)
    om.close()
    err = float(np.abs(plogits - ologits).max())
    print(f"{name}: persist vs oracle max|dlogit| {err:.2e} (launches vs oracle "
          f"{float(np.abs(llogits - ologits).max()):.2e}), persist vs launches {float(np.abs(plogits - llogits).max()):.2e}")
    assert np.array_equal(ptoks, otoks) and np.array_equal(ptoks, ltoks)
    assert err <= 1e-3
    assert float(np.abs(plogits - llogits).max()) <= 1e-3
    assert np.array_equal(ptoks2, ptoks) and np.array_equal(plogits2, plogits)  # deterministic


POSITIONS = [0, 1, 127, 128, 129, 255, 1000, 2046, 2047]


@pytest.mark.parametrize("world", [8, 4])
def test_persist_tp_shard_nocomm_matches_launches(gpu, monkeypatch, world):
    from simplellminference_amd.model import LlamaModel, preset
    monkeypatch.setenv("SLI_DEBUG_NOCOMM", "1")
    cfg = preset("llama2-7b", num_hidden_layers=2)
    m = LlamaModel(config=cfg, w_dtype="f16", kv_dtype="f16", seed=1, tp_rank=world - 1, tp_size=world).init()
    m.fill_kv_synthetic(7, 2047)
    rows = {}
    for mode in ("launches", "persist"):
        m.set_exec(mode)
        out = []
        for p in POSITIONS:
            a = m.forward(100 + p % 300, p)
            b = m.forward(100 + p % 300, p)
            assert np.array_equal(a, b), (mode, p)
            out.append(a)
        rows[mode] = np.stack(out)
        assert m.state()["error"] == 0
    m.close()
    a, b = rows["persist"], rows["launches"]
    assert np.isfinite(a).all()
    rel = float(np.abs(a - b).max() / max(1.0, float(np.abs(b).max())))
    print(f"TP-{world} rank {world - 1}: persist vs launches max rel {rel:.2e}")
    assert rel <= 1e-4


def test_persist_refuses_unfitting_shapes(gpu):
    from simplellminference_amd import SliError
    from simplellminference_amd.model import LlamaModel, preset
    m = LlamaModel(config=preset("llama2-7b", num_hidden_layers=1), w_dtype="f16", kv_dtype="f16", seed=1).init()
    with pytest.raises(SliError, match="persistent layers"):
        m.set_exec("persist")  # the unsharded 7B: shares beyond the kernel's LDS partial buffer
    m.close()
    m = LlamaModel(config=preset("tiny"), w_dtype="f16", kv_dtype="f16", seed=1).init()
    with pytest.raises(SliError, match="head_dim 128"):
        m.set_exec("persist")
    m.close()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                      SLI_DEBUG_NOCOMM="1",  # no RCCL communicator: the granule exchange is the only one
                      SLI_DEBUG_GEMV_MAX_BLOCKS=str(256 // (2 * world)))  # every rank's grid resident together
    import torch
    import torch.distributed as dist

    from simplellminference_amd import tp
    from simplellminference_amd.model import LlamaModel, preset
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = rank % torch.cuda.device_count()
        m = LlamaModel(config=preset(name), w_dtype="f16", kv_dtype="f16", tp_rank=rank, tp_size=world, device=dev,
                       seed=0).init()
        tp.open_oneshot(m)
        m.set_allreduce("fused_wg")
        m.set_exec("persist")
        dist.barrier()
        toks, logits = m.predict(PROMPT, 16, want_logits=True)
        err = m.state()["error"]
        parts = [torch.zeros(logits.shape, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(logits)))
        dist.barrier()
        m.close()
        if rank == 0:
            q.put(("ok", toks, np.concatenate([p.numpy() for p in parts], axis=-1), err))
    except Exception as e:  # report to the parent instead of hanging it
        q.put(("err", repr(e), None, None))
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("small-h128", 2), ("small-h128-gqa", 2), ("small-h128", 4)])
def test_persist_exchange_between_rank_processes(gpu, oracle, name, world):
    from simplellminference_amd.model import LlamaModel, preset
    ref = LlamaModel(config=preset(name), w_dtype="f16", kv_dtype="f16", seed=0).init()
    rtoks, rlogits = ref.predict(PROMPT, 16, want_logits=True)
    ref.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, toks, logits, err = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", toks
    assert err == 0
    assert np.array_equal(toks, rtoks)
    assert np.abs(logits - rlogits).max() <= 1e-3
    om = oracle.Model(_ocfg(oracle, preset(name)), seed=0, wmode=oracle.W_F16, kv_f16=True)
    otoks, ologits = om.predict(PROMPT, 16)
    om.close()
    assert np.array_equal(toks, otoks)
    assert np.abs(logits - ologits).max() <= 1e-3
