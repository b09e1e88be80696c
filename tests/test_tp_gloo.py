"""Tensor parallelism on CPU (gloo, world_size 2, 4 and 8): the shard plan libsli.so uses
(sli_tp_plan / sli_tp_vocab) applied to the oracle's weights, the per-rank partial computation the
engine performs (local heads / FFN columns / vocab rows, residual added on rank 0 only), gloo
all-reduces where the engine all-reduces over RCCL, and the packed-key distributed argmax. The result
must match the unsharded oracle: logits within 1e-4 (fp32, different summation order), tokens exact."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

PROMPT = [1, 17, 42, 99]
STEPS = 12


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _key(val: float, idx: int) -> int:
    """Signed-int64 form of the device's orderable argmax key (common.h argmax_key)."""
    u = int(np.array([val], np.float32).view(np.uint32)[0])
    ordv = (~u & 0xFFFFFFFF) if (u & 0x80000000) else (u | 0x80000000)
    return ((ordv << 32) | (0xFFFFFFFF - idx)) - (1 << 63)


def _cfg(n_kv):
    """tiny (MHA, 4 heads), tiny-gqa (4/2) or, for world 8 (config C2's degree), an 8-head MHA variant of
    the tiny shape (head_dim 32) so every rank owns one head."""
    from simplellminference_amd.model import preset
    if n_kv == 8:
        return preset("tiny", head_dim=32, kv_hidden_size=256, num_attention_heads=8, num_key_value_heads=8)
    return preset("tiny" if n_kv == 4 else "tiny-gqa")


def _worker(rank, world, port, n_kv, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import oracle as O
    from simplellminference_amd import tp

    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _cfg(n_kv)
    ocfg = O.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                    cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length, cfg.rms_norm_eps,
                    cfg.rope_theta)
    full = O.Model(ocfg, seed=0)
    L, D, hd, T = cfg.num_hidden_layers, cfg.hidden_size, cfg.head_dim, cfg.max_length
    hq, hkv = cfg.num_attention_heads // world, cfg.num_key_value_heads // world
    win = {k: tp.shard_window(cfg, k, rank, world) for k in ("wq", "wk", "wv", "wo", "gate", "up", "down")}
    W = {k: [np.ascontiguousarray(tp.take(full.weight(getattr(O, "T_" + k.upper()), l), win[k])) for l in range(L)]
         for k in win}
    vlo, vn = tp.vocab_shard(cfg, rank, world)
    emb = full.weight(O.T_EMB)
    head = np.ascontiguousarray(emb[vlo:vlo + vn])
    norms = [full.weight(O.T_NORM, i) for i in range(2 * L + 1)]
    sin_c, cos_c = O.rope_cache(hd, T, cfg.rope_theta)
    kc = np.zeros((L, T, hkv * hd), np.float32)
    vc = np.zeros_like(kc)

    def allreduce(a, op=dist.ReduceOp.SUM):
        t = torch.from_numpy(a)
        dist.all_reduce(t, op=op)
        return t.numpy()

    token, logits_all, toks = PROMPT[0], [], []
    for pos in range(STEPS):
        toks.append(token)
        x = O.embedding(token, emb)
        for l in range(L):
            h = O.rmsnorm(x, norms[2 * l], cfg.rms_norm_eps)
            q = O.matmul(h, W["wq"][l])
            k = O.matmul(h, W["wk"][l])
            v = O.matmul(h, W["wv"][l])
            q, k = O.rope(q, k, pos, sin_c, cos_c, hd)
            kc[l, pos], vc[l, pos] = k, v
            a = O.mha(q, kc, vc, l, pos, T, hd, hq, hkv)
            part = O.matmul(a, W["wo"][l])
            x1 = allreduce(x + part if rank == 0 else part)
            h = O.rmsnorm(x1, norms[2 * l + 1], cfg.rms_norm_eps)
            act = O.swiglu(O.matmul(h, W["up"][l]), O.matmul(h, W["gate"][l]))
            part = O.matmul(act, W["down"][l])
            x = allreduce(x1 + part if rank == 0 else part)
        h = O.rmsnorm(x, norms[2 * L], cfg.rms_norm_eps)
        local = O.matmul(h, head)
        i = O.argmax(local)
        key = allreduce(np.array([_key(local[i], vlo + i)], np.int64), dist.ReduceOp.MAX)[0]
        nxt = 0xFFFFFFFF - ((int(key) + (1 << 63)) & 0xFFFFFFFF)
        parts = [torch.zeros(vn, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(local))
        logits_all.append(np.concatenate([p.numpy() for p in parts]))
        token = PROMPT[pos + 1] if pos + 1 < len(PROMPT) else nxt
    if rank == 0:
        out.put((np.array(toks), np.stack(logits_all)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_kv", [(2, 4), (2, 2), (4, 4), (8, 8)])
def test_tensor_parallel_matches_unsharded_oracle(oracle, world, n_kv):
    from simplellminference_amd import build
    build.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_kv, q)) for r in range(world)]
    for p in procs:
        p.start()
    toks, logits = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg = _cfg(n_kv)
    m = oracle.Model(oracle.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                                   cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                                   cfg.rms_norm_eps, cfg.rope_theta), seed=0)
    otoks, ologits = m.predict(PROMPT, STEPS)
    assert np.array_equal(toks, otoks)
    assert np.abs(logits - ologits).max() < 1e-4


def test_shard_plan_covers_every_weight_exactly_once():
    from simplellminference_amd import build, tp
    from simplellminference_amd.model import preset
    build.build()
    for name, world in (("llama2-7b", 8), ("llama3-8b", 8), ("tiny-gqa", 2)):
        cfg = preset(name)
        shapes = {"wq": (cfg.hidden_size, cfg.hidden_size), "wk": (cfg.kv_hidden_size, cfg.hidden_size),
                  "wv": (cfg.kv_hidden_size, cfg.hidden_size), "wo": (cfg.hidden_size, cfg.hidden_size),
                  "gate": (cfg.intermediate_size, cfg.hidden_size), "up": (cfg.intermediate_size, cfg.hidden_size),
                  "down": (cfg.hidden_size, cfg.intermediate_size)}
        for k, (R, C) in shapes.items():
            cover = np.zeros((R, C), np.int8) if R * C < 2e8 else None
            total = 0
            for r in range(world):
                w = tp.shard_window(cfg, k, r, world)
                total += w.n_rows * w.n_cols
                if cover is not None:
                    cover[w.row_lo:w.row_lo + w.n_rows, w.col_lo:w.col_lo + w.n_cols] += 1
            assert total == R * C
            if cover is not None:
                assert (cover == 1).all()
        vs = [tp.vocab_shard(cfg, r, world) for r in range(world)]
        assert vs[0][0] == 0 and sum(n for _, n in vs) == cfg.vocab_size
        assert all(vs[i][0] + vs[i][1] == vs[i + 1][0] for i in range(world - 1))
