"""Kernel-level parity: each libsli.so operator (HIP, gfx950) against the C oracle on the same seeded
inputs. Tolerances (stated per test): fp32 ops compare within a few fp32 ulps of the row magnitude
(the reduction order differs from the reference's sequential sums); fp16/int8-weight GEMVs compare
against the oracle run in fp32 on the identically rounded / dequantised weights; index results
(argmax) are bit-exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rng(seed=0):
    return np.random.default_rng(seed)


def _t(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _close(got, want, rtol, atol):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    err = np.abs(got - want)
    lim = atol + rtol * np.abs(want)
    assert np.all(err <= lim), f"max err {err.max():.3e} (worst excess {(err - lim).max():.3e})"


@pytest.mark.parametrize("rows,cols", [(1, 8), (7, 256), (4096, 4096), (512, 11008), (33, 100), (250, 768)])
def test_matmul_f32(gpu, oracle, rows, cols):
    torch = gpu
    r = _rng(rows * 7 + cols)
    x = r.standard_normal(cols).astype(np.float32)
    w = (r.standard_normal((rows, cols)) / np.sqrt(cols)).astype(np.float32)
    want = oracle.matmul(x, w)
    from simplellminference_amd import ops
    got = ops.matmul(_t(torch, x), _t(torch, w)).cpu().numpy()
    # fp32 sum over `cols` terms in a different order: bound by cols * eps * sum|x w|
    bound = 4 * np.finfo(np.float32).eps * np.sqrt(cols) * (np.abs(w) @ np.abs(x))
    assert np.all(np.abs(got - want) <= bound + 1e-30), np.abs(got - want).max()


# (256 / 1000 / 2048 rows: fewer two-row units than the chip's 4096 waves, so gemv.h's column split cuts
# each unit's rows over 8 / 8 / 4 waves of its workgroup — the tensor-parallel shard path)
@pytest.mark.parametrize("rows,cols", [(4096, 4096), (11008, 4096), (4096, 11008), (32000, 4096), (768, 256),
                                       (256, 4096), (1000, 4096), (2048, 2048), (1376, 4096)])
def test_matmul_f16_weights(gpu, oracle, rows, cols):
    torch = gpu
    from simplellminference_amd import ops
    r = _rng(rows + cols)
    x = r.standard_normal(cols).astype(np.float32)
    w16 = (r.standard_normal((rows, cols)) / np.sqrt(cols)).astype(np.float16)
    want = oracle.matmul(x, w16.astype(np.float32))
    got = ops.matmul(_t(torch, x), _t(torch, w16)).cpu().numpy()
    _close(got, want, rtol=1e-4, atol=1e-4)  # fp32 accumulation on identical fp16 weights


@pytest.mark.parametrize("rows,cols", [(4096, 4096), (512, 11008), (100, 256), (200, 4096), (1536, 4096)])
def test_matmul_i8_weights(gpu, oracle, rows, cols):
    torch = gpu
    from simplellminference_amd import ops
    r = _rng(3 + rows)
    x = r.standard_normal(cols).astype(np.float32)
    w = (r.standard_normal((rows, cols)) / np.sqrt(cols)).astype(np.float32)
    q = np.empty((rows, cols), np.int8)
    s = np.empty(rows, np.float32)
    for i in range(rows):
        q[i], s[i] = oracle.quant_row_i8(w[i])
    deq = q.astype(np.float32) * s[:, None]
    want = oracle.matmul(x, deq)
    got = ops.matmul(_t(torch, x), _t(torch, q), row_scale=_t(torch, s)).cpu().numpy()
    _close(got, want, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dim", [256, 4096, 3072, 1000])
def test_rmsnorm(gpu, oracle, dim):
    torch = gpu
    from simplellminference_amd import ops
    r = _rng(dim)
    x = r.standard_normal(dim).astype(np.float32)
    w = (1 + 0.1 * r.standard_normal(dim)).astype(np.float32)
    want = oracle.rmsnorm(x, w, 1e-5)
    got = ops.rmsnorm(_t(torch, x), _t(torch, w), 1e-5).cpu().numpy()
    _close(got, want, rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("theta", [10000.0, 100000.0, 500000.0])
def test_rope_cache_bit_exact(gpu, oracle, theta):
    from simplellminference_amd import ops
    s, c = ops.rope_cache(128, 2048, theta)
    ws, wc = oracle.rope_cache(128, 2048, theta)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), ws.view(np.uint32))
    assert np.array_equal(c.cpu().numpy().view(np.uint32), wc.view(np.uint32))


@pytest.mark.parametrize("q_dim,k_dim,hd,pos", [(256, 256, 64, 0), (256, 128, 64, 35), (4096, 4096, 128, 2047),
                                                 (4096, 1024, 128, 1000)])
def test_rope(gpu, oracle, q_dim, k_dim, hd, pos):
    torch = gpu
    from simplellminference_amd import ops
    r = _rng(pos)
    q = r.standard_normal(q_dim).astype(np.float32)
    k = r.standard_normal(k_dim).astype(np.float32)
    s, c = oracle.rope_cache(hd, 2048, 10000.0)
    wq, wk = oracle.rope(q, k, pos, s, c, hd)
    tq, tk = _t(torch, q), _t(torch, k)
    ops.rope(tq, tk, pos, _t(torch, s), _t(torch, c), hd)
    _close(tq.cpu().numpy(), wq, rtol=1e-6, atol=1e-6)
    _close(tk.cpu().numpy(), wk, rtol=1e-6, atol=1e-6)
    # device-resident position (graph-capturable form) gives the same answer
    tq2, tk2 = _t(torch, q), _t(torch, k)
    ops.rope(tq2, tk2, torch.tensor([pos], dtype=torch.int32, device="cuda"), _t(torch, s), _t(torch, c), hd)
    assert torch.equal(tq, tq2) and torch.equal(tk, tk2)


@pytest.mark.parametrize("n", [1, 36, 1000, 4097])
def test_softmax(gpu, oracle, n):
    torch = gpu
    from simplellminference_amd import ops
    x = (3 * _rng(n).standard_normal(n)).astype(np.float32)
    want = oracle.softmax(x)
    got = ops.softmax_(_t(torch, x)).cpu().numpy()
    _close(got, want, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("kv_dtype", ["f32", "f16"])
@pytest.mark.parametrize("T,hd,H,Hkv,layer,pos", [(64, 64, 4, 4, 1, 0), (64, 64, 4, 2, 0, 35), (64, 64, 4, 2, 1, 63),
                                                 (2048, 128, 32, 32, 0, 2047), (2048, 128, 32, 8, 1, 777),
                                                 (300, 128, 8, 1, 0, 299),
                                                 # fp16: the MFMA kernel's split cap (one kv head, 16 splits of 256
                                                 # keys), tile / split boundaries, hd 64 GQA-8
                                                 (4096, 128, 4, 1, 0, 4095), (4096, 128, 4, 1, 1, 255),
                                                 (4096, 128, 32, 8, 1, 1024), (4096, 64, 16, 2, 0, 129),
                                                 # fp16: 8 kv heads x 16384 keys -> 4 tiles per wave, so the per-wave
                                                 # 2-slot ring is refilled (issue(j + NBUF), attn_mfma.h) with waves
                                                 # of 4 / 3 / 1 live tiles; the round-5 lab mismatches
                                                 # appeared exactly past the refill, under a full context
                                                 (16384, 128, 32, 8, 1, 16383), (16384, 128, 32, 8, 0, 16383 - 700),
                                                 (16384, 128, 32, 8, 1, 511 + 96),
                                                 # fp16 hd 64 over 1024 keys, 2 kv heads: the MFMA rule's one tile per
                                                 # wave would give 8 splits of 128 keys against 4 in the partial buffer
                                                 # (sized for the fp32 kernel's 256); the launch now splits at >= 256
                                                 (1024, 64, 16, 2, 1, 1023), (1024, 64, 16, 2, 0, 300)])
def test_mha(gpu, oracle, kv_dtype, T, hd, H, Hkv, layer, pos):
    torch = gpu
    from simplellminference_amd import ops
    r = _rng(T + pos)
    L = 2
    kv = Hkv * hd
    q = r.standard_normal(H * hd).astype(np.float32)
    kc = r.standard_normal((L, T, kv)).astype(np.float32)
    vc = r.standard_normal((L, T, kv)).astype(np.float32)
    if kv_dtype == "f16":
        kc = kc.astype(np.float16).astype(np.float32)
        vc = vc.astype(np.float16).astype(np.float32)
    want = oracle.mha(q, kc, vc, layer, pos, T, hd, H, Hkv)
    tdt = torch.float16 if kv_dtype == "f16" else torch.float32
    got = ops.mha(_t(torch, q), _t(torch, kc).to(tdt), _t(torch, vc).to(tdt), layer, pos, T, hd, H, Hkv)
    _close(got.cpu().numpy(), want, rtol=1e-5, atol=2e-6)


def test_swiglu_add(gpu, oracle):
    torch = gpu
    from simplellminference_amd import ops
    r = _rng(5)
    u = r.standard_normal(11008).astype(np.float32)
    g = (4 * r.standard_normal(11008)).astype(np.float32)
    _close(ops.swiglu(_t(torch, u), _t(torch, g)).cpu().numpy(), oracle.swiglu(u, g), rtol=2e-6, atol=1e-7)
    a = r.standard_normal(4096).astype(np.float32)
    b = r.standard_normal(4096).astype(np.float32)
    assert np.array_equal(ops.add(_t(torch, a), _t(torch, b)).cpu().numpy(), oracle.add(a, b))  # exact


@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_embedding(gpu, oracle, dtype):
    torch = gpu
    from simplellminference_amd import ops, SliError
    r = _rng(9)
    tab = r.standard_normal((512, 256)).astype(np.float32)
    if dtype == "f16":
        tab = tab.astype(np.float16)
    for tok in (0, 17, 511):
        got = ops.embedding(tok, _t(torch, tab)).cpu().numpy()
        assert np.array_equal(got, oracle.embedding(tok, tab.astype(np.float32)))
    with pytest.raises(SliError):
        ops.embedding(512, _t(torch, tab))  # emb_kernel.cpp:10 rejects out-of-range tokens
    for bad in (512, -1):  # a device token cannot be rejected before the launch: the row is poisoned (NaN)
        got = ops.embedding(torch.tensor([bad], dtype=torch.int32, device="cuda"), _t(torch, tab)).cpu().numpy()
        assert np.isnan(got).all()
    got = ops.embedding(torch.tensor([17], dtype=torch.int32, device="cuda"), _t(torch, tab)).cpu().numpy()
    assert np.array_equal(got, oracle.embedding(17, tab.astype(np.float32)))


def test_argmax_first_max(gpu, oracle):
    torch = gpu
    from simplellminference_amd import ops
    r = _rng(11)
    for n in (1, 7, 32000, 128256):
        x = r.standard_normal(n).astype(np.float32)
        assert int(ops.argmax(_t(torch, x)).item()) == oracle.argmax(x)
    x = np.zeros(1000, np.float32)
    x[[5, 17, 999]] = 3.0  # ties -> first index (std::max_element)
    assert int(ops.argmax(_t(torch, x)).item()) == 5 == oracle.argmax(x)
    x = np.full(64, -np.inf, np.float32)
    x[40] = -1e30
    assert int(ops.argmax(_t(torch, x)).item()) == 40


NAN = np.float32("nan")
SPECIAL = [
    [-0.0, 0.0],                      # -0 == +0 under `<`: the first one wins
    [0.0, -0.0],
    [-1.0, -0.0, 0.0, -0.0],
    [NAN, 1.0, 5.0],                  # NaN at index 0 is never displaced
    [1.0, NAN, 5.0, NAN],             # a NaN later never displaces the best
    [-np.inf, NAN, -np.inf],
    [NAN, NAN],
    [3.0, NAN, 3.0, np.inf, NAN, np.inf],
]


@pytest.mark.parametrize("vals", SPECIAL, ids=[str(i) for i in range(len(SPECIAL))])
def test_argmax_signed_zero_and_nan(gpu, oracle, vals):
    """std::max_element's `<` scan (argmax.cpp:11) on the values `<` does not order: bit-exact index."""
    torch = gpu
    from simplellminference_amd import ops
    x = np.array(vals, np.float32)
    want = oracle.argmax(x)
    assert int(ops.argmax(_t(torch, x)).item()) == want
    # the same values inside a long row (the LM-head shape): shifted right, padded with -inf
    y = np.full(32000, -np.inf, np.float32)
    y[1000:1000 + x.size] = x
    if x.size and np.isnan(x[0]):
        y[1000] = -np.inf  # a NaN away from index 0 loses: the oracle says the same
    assert int(ops.argmax(_t(torch, y)).item()) == oracle.argmax(y)


# ---- against the REFERENCE's own CPU build (committed vectors, tests/golden/ref_ops.npz) -------------------
# Every per-op case of tests/golden/ref_cases.py, recomputed by the HIP ops on the same regenerated inputs and
# compared with what the reference's source/kernel/cpu produced (make_ref_golden.py). Bars: fp32 reductions in
# another order within the per-family bounds below; RoPE tables, embedding rows and argmax indices bit-exact.
import os  # noqa: E402

from tests.golden import ref_cases as RC  # noqa: E402

_GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_ops.npz")


class _Hip:
    """The HIP ops behind the oracle's numpy signatures (so ref_cases can drive them)."""

    def __init__(self, torch):
        from simplellminference_amd import ops
        self.t, self.ops = torch, ops

    def _d(self, a):
        return _t(self.t, a)

    def matmul(self, x, w):
        return self.ops.matmul(self._d(x), self._d(w)).cpu().numpy()

    def rmsnorm(self, x, w, eps):
        return self.ops.rmsnorm(self._d(x), self._d(w), eps).cpu().numpy()

    def rope_cache(self, hd, T, theta):
        s, c = self.ops.rope_cache(hd, T, theta)
        return s.cpu().numpy(), c.cpu().numpy()

    def rope(self, q, k, pos, s, c, hd):
        tq, tk = self._d(q), self._d(k)
        self.ops.rope(tq, tk, pos, self._d(s), self._d(c), hd)
        return tq.cpu().numpy(), tk.cpu().numpy()

    def softmax(self, x):
        return self.ops.softmax_(self._d(x)).cpu().numpy()

    def mha(self, q, kc, vc, layer, pos, T, hd, H, Hkv):
        return self.ops.mha(self._d(q), self._d(kc), self._d(vc), layer, pos, T, hd, H, Hkv).cpu().numpy()

    def swiglu(self, up, gate):
        return self.ops.swiglu(self._d(up), self._d(gate)).cpu().numpy()

    def embedding(self, token, tab):
        return self.ops.embedding(token, self._d(tab)).cpu().numpy()

    def argmax(self, x):
        return int(self.ops.argmax(self._d(x)).item())


@pytest.mark.parametrize("name", sorted(RC.CASES))
def test_hip_ops_match_reference_build_vectors(gpu, oracle, name):
    gold = np.load(_GOLD)
    inputs, outputs = RC.CASES[name](_Hip(gpu), oracle)
    fam = name.split("_")[0]
    if fam in ("embedding", "argmax") or name.startswith("rope_cache"):
        RC.check(name, gold, inputs, outputs)  # bit-exact
        return
    for k, v in inputs.items():  # the regenerated inputs are the ones the reference saw
        assert float(np.asarray(v, np.float64).sum()) == float(gold[f"{name}/in/{k}/sum64"])
    for k, got in outputs.items():
        want = gold[f"{name}/out/{k}"]
        if fam == "matmul":
            x, w = inputs["x"], inputs["w"]
            bound = 4 * np.finfo(np.float32).eps * np.sqrt(x.size) * (np.abs(w) @ np.abs(x))
            assert np.all(np.abs(got.astype(np.float64) - want) <= bound + 1e-30), np.abs(got - want).max()
        else:
            rtol, atol = {"rmsnorm": (2e-6, 1e-7), "rope": (1e-6, 1e-6), "softmax": (1e-5, 1e-8),
                          "mha": (1e-5, 2e-6), "swiglu": (2e-6, 1e-7)}[fam]
            _close(got, want, rtol=rtol, atol=atol)
