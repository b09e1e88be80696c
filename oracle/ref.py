"""The REFERENCE's own CPU path, built in place — TEST INFRASTRUCTURE ONLY.

ctypes bindings for ``oracle/_ref/libref.so``: ``make -C oracle ref`` compiles the reference's
``source/kernel/cpu``, ``source/memory``, ``source/op`` (minus add/encode) and ``weight_loader.cpp`` straight
from ``/root/reference`` together with ``oracle/ref_harness.cpp`` (our plain-pointer wrapper, plus the
restated model.cpp op wiring). It pins ``sli_oracle.c`` (tests/golden/make_ref_golden.py writes the
committed ``tests/golden/ref_*.npz`` from it) and calibrates the CPU baseline. ``/root/reference`` does
not exist on the GPU box: everything here is optional there (``available()`` is False), and nothing in
the product package imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REF_ROOT = os.environ.get("SLI_REFERENCE", "/root/reference")
LIB_PATH = os.environ.get("SLI_REF_LIB") or os.path.join(_HERE, "_ref", "libref.so")  # (asan_check.sh: _ref/asan/)
_lib = None

F32P = ctypes.POINTER(ctypes.c_float)
I32P = ctypes.POINTER(ctypes.c_int)


def source_present() -> bool:
    return os.path.isfile(os.path.join(REF_ROOT, "source", "kernel", "cpu", "matmul_kernel.cpp"))


def build(force: bool = False) -> str | None:
    """Build _ref/libref.so from the reference sources (only where /root/reference exists)."""
    if not source_present():
        return LIB_PATH if os.path.exists(LIB_PATH) else None
    subprocess.run(["make", "-s", "-C", _HERE, "ref", f"REF={REF_ROOT}"] + (["-B"] if force else []), check=True)
    return LIB_PATH


def available() -> bool:
    return os.path.exists(LIB_PATH) or source_present()


def lib():
    global _lib
    if _lib is None:
        if build() is None:
            raise RuntimeError("reference CPU build unavailable (no /root/reference and no oracle/_ref/libref.so)")
        # RTLD_LAZY: alloc.cpp's cuda* calls and the ops' kernel::*_cuda branches stay unresolved (never reached)
        L = ctypes.CDLL(LIB_PATH, mode=os.RTLD_LAZY | os.RTLD_LOCAL)
        L.ref_matmul.argtypes = [F32P, F32P, F32P, ctypes.c_int, ctypes.c_int, ctypes.c_float]
        L.ref_rmsnorm.argtypes = [F32P, F32P, F32P, ctypes.c_int, ctypes.c_float]
        L.ref_rope_cache.argtypes = [ctypes.c_int, ctypes.c_int, F32P, F32P, ctypes.c_float]
        L.ref_rope.argtypes = [F32P, F32P, ctypes.c_int, F32P, F32P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ref_softmax.argtypes = [F32P, ctypes.c_int]
        L.ref_mha.argtypes = [F32P, F32P, F32P, F32P, F32P] + [ctypes.c_int] * 7
        L.ref_swiglu.argtypes = [F32P, F32P, F32P, ctypes.c_int]
        L.ref_embedding.argtypes = [ctypes.c_int, F32P, F32P, ctypes.c_int, ctypes.c_int]
        L.ref_argmax.argtypes = [F32P, ctypes.c_int]
        L.ref_argmax.restype = ctypes.c_int
        L.ref_model_create.argtypes = [ctypes.c_int] * 8 + [ctypes.c_float, ctypes.c_float, ctypes.c_char_p]
        L.ref_model_create.restype = ctypes.c_void_p
        L.ref_model_create_mem.argtypes = [ctypes.c_int] * 8 + [ctypes.c_float, ctypes.c_float, F32P, ctypes.c_size_t]
        L.ref_model_create_mem.restype = ctypes.c_void_p
        L.ref_model_free.argtypes = [ctypes.c_void_p]
        L.ref_model_kv.argtypes = [ctypes.c_void_p, ctypes.POINTER(F32P), ctypes.POINTER(F32P)]
        L.ref_model_last_timing.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_double)] * 3
        L.ref_model_forward.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, F32P]
        L.ref_model_predict.argtypes = [ctypes.c_void_p, I32P, ctypes.c_int, ctypes.c_int, I32P, F32P]
        L.ref_model_predict.restype = ctypes.c_int
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(F32P)


def _c(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def matmul(x, w, scale=1.0):
    x, w = _c(x), _c(w)
    y = np.empty(w.shape[0], np.float32)
    lib().ref_matmul(_f(x), _f(w), _f(y), w.shape[0], w.shape[1], scale)
    return y


def rmsnorm(x, w, eps):
    x, w = _c(x), _c(w)
    y = np.empty_like(x)
    lib().ref_rmsnorm(_f(x), _f(w), _f(y), x.size, eps)
    return y


def rope_cache(head_dim, max_len, theta):
    s = np.empty((max_len, head_dim // 2), np.float32)
    c = np.empty_like(s)
    lib().ref_rope_cache(head_dim, max_len, _f(s), _f(c), theta)
    return s, c


def rope(q, k, pos, sin_c, cos_c, head_dim):
    """rope_kernel.cpp:22-41 rotates k over len(q) floats: k is padded to len(q) here and the first
    len(k) values are returned (the rest is the reference's out-of-range write)."""
    q = _c(q).copy()
    kk = np.zeros(q.size, np.float32)
    kk[:k.size] = k
    sin_c, cos_c = _c(sin_c), _c(cos_c)
    lib().ref_rope(_f(q), _f(kk), pos, _f(sin_c), _f(cos_c), q.size, head_dim, sin_c.shape[0])
    return q, kk[:k.size].copy()


def softmax(x):
    x = _c(x).copy()
    lib().ref_softmax(_f(x), x.size)
    return x


def mha(q, kcache, vcache, layer, pos, max_len, head_dim, n_heads, n_kv_heads):
    """kcache/vcache [L][T][KV] fp32 (model.cpp:264-265)."""
    q, kc, vc = _c(q), _c(kcache), _c(vcache)
    score = np.zeros((n_heads, max_len), np.float32)
    out = np.empty(n_heads * head_dim, np.float32)
    lib().ref_mha(_f(q), _f(score), _f(kc), _f(vc), _f(out), layer, pos, max_len, head_dim, n_heads, n_kv_heads,
                  kc.shape[0])
    return out


def swiglu(up, gate):
    up, gate = _c(up), _c(gate)
    out = np.empty_like(up)
    lib().ref_swiglu(_f(up), _f(gate), _f(out), up.size)
    return out


def embedding(token, table):
    table = _c(table)
    if not 0 <= token <= table.shape[0]:
        raise ValueError("the reference exits on token > vocab (emb_kernel.cpp:10)")
    out = np.empty(table.shape[1], np.float32)
    lib().ref_embedding(token, _f(table), _f(out), table.shape[0], table.shape[1])
    return out


def argmax(logits):
    logits = _c(logits)
    return int(lib().ref_argmax(_f(logits), logits.size))


class Model:
    """LlamaModel over the reference's op layers, weights from the reference's flat fp32 file
    (the oracle writes it: oracle.Model.write_flat)."""

    def __init__(self, cfg, flat_path: str | None = None, flat: np.ndarray | None = None):
        """flat_path: the reference's flat fp32 weight file; or flat: the same image in memory (kept alive)."""
        self.cfg = cfg
        self._flat = None
        if flat is not None:
            self._flat = np.ascontiguousarray(flat, np.float32)
            self._h = lib().ref_model_create_mem(cfg.vocab, cfg.dim, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim,
                                                 cfg.ffn, cfg.n_layers, cfg.max_len, cfg.eps, cfg.theta,
                                                 _f(self._flat), self._flat.size)
        else:
            self._h = lib().ref_model_create(cfg.vocab, cfg.dim, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim,
                                             cfg.ffn, cfg.n_layers, cfg.max_len, cfg.eps, cfg.theta,
                                             flat_path.encode())
        if not self._h:
            raise RuntimeError(f"ref_model_create failed ({flat_path or 'in-memory image'})")

    def kv_cache(self):
        """(K, V) caches as [L][T][KV] fp32 views of the model's own buffers."""
        k, v = F32P(), F32P()
        lib().ref_model_kv(self._h, ctypes.byref(k), ctypes.byref(v))
        c = self.cfg
        shape = (c.n_layers, c.max_len, c.n_kv_heads * c.head_dim)
        n = int(np.prod(shape))
        return (np.ctypeslib.as_array(k, (n,)).reshape(shape), np.ctypeslib.as_array(v, (n,)).reshape(shape))

    def last_timing(self):
        e, l, h = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        lib().ref_model_last_timing(self._h, ctypes.byref(e), ctypes.byref(l), ctypes.byref(h))
        return e.value, l.value, h.value

    def close(self):
        if self._h:
            lib().ref_model_free(self._h)
            self._h = None
        self._flat = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def forward(self, token: int, pos: int) -> np.ndarray:
        out = np.empty(self.cfg.vocab, np.float32)
        lib().ref_model_forward(self._h, token, pos, _f(out))
        return out

    def predict(self, prompt, max_length: int):
        p = np.ascontiguousarray(prompt, dtype=np.int32)
        toks = np.empty(max_length, np.int32)
        logits = np.empty((max_length, self.cfg.vocab), np.float32)
        lib().ref_model_predict(self._h, p.ctypes.data_as(I32P), p.size, max_length, toks.ctypes.data_as(I32P),
                                _f(logits))
        return toks, logits
