"""CPU oracle — TEST INFRASTRUCTURE ONLY.

ctypes bindings for ``liboracle.so`` (the C restatement of the reference CPU path, sli_oracle.c).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module, as the checker or the timed CPU baseline; the product package never does.

Parity status: "parity unpinned" (see sli_oracle.h and DESIGN.md §2).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SLI_ORACLE_LIB: an alternative build of the same source (tools/asan_check.sh: the ASan/UBSan build, _ref/asan/)
_LIB_PATH = os.environ.get("SLI_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
_lib = None

F32P = ctypes.POINTER(ctypes.c_float)
I32P = ctypes.POINTER(ctypes.c_int)

# tensor kinds, mirror include/sli_synth.h
T_EMB, T_NORM, T_WQ, T_WK, T_WV, T_WO, T_UP, T_GATE, T_DOWN = 1, 2, 3, 4, 5, 6, 7, 8, 9
W_F32, W_F16, W_I8 = 0, 1, 2


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    if os.environ.get("SLI_ORACLE_LIB"):
        return _LIB_PATH
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE] + (["-B"] if force else []), check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_matmul.argtypes = [F32P, F32P, F32P, ctypes.c_int, ctypes.c_int, ctypes.c_float]
        L.orc_rmsnorm.argtypes = [F32P, F32P, F32P, ctypes.c_int, ctypes.c_float]
        L.orc_rope_cache.argtypes = [ctypes.c_int, ctypes.c_int, F32P, F32P, ctypes.c_float]
        L.orc_rope.argtypes = [F32P, F32P, ctypes.c_int, F32P, F32P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_softmax.argtypes = [F32P, ctypes.c_int]
        L.orc_mha.argtypes = [F32P, F32P, F32P, F32P, F32P] + [ctypes.c_int] * 6
        L.orc_swiglu.argtypes = [F32P, F32P, F32P, ctypes.c_int]
        L.orc_add.argtypes = [F32P, F32P, F32P, ctypes.c_int]
        L.orc_embedding.argtypes = [ctypes.c_int, F32P, F32P, ctypes.c_int, ctypes.c_int]
        L.orc_embedding.restype = ctypes.c_int
        L.orc_argmax.argtypes = [F32P, ctypes.c_int]
        L.orc_argmax.restype = ctypes.c_int
        L.orc_f32_to_f16_bits.argtypes = [ctypes.c_float]
        L.orc_f32_to_f16_bits.restype = ctypes.c_uint16
        L.orc_round_f16.argtypes = [ctypes.c_float]
        L.orc_round_f16.restype = ctypes.c_float
        L.orc_quant_row_i8.argtypes = [F32P, ctypes.c_int, ctypes.POINTER(ctypes.c_int8), F32P]
        L.orc_synth_fill.argtypes = [F32P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float,
                                     ctypes.c_float]
        L.orc_model_create.argtypes = [ctypes.c_void_p]
        L.orc_model_create.restype = ctypes.c_void_p
        L.orc_model_create_lazy.argtypes = [ctypes.c_void_p]
        L.orc_model_create_lazy.restype = ctypes.c_void_p
        L.orc_model_free.argtypes = [ctypes.c_void_p]
        L.orc_model_init_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
        L.orc_model_weight.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.orc_model_weight.restype = F32P
        L.orc_model_set_kv_f16.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_model_kcache.argtypes = [ctypes.c_void_p]
        L.orc_model_kcache.restype = F32P
        L.orc_model_vcache.argtypes = [ctypes.c_void_p]
        L.orc_model_vcache.restype = F32P
        L.orc_model_fill_kv_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
        L.orc_model_forward.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, F32P]
        L.orc_model_forward.restype = ctypes.c_int
        L.orc_model_predict.argtypes = [ctypes.c_void_p, I32P, ctypes.c_int, ctypes.c_int, I32P, F32P]
        L.orc_model_predict.restype = ctypes.c_int
        L.orc_model_last_timing.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_double)] * 3
        L.orc_model_set_threads.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_model_write_flat.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.orc_model_write_flat.restype = ctypes.c_int
        _lib = L
    return _lib


def _f(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(F32P)


def _i(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(I32P)


# ------------------------------------------------------------------ per-op wrappers (numpy in / out)
def matmul(x, w, scale=1.0):
    rows, cols = w.shape
    y = np.empty(rows, np.float32)
    lib().orc_matmul(_f(x), _f(w), _f(y), rows, cols, scale)
    return y


def rmsnorm(x, w, eps):
    y = np.empty_like(x)
    lib().orc_rmsnorm(_f(x), _f(w), _f(y), x.size, eps)
    return y


def rope_cache(head_dim, max_len, theta):
    s = np.empty((max_len, head_dim // 2), np.float32)
    c = np.empty_like(s)
    lib().orc_rope_cache(head_dim, max_len, _f(s), _f(c), theta)
    return s, c


def rope(q, k, pos, sin_c, cos_c, head_dim):
    q = q.copy()
    k = k.copy()
    lib().orc_rope(_f(q), _f(k), pos, _f(sin_c), _f(cos_c), q.size, k.size, head_dim)
    return q, k


def softmax(x):
    x = x.copy()
    lib().orc_softmax(_f(x), x.size)
    return x


def mha(q, kcache, vcache, layer, pos, max_len, head_dim, n_heads, n_kv_heads):
    """kcache/vcache in reference layout [L][T][KV]."""
    score = np.zeros((n_heads, max_len), np.float32)
    out = np.empty(n_heads * head_dim, np.float32)
    lib().orc_mha(_f(q), _f(score), _f(kcache), _f(vcache), _f(out), layer, pos, max_len, head_dim, n_heads,
                  n_kv_heads)
    return out


def swiglu(up, gate):
    out = np.empty_like(up)
    lib().orc_swiglu(_f(up), _f(gate), _f(out), up.size)
    return out


def add(a, b):
    out = np.empty_like(a)
    lib().orc_add(_f(a), _f(b), _f(out), a.size)
    return out


def embedding(token, table):
    vocab, dim = table.shape
    out = np.empty(dim, np.float32)
    rc = lib().orc_embedding(int(token), _f(table), _f(out), vocab, dim)
    if rc != 0:
        raise IndexError(f"token {token} out of range for vocab {vocab}")
    return out


def argmax(logits):
    return int(lib().orc_argmax(_f(logits), logits.size))


def round_f16(a: np.ndarray) -> np.ndarray:
    return np.array([lib().orc_round_f16(float(v)) for v in a.ravel()], np.float32).reshape(a.shape)


def f16_bits(v: float) -> int:
    return int(lib().orc_f32_to_f16_bits(v))


def quant_row_i8(row):
    q = np.empty(row.size, np.int8)
    s = ctypes.c_float()
    lib().orc_quant_row_i8(_f(row), row.size, q.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)), ctypes.byref(s))
    return q, s.value


def synth_fill(n, seed, stream, c, offset=0.0):
    out = np.empty(n, np.float32)
    lib().orc_synth_fill(_f(out), n, seed, stream, c, offset)
    return out


def synth_c(std: float) -> float:
    """SLI_SYNTH_C(std) from include/sli_synth.h (double -> float)."""
    return float(np.float32(std * 1.7320508075688772 / 65536.0))


def stream_id(kind: int, index: int) -> int:
    return (kind << 16) | (index & 0xFFFF)


# ------------------------------------------------------------------ model
@dataclass
class Config:
    vocab: int
    dim: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    ffn: int
    n_layers: int
    max_len: int
    eps: float = 1e-5
    theta: float = 10000.0


class _CConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("vocab", "dim", "n_heads", "n_kv_heads", "head_dim", "ffn", "n_layers", "max_len")] + \
               [("eps", ctypes.c_float), ("theta", ctypes.c_float)]


class Model:
    """LlamaModel restatement (model.cpp:40-187) with synthetic weights (sli_synth.h)."""

    def __init__(self, cfg: Config, seed: int = 0, wmode: int = W_F32, kv_f16: bool = False, lazy: bool = False):
        """lazy: hold one layer of weights and regenerate each layer inside forward (full-size models such as
        the 32-layer Llama-2-7B step; weight() then serves only the embedding and norms)."""
        self.cfg = cfg
        c = _CConfig(cfg.vocab, cfg.dim, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.ffn, cfg.n_layers,
                     cfg.max_len, cfg.eps, cfg.theta)
        self._h = (lib().orc_model_create_lazy if lazy else lib().orc_model_create)(ctypes.byref(c))
        lib().orc_model_init_synthetic(self._h, seed, wmode)
        lib().orc_model_set_kv_f16(self._h, 1 if kv_f16 else 0)

    def close(self):
        if self._h:
            lib().orc_model_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def weight(self, kind: int, index: int = 0) -> np.ndarray:
        c = self.cfg
        kv = c.n_kv_heads * c.head_dim
        shapes = {T_EMB: (c.vocab, c.dim), T_NORM: (c.dim,), T_WQ: (c.dim, c.dim), T_WK: (kv, c.dim),
                  T_WV: (kv, c.dim), T_WO: (c.dim, c.dim), T_UP: (c.ffn, c.dim), T_GATE: (c.ffn, c.dim),
                  T_DOWN: (c.dim, c.ffn)}
        shp = shapes[kind]
        p = lib().orc_model_weight(self._h, kind, index)
        return np.ctypeslib.as_array(p, shape=shp)

    def kv_cache(self):
        c = self.cfg
        shp = (c.n_layers, c.max_len, c.n_kv_heads * c.head_dim)
        k = np.ctypeslib.as_array(lib().orc_model_kcache(self._h), shape=shp)
        v = np.ctypeslib.as_array(lib().orc_model_vcache(self._h), shape=shp)
        return k, v

    def fill_kv_synthetic(self, seed: int, upto: int):
        lib().orc_model_fill_kv_synthetic(self._h, seed, upto)

    def forward(self, token: int, pos: int) -> np.ndarray:
        out = np.empty(self.cfg.vocab, np.float32)
        rc = lib().orc_model_forward(self._h, int(token), int(pos), _f(out))
        if rc != 0:
            raise RuntimeError(f"orc_model_forward rc={rc}")
        return out

    def predict(self, prompt, max_length: int, want_logits: bool = True):
        prompt = np.ascontiguousarray(prompt, np.int32)
        toks = np.empty(max_length, np.int32)
        logits = np.empty((max_length, self.cfg.vocab), np.float32) if want_logits else None
        rc = lib().orc_model_predict(self._h, _i(prompt), prompt.size, max_length, _i(toks),
                                     _f(logits) if want_logits else None)
        if rc != max_length:
            raise RuntimeError(f"orc_model_predict rc={rc}")
        return toks, logits

    def last_timing(self):
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        lib().orc_model_last_timing(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def set_threads(self, n: int):
        """GEMV rows over n host threads (bit-identical; the all-cores CPU line, not the reference)."""
        lib().orc_model_set_threads(self._h, n)

    def flat_image(self) -> np.ndarray:
        """The reference's flat fp32 weight image (model.cpp:336-469 order) in memory."""
        c = self.cfg
        parts = [self.weight(T_EMB).ravel()] + [self.weight(T_NORM, i) for i in range(2 * c.n_layers + 1)]
        for kind in (T_WQ, T_WK, T_WV, T_WO, T_UP, T_GATE, T_DOWN):
            parts += [self.weight(kind, l).ravel() for l in range(c.n_layers)]
        return np.concatenate(parts)

    def write_flat(self, path: str):
        if lib().orc_model_write_flat(self._h, path.encode()) != 0:
            raise OSError(f"cannot write {path}")
