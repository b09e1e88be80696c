"""Kernel-level operators over device tensors — the Python mirror of the reference's
``kernel::*_cuda`` launchers (include/kernel/cuda/*.cuh), each a thin call into libsli.so.

Tensors are torch tensors on the HIP device (PyTorch here is only the device-memory and stream
plumbing); every function launches on ``torch.cuda.current_stream()``.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import DT_F16, DT_F32, DT_I8, call

_DT = {torch.float32: DT_F32, torch.float16: DT_F16, torch.int8: DT_I8}


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dev(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or not t.is_contiguous()):
            raise ValueError("operands must be contiguous device tensors")


def matmul(x, w, y=None, scale: float = 1.0, row_scale=None):
    """matmul_kernel_cuda (matmul_kernel.cuh:6-7): y = scale * W @ x, W [rows, cols] f32/f16/int8."""
    rows, cols = w.shape
    if x.numel() != cols:
        raise ValueError("Tensor with Wrong Dim!")  # matmul_kernel.cpp:8
    y = torch.empty(rows, device=x.device, dtype=torch.float32) if y is None else y
    _dev(x, w, y, row_scale)
    call("sli_matmul", _p(x), _p(w), _DT[w.dtype], _p(row_scale), _p(y), rows, cols, scale, _s())
    return y


def matmul_batch(x, w, y=None):
    """Batched projection for B <= 8 sequences on MFMA (bgemm.h): y[b] = W @ x[b]; x [B, cols] fp32, W
    [rows, cols] fp16, y [B, rows] fp32. No reference counterpart (the reference is batch 1)."""
    batch, cols = x.shape
    rows = w.shape[0]
    if w.shape[1] != cols:
        raise ValueError("Tensor with Wrong Dim!")
    y = torch.empty(batch, rows, device=x.device, dtype=torch.float32) if y is None else y
    nbytes = _lib.load().sli_matmul_batch_workspace_bytes(rows, cols, batch)
    if nbytes == 0:
        raise ValueError("unsupported batched shape (cols % 32 != 0 or batch > 8)")
    ws = torch.empty(nbytes // 4 + 1, device=x.device, dtype=torch.float32)
    _dev(x, w, y, ws)
    call("sli_matmul_batch", _p(x), _p(w), _DT[w.dtype], _p(y), rows, cols, batch, _p(ws), ws.numel() * 4, _s())
    return y


def rmsnorm(x, w, eps: float, y=None):
    """rmsnorm_kernel_cuda (rms_kernel.cuh:6-7)."""
    y = torch.empty_like(x) if y is None else y
    _dev(x, w, y)
    call("sli_rmsnorm", _p(x), _p(w), _p(y), x.numel(), eps, _s())
    return y


def rope_cache(head_dim: int, max_len: int, theta: float, device="cuda"):
    """rope_cache_cal_cuda (rope_kernel.cuh:5-6): (sin, cos) tables [max_len, head_dim/2]."""
    s = torch.empty(max_len, head_dim // 2, device=device, dtype=torch.float32)
    c = torch.empty_like(s)
    call("sli_rope_cache", head_dim, max_len, _p(s), _p(c), theta, _s())
    return s, c


def rope(q, k, pos, sin_c, cos_c, head_dim: int):
    """rope_kernel_cuda (rope_kernel.cuh:7-8), in place on q and k. pos: int or int32 device tensor."""
    _dev(q, k, sin_c, cos_c)
    pos_dev = pos if isinstance(pos, torch.Tensor) else None
    call("sli_rope", _p(q), _p(k), 0 if pos_dev is not None else int(pos), _p(pos_dev), _p(sin_c), _p(cos_c),
         q.numel(), k.numel(), head_dim, _s())
    return q, k


def mha(q, kcache, vcache, layer: int, pos: int, max_len: int, head_dim: int, n_heads: int, n_kv_heads: int,
        out=None, workspace=None):
    """mha_kernel_cuda (mha_kernel.cuh:6-21) over a reference-layout [L, T, KV] cache (f32 or f16)."""
    out = torch.empty(n_heads * head_dim, device=q.device, dtype=torch.float32) if out is None else out
    nbytes = _lib.load().sli_mha_workspace_bytes(max_len, n_heads, head_dim)
    if workspace is None:
        workspace = torch.empty(max(nbytes // 4, 1), device=q.device, dtype=torch.float32)
    _dev(q, kcache, vcache, out, workspace)
    call("sli_mha", _p(q), _p(kcache), _p(vcache), _DT[kcache.dtype], _p(out), layer, pos, max_len, head_dim,
         n_heads, n_kv_heads, _p(workspace), workspace.numel() * 4, _s())
    return out


def softmax_(x):
    """softmax_kernel_cpu semantics (mha_kernel.cpp:7-20), in place."""
    _dev(x)
    call("sli_softmax", _p(x), x.numel(), _s())
    return x


def swiglu(up, gate, out=None):
    """swiglu_kernel_cuda (swiglu_kernel.cuh:5): sigmoid(gate) * up."""
    out = torch.empty_like(up) if out is None else out
    _dev(up, gate, out)
    call("sli_swiglu", _p(up), _p(gate), _p(out), up.numel(), _s())
    return out


def add(a, b, out=None):
    """add_kernel_cuda (add_kernel.cuh:6)."""
    out = torch.empty_like(a) if out is None else out
    _dev(a, b, out)
    call("sli_add", _p(a), _p(b), _p(out), a.numel(), _s())
    return out


def embedding(token, table, out=None, row_scale=None):
    """emb_kernel_cuda (emb_kernel.cuh:6-7). token: int or int32 device tensor."""
    vocab, dim = table.shape
    out = torch.empty(dim, device=table.device, dtype=torch.float32) if out is None else out
    tok_dev = token if isinstance(token, torch.Tensor) else None
    _dev(table, out, row_scale)
    call("sli_embedding", 0 if tok_dev is not None else int(token), _p(tok_dev), _p(table), _DT[table.dtype],
         _p(row_scale), _p(out), vocab, dim, _s())
    return out


def argmax(logits, out=None):
    """argmaxLayer::forward (argmax.cpp:7-17) on device: first index of the maximum."""
    out = torch.empty(1, device=logits.device, dtype=torch.int32) if out is None else out
    _dev(logits, out)
    call("sli_argmax", _p(logits), logits.numel(), _p(out), _s())
    return out
