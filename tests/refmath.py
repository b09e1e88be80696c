"""Independent float64 numpy restatement of the reference decode step.

Used only to cross-check the C oracle (oracle/sli_oracle.c): two restatements written separately —
one fp32-sequential in C, one float64-vectorised here — must agree to fp32 rounding error. The
reference itself cannot be built in this image, so this is the strongest check
available on the oracle's algorithm. Citations are /root/reference paths.
"""
from __future__ import annotations

import numpy as np


def rmsnorm(x, w, eps):  # source/kernel/cpu/rms_kernel.cpp:5-23
    x = x.astype(np.float64)
    return x / np.sqrt(np.mean(x * x) + eps) * w


def rope_tables(head_dim, max_len, theta):  # source/kernel/cpu/rope_kernel.cpp:4-19 (float32 table)
    d = np.arange(head_dim // 2, dtype=np.float32)
    freq = np.float32(1.0) / np.power(np.float32(theta), (2 * d).astype(np.float32) / np.float32(head_dim))
    t = np.arange(max_len, dtype=np.float32)[:, None]
    val = (freq[None, :] * t).astype(np.float32)
    return np.sin(val.astype(np.float64)), np.cos(val.astype(np.float64))


def rope(v, pos, sin_t, cos_t, head_dim):  # rope_kernel.cpp:22-41, rotate-half per head block
    v = v.astype(np.float64).reshape(-1, head_dim).copy()
    h = head_dim // 2
    s, c = sin_t[pos], cos_t[pos]
    v0, v1 = v[:, :h].copy(), v[:, h:].copy()
    v[:, :h] = v0 * c - v1 * s
    v[:, h:] = v1 * c + v0 * s
    return v.ravel()


def mha(q, kc, vc, pos, head_dim, n_heads, n_kv_heads):  # mha_kernel.cpp:36-77
    g = n_heads // n_kv_heads
    out = np.empty(n_heads * head_dim)
    for h in range(n_heads):
        kv = h // g
        K = kc[: pos + 1, kv * head_dim:(kv + 1) * head_dim].astype(np.float64)
        V = vc[: pos + 1, kv * head_dim:(kv + 1) * head_dim].astype(np.float64)
        s = K @ q[h * head_dim:(h + 1) * head_dim] / np.sqrt(head_dim)
        p = np.exp(s - s.max())
        p /= p.sum()
        out[h * head_dim:(h + 1) * head_dim] = p @ V
    return out


def swiglu(u, g):  # swiglu_kernel.cpp:5-15 — sigmoid(gate) * up (reference variant)
    return u / (1.0 + np.exp(-g))


class Model64:
    """model.cpp:40-140 in float64 on the given (fp32) weights; optional fp16 K/V rounding."""

    def __init__(self, cfg, weights, kv_f16=False):
        self.c = cfg
        self.w = weights  # dict: emb, norm[list], wq[list] ...
        kv = cfg.n_kv_heads * cfg.head_dim
        self.kc = np.zeros((cfg.n_layers, cfg.max_len, kv))
        self.vc = np.zeros((cfg.n_layers, cfg.max_len, kv))
        self.sin, self.cos = rope_tables(cfg.head_dim, cfg.max_len, cfg.theta)
        self.kv_f16 = kv_f16

    def forward(self, token, pos):
        c, w = self.c, self.w
        x = w["emb"][token].astype(np.float64)
        for l in range(c.n_layers):
            h = rmsnorm(x, w["norm"][2 * l], c.eps)
            q = w["wq"][l] @ h
            k = w["wk"][l] @ h
            v = w["wv"][l] @ h
            q = rope(q, pos, self.sin, self.cos, c.head_dim)
            k = rope(k, pos, self.sin, self.cos, c.head_dim)
            if self.kv_f16:
                k = k.astype(np.float16).astype(np.float64)
                v = v.astype(np.float16).astype(np.float64)
            self.kc[l, pos] = k
            self.vc[l, pos] = v
            a = mha(q, self.kc[l], self.vc[l], pos, c.head_dim, c.n_heads, c.n_kv_heads)
            x1 = x + w["wo"][l] @ a
            h = rmsnorm(x1, w["norm"][2 * l + 1], c.eps)
            act = swiglu(w["up"][l] @ h, w["gate"][l] @ h)
            x = x1 + w["down"][l] @ act
        h = rmsnorm(x, w["norm"][2 * c.n_layers], c.eps)
        return w["emb"] @ h
