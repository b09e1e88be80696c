"""Tensor-parallel helpers (host side): the shard plan libsli.so places weights with, and the RCCL
unique-id exchange over torch.distributed (gloo) for one-process-per-GPU launches.

The plan itself lives in C (sli_tp_plan / sli_tp_vocab, csrc/tp_plan.hip) so the GPU engine and the
CPU tests slice weights identically.
"""
from __future__ import annotations

import ctypes

from ._lib import ModelConfig, ShardWindow, call
from .model import LlamaModelConfig

KINDS = {"emb": 1, "norm": 2, "wq": 3, "wk": 4, "wv": 5, "wo": 6, "up": 7, "gate": 8, "down": 9}


def _cfg(c: LlamaModelConfig, rank: int, size: int) -> ModelConfig:
    return ModelConfig(c.vocab_size, c.hidden_size, c.num_attention_heads, c.num_key_value_heads, c.head_dim,
                       c.intermediate_size, c.num_hidden_layers, c.max_length, c.rms_norm_eps, c.rope_theta,
                       1, 1, 0, rank, size, 0)


def shard_window(c: LlamaModelConfig, kind: str, rank: int, size: int) -> ShardWindow:
    w = ShardWindow()
    call("sli_tp_plan", ctypes.byref(_cfg(c, rank, size)), KINDS[kind], ctypes.byref(w))
    return w


def vocab_shard(c: LlamaModelConfig, rank: int, size: int) -> tuple[int, int]:
    lo, n = ctypes.c_int32(), ctypes.c_int32()
    call("sli_tp_vocab", ctypes.byref(_cfg(c, rank, size)), ctypes.byref(lo), ctypes.byref(n))
    return lo.value, n.value


def take(full, w: ShardWindow):
    """The window of a full reference-layout [rows, cols] array."""
    return full[w.row_lo:w.row_lo + w.n_rows, w.col_lo:w.col_lo + w.n_cols]


def broadcast_comm_id(rank: int) -> bytes:
    """Rank 0 creates the RCCL unique id; every rank receives it over the default process group."""
    import torch.distributed as dist

    from .model import comm_id
    box = [comm_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def open_oneshot(model) -> None:
    """Exchange every rank's one-shot all-reduce buffer handle over the default process group (gloo) and
    map the peers' buffers (sli_model_comm_open); the model then still all-reduces over RCCL until
    set_allreduce("oneshot")."""
    import torch.distributed as dist
    mine = model.comm_handle()
    allh = [None] * dist.get_world_size()
    dist.all_gather_object(allh, mine)
    model.comm_open(allh)
