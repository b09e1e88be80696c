"""ctypes bindings for libsli.so — the C ABI declared in include/sli.h.

The product path has no fallback: if the HIP library is missing or fails to load, every call raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SLI_LIB_VARIANT=<name> loads libsli_<name>.so from the same directory (A/B experiments in tools/ only)
LIB_PATH = os.path.join(_HERE, "libsli.so" if not os.environ.get("SLI_LIB_VARIANT")
                        else f"libsli_{os.environ['SLI_LIB_VARIANT']}.so")

SLI_OK = 0
STATUS = {0: "ok", 1: "invalid argument", 2: "shape mismatch", 3: "index out of range", 4: "HIP runtime error",
          5: "out of device memory", 6: "RCCL error", 7: "invalid state", 8: "communicator wait timed out"}
SLI_ERR_COMM, SLI_ERR_TIMEOUT = 6, 8
DT_F32, DT_F16, DT_I8 = 0, 1, 2

c_int, c_i32, c_u32, c_i64, c_f, c_d, c_vp, c_sz = (ctypes.c_int, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64,
                                                    ctypes.c_float, ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t)
P_f = ctypes.POINTER(ctypes.c_float)
P_i32 = ctypes.POINTER(ctypes.c_int32)
P_d = ctypes.POINTER(ctypes.c_double)


class SliError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str):
        super().__init__(f"{where}: {STATUS.get(code, code)} ({detail})")
        self.code = code


class ModelConfig(ctypes.Structure):
    _fields_ = [(n, c_i32) for n in ("vocab", "dim", "n_heads", "n_kv_heads", "head_dim", "ffn", "n_layers",
                                     "max_len")] + \
               [("eps", c_f), ("theta", c_f)] + \
               [(n, c_i32) for n in ("w_dtype", "kv_dtype", "act_mode", "tp_rank", "tp_size", "device", "batch")]


class ShardWindow(ctypes.Structure):
    _fields_ = [(n, c_i32) for n in ("row_lo", "n_rows", "col_lo", "n_cols", "full_cols", "dst_row_off")]


# name -> (restype, argtypes)
_SIGS = {
    "sli_version": (c_int, []),
    "sli_status_str": (ctypes.c_char_p, [c_int]),
    "sli_last_error": (ctypes.c_char_p, []),
    "sli_device_count": (c_int, [ctypes.POINTER(c_int)]),
    "sli_set_device": (c_int, [c_int]),
    "sli_malloc": (c_int, [ctypes.POINTER(c_vp), c_sz]),
    "sli_free": (c_int, [c_vp]),
    "sli_memset": (c_int, [c_vp, c_int, c_sz, c_vp]),
    "sli_memcpy_h2d": (c_int, [c_vp, c_vp, c_sz, c_vp]),
    "sli_memcpy_d2h": (c_int, [c_vp, c_vp, c_sz, c_vp]),
    "sli_memcpy_d2d": (c_int, [c_vp, c_vp, c_sz, c_vp]),
    "sli_stream_create": (c_int, [ctypes.POINTER(c_vp)]),
    "sli_stream_destroy": (c_int, [c_vp]),
    "sli_stream_sync": (c_int, [c_vp]),
    "sli_matmul": (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_i32, c_i32, c_f, c_vp]),
    "sli_matmul_batch_workspace_bytes": (c_sz, [c_i32, c_i32, c_i32]),
    "sli_matmul_batch": (c_int, [c_vp, c_vp, c_int, c_vp, c_i32, c_i32, c_i32, c_vp, c_sz, c_vp]),
    "sli_rmsnorm": (c_int, [c_vp, c_vp, c_vp, c_i32, c_f, c_vp]),
    "sli_rope_cache": (c_int, [c_i32, c_i32, c_vp, c_vp, c_f, c_vp]),
    "sli_rope": (c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp]),
    "sli_mha_workspace_bytes": (c_sz, [c_i32, c_i32, c_i32]),
    "sli_mha": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_sz, c_vp]),
    "sli_softmax": (c_int, [c_vp, c_i32, c_vp]),
    "sli_swiglu": (c_int, [c_vp, c_vp, c_vp, c_i32, c_vp]),
    "sli_add": (c_int, [c_vp, c_vp, c_vp, c_i32, c_vp]),
    "sli_embedding": (c_int, [c_i32, c_vp, c_vp, c_int, c_vp, c_vp, c_i32, c_i32, c_vp]),
    "sli_argmax": (c_int, [c_vp, c_i32, c_vp, c_vp]),
    "sli_tp_plan": (c_int, [ctypes.POINTER(ModelConfig), c_i32, ctypes.POINTER(ShardWindow)]),
    "sli_tp_vocab": (c_int, [ctypes.POINTER(ModelConfig), P_i32, P_i32]),
    "sli_comm_id_bytes": (c_int, []),
    "sli_comm_get_id": (c_int, [c_vp]),
    "sli_model_create": (c_int, [ctypes.POINTER(ModelConfig), c_vp, ctypes.POINTER(c_vp)]),
    "sli_model_destroy": (c_int, [c_vp]),
    "sli_model_init_synthetic": (c_int, [c_vp, c_u32]),
    "sli_model_set_weight": (c_int, [c_vp, c_i32, c_i32, c_vp, c_i64]),
    "sli_model_load_flat": (c_int, [c_vp, ctypes.c_char_p]),
    "sli_model_reset": (c_int, [c_vp]),
    "sli_model_fill_kv_synthetic": (c_int, [c_vp, c_u32, c_i32]),
    "sli_model_set_state": (c_int, [c_vp, c_i32, c_i32, c_i32]),
    "sli_model_set_prompt": (c_int, [c_vp, c_vp, c_i32]),
    "sli_model_get_state": (c_int, [c_vp, P_i32, P_i32, P_i32, P_i32]),
    "sli_model_set_state_seq": (c_int, [c_vp, c_i32, c_i32, c_i32, c_i32]),
    "sli_model_set_prompt_seq": (c_int, [c_vp, c_i32, c_vp, c_i32]),
    "sli_model_get_state_seq": (c_int, [c_vp, c_i32, P_i32, P_i32, P_i32, P_i32]),
    "sli_model_prefill": (c_int, [c_vp, c_vp, c_i32]),
    "sli_model_predict_prefill": (c_int, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "sli_model_prefill_path": (c_int, [c_vp]),
    "sli_model_fused_qkv_attn": (c_int, [c_vp]),
    "sli_model_get_history": (c_int, [c_vp, c_i32, c_i32, c_vp]),
    "sli_model_set_exec": (c_int, [c_vp, c_i32]),
    "sli_model_get_exec": (c_int, [c_vp, P_i32]),
    "sli_model_step": (c_int, [c_vp]),
    "sli_model_sync": (c_int, [c_vp]),
    "sli_model_get_logits": (c_int, [c_vp, c_vp, c_i32, P_i32]),
    "sli_model_predict": (c_int, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "sli_model_predict_batch": (c_int, [c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "sli_model_get_kv": (c_int, [c_vp, c_i32, c_i32, c_i32, c_vp]),
    "sli_model_get_kv_seq": (c_int, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp]),
    "sli_model_get_weight": (c_int, [c_vp, c_i32, c_i32, c_vp, c_i64]),
    "sli_model_stream": (c_int, [c_vp, ctypes.POINTER(c_vp)]),
    "sli_model_step_bytes": (c_int, [c_vp, P_d, P_d]),
    "sli_model_time_gemv": (c_int, [c_vp, c_i32, P_d, P_d, P_i32]),
    "sli_model_comm_handle_bytes": (c_int, []),
    "sli_model_comm_handle": (c_int, [c_vp, c_vp, c_i32]),
    "sli_model_comm_open": (c_int, [c_vp, c_vp, c_i32]),
    "sli_model_set_allreduce": (c_int, [c_vp, c_i32]),
    "sli_model_time_steps": (c_int, [c_vp, c_i32, P_d]),
    "sli_model_time_families": (c_int, [c_vp, c_i32, P_d, P_d, P_i32]),
    "sli_model_time_stream": (c_int, [c_vp, c_i32, P_d]),
    "sli_debug_bounded_wait": (c_int, [c_i32, c_d, P_d]),
    "sli_tp_group_create": (c_int, [ctypes.POINTER(ModelConfig), c_i32, ctypes.POINTER(c_vp)]),
    "sli_tp_group_destroy": (c_int, [c_vp]),
    "sli_tp_group_rank": (c_int, [c_vp, c_i32, ctypes.POINTER(c_vp)]),
    "sli_tp_group_step": (c_int, [c_vp]),
    "sli_tp_group_sync": (c_int, [c_vp]),
    "sli_tp_group_predict_batch": (c_int, [c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "sli_tp_group_prefill": (c_int, [c_vp, c_vp, c_i32]),
    "sli_tp_group_predict_prefill": (c_int, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load libsli.so; raises (never falls back) if the HIP extension is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -m simplellminference_amd.build` "
                              "(no CPU fallback exists for the decode path)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def exported_symbols() -> list[str]:
    return sorted(_SIGS)


def check(rc: int, where: str) -> None:
    if rc != SLI_OK:
        detail = load().sli_last_error()
        raise SliError(rc, where, detail.decode() if detail else "")


def call(name: str, *args) -> int:
    rc = getattr(load(), name)(*args)
    if isinstance(rc, int) and name not in ("sli_version", "sli_mha_workspace_bytes", "sli_comm_id_bytes",
                                                 "sli_model_comm_handle_bytes",
                                                 "sli_matmul_batch_workspace_bytes"):
        check(rc, name)
    return rc
