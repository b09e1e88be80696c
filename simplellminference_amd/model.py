"""``LlamaModel`` — Python mirror of the reference's model::LlamaModel (include/model/model.h:59-89)
over the fused, graph-captured HIP decode step of libsli.so (engine.hip).

Differences from the reference, all deliberate and documented in DESIGN.md:
  * the model shape is a runtime ``LlamaModelConfig`` (the reference hard-codes config.h:5-17 and
    copies it back in read_model_file, model.cpp:219-230);
  * ``predict`` takes token ids, or text when a ``tokenizer_path`` is given (``encode.SPELayer`` over the Python
    sentencepiece package, encode.cpp:5-27; loaded in ``init`` as create_nonparam_layers does, model.cpp:328);
  * weights are either the reference's flat fp32 file (model_path) or seeded synthetic weights.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, replace

import numpy as np

from . import _lib
from ._lib import DT_F16, DT_F32, DT_I8, ModelConfig, call

_DTYPES = {"f32": DT_F32, "fp32": DT_F32, "f16": DT_F16, "fp16": DT_F16, "i8": DT_I8, "int8": DT_I8}


@dataclass(frozen=True)
class LlamaModelConfig:
    """include/model/config.h:5-17 (same field names)."""
    vocab_size: int = 128256
    head_dim: int = 128
    hidden_size: int = 3072
    kv_hidden_size: int = 1024
    intermediate_size: int = 8192
    max_length: int = 1024
    num_hidden_layers: int = 28
    num_attention_heads: int = 24
    num_key_value_heads: int = 8
    rms_norm_eps: float = 1e-5
    rope_theta: float = 100000.0


PRESETS = {
    # BASELINE.json configs[0]: tiny-llama shape (2 layers, d=256, 4 heads), greedy 32 tokens
    "tiny": LlamaModelConfig(512, 64, 256, 256, 768, 64, 2, 4, 4, 1e-5, 10000.0),
    "tiny-gqa": LlamaModelConfig(512, 64, 256, 128, 768, 64, 2, 4, 2, 1e-5, 10000.0),
    # tiny shapes wide enough for tensor parallelism over 8 ranks (heads and kv heads divisible by 8)
    "tiny-h8": LlamaModelConfig(512, 64, 512, 512, 1024, 64, 2, 8, 8, 1e-5, 10000.0),
    "tiny-gqa-h16": LlamaModelConfig(512, 64, 1024, 512, 2048, 64, 2, 16, 8, 1e-5, 10000.0),
    # small head_dim-128 shapes for the persistent layer stack (tp_layers.h: head_dim 128, per-CU shares that fit)
    "small-h128": LlamaModelConfig(1000, 128, 1024, 1024, 2816, 512, 2, 8, 8, 1e-5, 10000.0),
    "small-h128-gqa": LlamaModelConfig(1000, 128, 1024, 512, 2816, 512, 2, 8, 4, 1e-5, 10000.0),
    # configs[1..3]: Llama-2 7B (public model card shape), ctx 2048
    "llama2-7b": LlamaModelConfig(32000, 128, 4096, 4096, 11008, 2048, 32, 32, 32, 1e-5, 10000.0),
    # configs[4]: Llama-3 8B (GQA), ctx 4096
    "llama3-8b": LlamaModelConfig(128256, 128, 4096, 1024, 14336, 4096, 32, 32, 8, 1e-5, 500000.0),
    # the reference's own hard-coded default (config.h:5-17, Llama-3.2-3B shape)
    "reference-default": LlamaModelConfig(),
}


def preset(name: str, **overrides) -> LlamaModelConfig:
    return replace(PRESETS[name], **overrides)


class LlamaModel:
    def __init__(self, tokenizer_path: str = "", model_path: str = "", device_type: str = "cuda",
                 config: LlamaModelConfig | None = None, w_dtype: str = "f16", kv_dtype: str = "f16",
                 act_mode: int = 0, tp_rank: int = 0, tp_size: int = 1, comm_id: bytes | None = None,
                 device: int = 0, seed: int | None = None, batch: int = 1):
        if device_type not in ("cuda", "hip"):
            raise ValueError("Device Type ERROR!")  # op/*.cpp dispatch: only the HIP backend exists here
        self.tokenizer_path = tokenizer_path
        self.model_path = model_path
        self.config = config or LlamaModelConfig()
        self.w_dtype = _DTYPES[w_dtype]
        self.kv_dtype = _DTYPES[kv_dtype]
        self.act_mode = act_mode
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.comm_id = comm_id
        self.device = device
        self.seed = seed
        self.batch = batch  # sequences decoding in lockstep (extension: the reference is batch 1)
        self._h = None
        self.encode_layer = None

    # ------------------------------------------------------------------ model.h:63-67
    def _config_struct(self) -> ModelConfig:
        c = self.config
        if c.kv_hidden_size != c.num_key_value_heads * c.head_dim:
            raise ValueError("kv_hidden_size must equal num_key_value_heads * head_dim")
        return ModelConfig(c.vocab_size, c.hidden_size, c.num_attention_heads, c.num_key_value_heads, c.head_dim,
                           c.intermediate_size, c.num_hidden_layers, c.max_length, c.rms_norm_eps, c.rope_theta,
                           self.w_dtype, self.kv_dtype, self.act_mode, self.tp_rank, self.tp_size, self.device,
                           self.batch)

    def init(self) -> "LlamaModel":
        if self.tokenizer_path:  # model.cpp:328 (RuntimeError when the model file does not load, encode.cpp:8-10)
            from .encode import SPELayer
            self.encode_layer = SPELayer(self.tokenizer_path)
        mc = self._config_struct()
        h = ctypes.c_void_p()
        cid = ctypes.create_string_buffer(self.comm_id, len(self.comm_id)) if self.comm_id else None
        call("sli_model_create", ctypes.byref(mc), cid, ctypes.byref(h))
        self._h = h
        return self._load_weights()

    def _load_weights(self) -> "LlamaModel":
        if self.model_path:
            call("sli_model_load_flat", self._h, self.model_path.encode())
        elif self.seed is not None:
            call("sli_model_init_synthetic", self._h, self.seed)
        else:
            raise ValueError("No model weigth file!")  # model.cpp:205-207
        return self

    _borrowed = False  # a rank of a TPGroup: the group owns (steps, destroys) the engine

    def close(self):
        if self._h is not None and not self._borrowed:
            _lib.load().sli_model_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ weights / state
    def set_weight(self, kind: int, index: int, tensor: np.ndarray):
        t = np.ascontiguousarray(tensor, np.float32)
        call("sli_model_set_weight", self._h, kind, index, t.ctypes.data_as(ctypes.c_void_p), t.size)

    def reset(self):
        call("sli_model_reset", self._h)

    def fill_kv_synthetic(self, seed: int, upto: int):
        call("sli_model_fill_kv_synthetic", self._h, seed, upto)

    def set_state(self, token: int, pos: int, advance: bool = True):
        call("sli_model_set_state", self._h, token, pos, 1 if advance else 0)

    def set_prompt(self, ids):
        a = np.ascontiguousarray(ids, np.int32)
        call("sli_model_set_prompt", self._h, a.ctypes.data_as(ctypes.c_void_p), a.size)

    def state(self, seq: int = 0):
        p, t, a, e = (ctypes.c_int32() for _ in range(4))
        call("sli_model_get_state_seq", self._h, seq, ctypes.byref(p), ctypes.byref(t), ctypes.byref(a),
             ctypes.byref(e))
        return {"pos": p.value, "token": t.value, "last_argmax": a.value, "error": e.value}

    def set_state_seq(self, seq: int, token: int, pos: int, advance: bool = True):
        call("sli_model_set_state_seq", self._h, seq, token, pos, 1 if advance else 0)

    def set_prompt_seq(self, seq: int, ids):
        a = np.ascontiguousarray(ids, np.int32)
        call("sli_model_set_prompt_seq", self._h, seq, a.ctypes.data_as(ctypes.c_void_p), a.size)

    def history(self, seq: int, n: int) -> np.ndarray:
        out = np.empty(n, np.int32)
        call("sli_model_get_history", self._h, seq, n, out.ctypes.data_as(ctypes.c_void_p))
        return out

    @property
    def local_vocab(self) -> int:
        c = self.config
        chunk = -(-c.vocab_size // self.tp_size)
        return max(0, min(chunk, c.vocab_size - self.tp_rank * chunk))

    # ------------------------------------------------------------------ execution
    EXEC = {"launches": 0, "persist": 2}

    def set_exec(self, mode: str) -> "LlamaModel":
        """"launches": one graph of fused launches per layer; "persist": the embedding, every layer as ONE persistent
        launch (csrc/tp_layers.h; batch-1 fp16 models at head_dim 128 whose per-CU shares fit, e.g. the TP-4 / TP-8
        shards of Llama-2-7B; under tensor parallelism after set_allreduce("fused_wg") or without a communicator),
        then the LM head. Any other name (e.g. the removed "persistent") goes to the C layer as an unknown mode, which
        raises SliError(SLI_ERR_ARG) with its message."""
        call("sli_model_set_exec", self._h, self.EXEC.get(mode, -1))
        return self

    def exec_mode(self) -> str:
        v = ctypes.c_int32()
        call("sli_model_get_exec", self._h, ctypes.byref(v))
        return {i: k for k, i in self.EXEC.items()}[v.value]

    # ------------------------------------------------------------------ tensor-parallel all-reduce
    def comm_handle(self) -> bytes:
        """This rank's one-shot all-reduce buffer as an IPC handle (exchange it with the other ranks)."""
        n = _lib.load().sli_model_comm_handle_bytes()
        buf = ctypes.create_string_buffer(n)
        call("sli_model_comm_handle", self._h, buf, n)
        return buf.raw

    def comm_open(self, handles: list[bytes]) -> "LlamaModel":
        blob = b"".join(handles)
        buf = ctypes.create_string_buffer(blob, len(blob))
        call("sli_model_comm_open", self._h, buf, len(handles))
        return self

    def set_allreduce(self, mode: str) -> "LlamaModel":
        """"rccl" (ncclAllReduce in the step graph), "oneshot" (oneshot.h, after comm_open), "fused" (the
        one-shot exchange inside the wo / down GEMV launches, batch 1; oneshot.h EpiPush) or "fused_wg" (the
        same per workgroup: ranks on distinct devices, sli.h SLI_ALLREDUCE_FUSED_WG)."""
        call("sli_model_set_allreduce", self._h, {"rccl": 0, "oneshot": 1, "fused": 2, "fused_wg": 3}[mode])
        return self

    # ------------------------------------------------------------------ model.cpp:40-140
    def step(self):
        call("sli_model_step", self._h)

    def sync(self):
        call("sli_model_sync", self._h)

    def logits(self) -> tuple[np.ndarray, int]:
        """This rank's vocab shard of the last step's logits: [local vocab], or [batch, local vocab]."""
        out = np.empty(self.batch * self.local_vocab, np.float32)
        lo = ctypes.c_int32()
        call("sli_model_get_logits", self._h, out.ctypes.data_as(ctypes.c_void_p), out.size, ctypes.byref(lo))
        return (out.reshape(self.batch, -1) if self.batch > 1 else out), lo.value

    def forward(self, token: int, pos: int) -> np.ndarray:
        """One decode step at (token, pos); returns this rank's logits shard."""
        self.set_state(token, pos, advance=False)
        self.step()
        return self.logits()[0]

    def forward_batch(self, tokens, positions) -> np.ndarray:
        """One decode step of every sequence b at (tokens[b], positions[b]); returns [batch, local vocab]."""
        for b in range(self.batch):
            self.set_state_seq(b, int(tokens[b]), int(positions[b]), advance=False)
        self.step()
        return self.logits()[0].reshape(self.batch, -1)

    # ------------------------------------------------------------------ model.cpp:142-187
    def predict(self, prompt_ids, max_length: int, want_logits: bool = False):
        """Token ids in: the tokens fed at positions 0..max_length-1 (and the logits). Text in (the reference's
        ``predict(const std::string prompt, int max_length)``): encode it, run the same loop, print and return
        the text model.cpp:154-186 writes — every fed token and the final argmax, decoded one by one."""
        if isinstance(prompt_ids, str):
            return self._predict_text(prompt_ids, max_length)
        p = np.ascontiguousarray(prompt_ids, np.int32)
        toks = np.empty(max_length, np.int32)
        logits = np.empty((max_length, self.local_vocab), np.float32) if want_logits else None
        call("sli_model_predict", self._h, p.ctypes.data_as(ctypes.c_void_p), p.size, max_length,
             toks.ctypes.data_as(ctypes.c_void_p), logits.ctypes.data_as(ctypes.c_void_p) if want_logits else None)
        return (toks, logits) if want_logits else toks

    def _predict_text(self, prompt: str, max_length: int) -> str:
        from .encode import render_predict
        if self.encode_layer is None:
            raise RuntimeError("predict(text) needs a tokenizer_path")
        ids = self.encode_layer.encode(prompt)
        if not ids:
            raise ValueError("the prompt encodes to no tokens")
        if max_length <= 0:  # the loop body never runs: only the first prompt token is printed (model.cpp:154-155)
            text = render_predict(self.encode_layer, [], ids[0])
        else:
            fed = self.predict(ids, max_length)
            text = render_predict(self.encode_layer, fed.reshape(-1, max_length)[0], self.state()["token"])
        print(text, end="")
        return text

    def prefill(self, prompt_ids):
        """Run prompt positions 0..n-2 through the layers in chunks of up to 256 (MFMA GEMM projections,
        block-causal attention) and leave the state at the last prompt token, so the next step() yields the
        first greedy token (sli_model_prefill). Under multi-process tensor parallelism every rank calls it."""
        p = np.ascontiguousarray(prompt_ids, np.int32)
        call("sli_model_prefill", self._h, p.ctypes.data_as(ctypes.c_void_p), p.size)

    def prefill_path(self) -> str:
        """'mfma' (chunked MFMA GEMMs) or 'decode' (teacher-forced decode steps): sli_model_prefill_path."""
        return "mfma" if _lib.load().sli_model_prefill_path(self._h) == 1 else "decode"

    def fused_qkv_attn(self) -> int:
        """1 when the decode step runs q/k/v + attention as one launch per layer, 0 otherwise:
        sli_model_fused_qkv_attn."""
        return int(_lib.load().sli_model_fused_qkv_attn(self._h))

    def predict_prefill(self, prompt_ids, max_length: int, want_logits: bool = False):
        """predict() with the prompt prefilled; logits rows of positions < len(prompt) - 1 are NaN."""
        p = np.ascontiguousarray(prompt_ids, np.int32)
        toks = np.empty(max_length, np.int32)
        logits = np.empty((max_length, self.local_vocab), np.float32) if want_logits else None
        call("sli_model_predict_prefill", self._h, p.ctypes.data_as(ctypes.c_void_p), p.size, max_length,
             toks.ctypes.data_as(ctypes.c_void_p), logits.ctypes.data_as(ctypes.c_void_p) if want_logits else None)
        return (toks, logits) if want_logits else toks

    def predict_batch(self, prompts, max_length: int, want_logits: bool = False):
        """predict for `batch` sequences with their own prompts (ragged lengths allowed): tokens [batch,
        max_length] (the token fed at each position), logits [batch, max_length, local vocab]."""
        if len(prompts) != self.batch:
            raise ValueError(f"need {self.batch} prompts")
        ld = max(len(p) for p in prompts)
        P = np.zeros((self.batch, ld), np.int32)
        for b, p in enumerate(prompts):
            P[b, :len(p)] = p
        lens = np.array([len(p) for p in prompts], np.int32)
        toks = np.empty((self.batch, max_length), np.int32)
        logits = np.empty((max_length, self.batch, self.local_vocab), np.float32) if want_logits else None
        call("sli_model_predict_batch", self._h, P.ctypes.data_as(ctypes.c_void_p), lens.ctypes.data_as(ctypes.c_void_p),
             ld, max_length, toks.ctypes.data_as(ctypes.c_void_p),
             logits.ctypes.data_as(ctypes.c_void_p) if want_logits else None)
        return (toks, logits.transpose(1, 0, 2).copy()) if want_logits else toks

    def weight_shard(self, kind: int, index: int = 0) -> np.ndarray:
        """This rank's shard of a weight (sli_tp_plan window) read back as fp32."""
        from .tp import KINDS, shard_window
        name = {v: k for k, v in KINDS.items()}[kind]
        if name == "norm":
            shape = (self.config.hidden_size,)
        else:
            w = shard_window(self.config, name, self.tp_rank, self.tp_size)
            shape = (w.n_rows, w.n_cols)
        out = np.empty(shape, np.float32)
        call("sli_model_get_weight", self._h, kind, index, out.ctypes.data_as(ctypes.c_void_p), out.size)
        return out

    def kv(self, layer: int, which: int, upto: int, seq: int = 0) -> np.ndarray:
        c = self.config
        out = np.empty((upto, c.num_key_value_heads // self.tp_size * c.head_dim), np.float32)
        call("sli_model_get_kv_seq", self._h, seq, layer, which, upto, out.ctypes.data_as(ctypes.c_void_p))
        return out

    # ------------------------------------------------------------------ measurement
    def stream(self) -> int:
        s = ctypes.c_void_p()
        call("sli_model_stream", self._h, ctypes.byref(s))
        return s.value or 0

    def step_bytes(self) -> tuple[float, float]:
        w, k = ctypes.c_double(), ctypes.c_double()
        call("sli_model_step_bytes", self._h, ctypes.byref(w), ctypes.byref(k))
        return w.value, k.value

    def time_steps(self, iters: int = 20) -> float:
        """Mean device µs of one replayed step (HIP events on the model's stream)."""
        v = ctypes.c_double()
        call("sli_model_time_steps", self._h, iters, ctypes.byref(v))
        return v.value

    FAMILIES = ("qkv", "attention", "wo", "gate_up", "down", "lm_head")

    def time_families(self, iters: int = 20) -> dict:
        """Per kernel family: mean device µs per launch, algorithmic bytes per launch, launches per step."""
        n = len(self.FAMILIES)
        us, b, k = (ctypes.c_double * n)(), (ctypes.c_double * n)(), (ctypes.c_int32 * n)()
        call("sli_model_time_families", self._h, iters, us, b, k)
        return {f: {"avg_us": us[i], "bytes_per_launch": b[i], "launches_per_step": k[i]}
                for i, f in enumerate(self.FAMILIES)}

    def time_stream(self, iters: int = 20) -> dict:
        """Per kernel family: mean device µs of a pure streaming read of the same buffers (the floor)."""
        n = len(self.FAMILIES)
        us = (ctypes.c_double * n)()
        call("sli_model_time_stream", self._h, iters, us)
        return {f: us[i] for i, f in enumerate(self.FAMILIES)}

    def time_gemv(self, iters: int = 20) -> dict:
        us, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
        call("sli_model_time_gemv", self._h, iters, ctypes.byref(us), ctypes.byref(b), ctypes.byref(n))
        return {"avg_us": us.value, "bytes_per_launch": b.value, "launches_per_step": n.value}


def comm_id() -> bytes:
    """A fresh RCCL unique id (rank 0 creates it and broadcasts it to the other ranks)."""
    n = _lib.load().sli_comm_id_bytes()
    buf = ctypes.create_string_buffer(n)
    call("sli_comm_get_id", buf)
    return buf.raw


class TPGroup:
    """In-process tensor parallelism (sli_tp_group): ``tp_size`` rank engines on one
    device, stepped in lockstep by one graph whose all-reduces are device-side reductions over the ranks'
    buffers. ``ranks[r]`` is a borrowed ``LlamaModel`` of rank r (weights, state, logits shard)."""

    def __init__(self, config: LlamaModelConfig, tp_size: int, w_dtype: str = "f16", kv_dtype: str = "f16",
                 act_mode: int = 0, device: int = 0, seed: int | None = None, batch: int = 1,
                 model_path: str = ""):
        self.config, self.tp_size, self.batch = config, tp_size, batch
        proto = LlamaModel(model_path=model_path, config=config, w_dtype=w_dtype, kv_dtype=kv_dtype,
                           act_mode=act_mode, tp_rank=0, tp_size=tp_size, device=device, seed=seed, batch=batch)
        mc = proto._config_struct()
        g = ctypes.c_void_p()
        call("sli_tp_group_create", ctypes.byref(mc), tp_size, ctypes.byref(g))
        self._g = g
        self.ranks = []
        for r in range(tp_size):
            h = ctypes.c_void_p()
            call("sli_tp_group_rank", g, r, ctypes.byref(h))
            m = LlamaModel(model_path=model_path, config=config, w_dtype=w_dtype, kv_dtype=kv_dtype,
                           act_mode=act_mode, tp_rank=r, tp_size=tp_size, device=device, seed=seed, batch=batch)
            m._h = h
            m._borrowed = True
            self.ranks.append(m)

    def init(self) -> "TPGroup":
        for m in self.ranks:
            m._load_weights()
        return self

    def close(self):
        if self._g is not None:
            for m in self.ranks:
                m._h = None
            _lib.load().sli_tp_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fill_kv_synthetic(self, seed: int, upto: int):
        for m in self.ranks:
            m.fill_kv_synthetic(seed, upto)

    def step(self):
        call("sli_tp_group_step", self._g)

    def sync(self):
        call("sli_tp_group_sync", self._g)

    def logits(self) -> np.ndarray:
        """The full-vocabulary logits of the last step ([vocab] or [batch, vocab]), the ranks' shards in place."""
        parts = [m.logits()[0] for m in self.ranks]
        return np.concatenate(parts, axis=-1)

    def forward_batch(self, tokens, positions) -> np.ndarray:
        for m in self.ranks:
            for b in range(self.batch):
                m.set_state_seq(b, int(tokens[b]), int(positions[b]), advance=False)
        self.step()
        return self.logits().reshape(self.batch, -1)

    def forward(self, token: int, pos: int) -> np.ndarray:
        return self.forward_batch([token] * self.batch, [pos] * self.batch)[0]

    def predict_batch(self, prompts, max_length: int, want_logits: bool = False):
        if len(prompts) != self.batch:
            raise ValueError(f"need {self.batch} prompts")
        ld = max(len(p) for p in prompts)
        P = np.zeros((self.batch, ld), np.int32)
        for b, p in enumerate(prompts):
            P[b, :len(p)] = p
        lens = np.array([len(p) for p in prompts], np.int32)
        toks = np.empty((self.batch, max_length), np.int32)
        V = self.config.vocab_size
        logits = np.empty((max_length, self.batch, V), np.float32) if want_logits else None
        call("sli_tp_group_predict_batch", self._g, P.ctypes.data_as(ctypes.c_void_p),
             lens.ctypes.data_as(ctypes.c_void_p), ld, max_length, toks.ctypes.data_as(ctypes.c_void_p),
             logits.ctypes.data_as(ctypes.c_void_p) if want_logits else None)
        return (toks, logits.transpose(1, 0, 2).copy()) if want_logits else toks

    def prefill(self, prompt_ids):
        """sli_tp_group_prefill: the ranks' prefill chunks in lockstep (batch-1 groups)."""
        p = np.ascontiguousarray(prompt_ids, np.int32)
        call("sli_tp_group_prefill", self._g, p.ctypes.data_as(ctypes.c_void_p), p.size)

    def predict_prefill(self, prompt_ids, max_length: int, want_logits: bool = False):
        """predict() with the prompt prefilled; logits [max_length, vocab], rows < len(prompt) - 1 NaN."""
        p = np.ascontiguousarray(prompt_ids, np.int32)
        toks = np.empty(max_length, np.int32)
        logits = np.empty((max_length, self.config.vocab_size), np.float32) if want_logits else None
        call("sli_tp_group_predict_prefill", self._g, p.ctypes.data_as(ctypes.c_void_p), p.size, max_length,
             toks.ctypes.data_as(ctypes.c_void_p), logits.ctypes.data_as(ctypes.c_void_p) if want_logits else None)
        return (toks, logits) if want_logits else toks

    def predict(self, prompt_ids, max_length: int, want_logits: bool = False):
        r = self.predict_batch([list(prompt_ids)] * self.batch, max_length, want_logits)
        if want_logits:
            return r[0][0], r[1][0]
        return r[0]
