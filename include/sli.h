/*
 * sli.h — the C ABI of the MI355X-native decode path (libsli.so).
 *
 * Plain pointers, sizes and status codes only (no torch or HIP types in any signature; a stream is an
 * opaque void* that is a hipStream_t, NULL = the default stream). Device pointers are HIP device
 * memory on the current device. Every entry point returns SLI_OK (0) or an sli_status code; the text
 * of the last error on the calling thread is available from sli_last_error().
 *
 * Two layers:
 *  (1) kernel level — one entry point per reference launcher in include/kernel/cuda/ (*.cuh); the C++
 *      drop-in op:: layer (include/op/, simplellminference_amd/csrc/host/) unpacks mem::Tensor and
 *      calls these;
 *  (2) model level — the whole LlamaModel decode step (source/model/model.cpp:40-187) as one fused,
 *      graph-captured HIP step per token, optionally tensor-parallel over RCCL.
 * Reference citations are /root/reference paths.
 */
#ifndef SLI_H_
#define SLI_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SLI_OK = 0,
    SLI_ERR_ARG = 1,    /* null pointer / bad enum / bad scalar */
    SLI_ERR_SHAPE = 2,  /* tensor dimensions inconsistent (reference: LOG("Tensor with Wrong Dim!")) */
    SLI_ERR_RANGE = 3,  /* token or position out of range (reference: emb_kernel.cpp:10) */
    SLI_ERR_HIP = 4,    /* HIP runtime error */
    SLI_ERR_NOMEM = 5,  /* device allocation failed */
    SLI_ERR_COMM = 6,   /* RCCL error */
    SLI_ERR_STATE = 7,  /* call not valid in the object's current state */
    SLI_ERR_TIMEOUT = 8 /* a host wait on a stream with RCCL collectives made no progress for SLI_COMM_TIMEOUT_MS
                           (default 120 s): a peer or the communicator is wedged; the communicator was aborted */
} sli_status;

typedef enum { SLI_DT_F32 = 0, SLI_DT_F16 = 1, SLI_DT_I8 = 2 } sli_dtype;

typedef void* sli_stream_t;

int sli_version(void);
const char* sli_status_str(int status);
const char* sli_last_error(void);

/* ---------------------------------------------------------------- device helpers */
int sli_device_count(int* n);
int sli_set_device(int device);
int sli_malloc(void** ptr, size_t bytes);
int sli_free(void* ptr);
int sli_memset(void* ptr, int value, size_t bytes, sli_stream_t stream);
int sli_memcpy_h2d(void* dst, const void* src, size_t bytes, sli_stream_t stream);
int sli_memcpy_d2h(void* dst, const void* src, size_t bytes, sli_stream_t stream);
int sli_memcpy_d2d(void* dst, const void* src, size_t bytes, sli_stream_t stream);
int sli_stream_create(sli_stream_t* out);
int sli_stream_destroy(sli_stream_t stream);
int sli_stream_sync(sli_stream_t stream);

/* ---------------------------------------------------------------- kernel level
 * Each replaces one reference CUDA launcher; semantics follow the reference CPU kernel (the oracle). */

/* kernel::matmul_kernel_cuda (include/kernel/cuda/matmul_kernel.cuh:6-7; CPU semantics
 * source/kernel/cpu/matmul_kernel.cpp:5-28): y[r] = scale * sum_c x[c] * W[r][c]; W row-major
 * [rows][cols] in w_dtype; w_row_scale[rows] multiplies each row for SLI_DT_I8 (NULL otherwise). */
int sli_matmul(const float* x, const void* w, int w_dtype, const float* w_row_scale, float* y, int32_t rows,
               int32_t cols, float scale, sli_stream_t stream);

/* Batched projection for B sequences decoding in lockstep (the reference is batch 1; this serves
 * SURVEY.md §8 config C4): y[b][r] = sum_c x[b][c] * W[r][c] for b < batch <= 8, on MFMA
 * (v_mfma_f32_16x16x32_f16; the fp32 input is carried as fp16 hi + lo columns). x [batch][cols] fp32, W
 * [rows][cols] fp16 (SLI_DT_F16 only), y [batch][rows] fp32, cols % 32 == 0. The workspace
 * (sli_matmul_batch_workspace_bytes, 0 = unsupported shape) holds split-K partials and counters. */
size_t sli_matmul_batch_workspace_bytes(int32_t rows, int32_t cols, int32_t batch);
int sli_matmul_batch(const float* x, const void* w, int w_dtype, float* y, int32_t rows, int32_t cols, int32_t batch,
                     void* workspace, size_t workspace_bytes, sli_stream_t stream);

/* kernel::rmsnorm_kernel_cuda (rms_kernel.cuh:6-7; CPU rms_kernel.cpp:5-23): y = x / sqrt(mean(x^2)+eps) * w.
 * Single-workgroup reduction: no atomics, no per-call allocation (the reference allocates + memsets a
 * {1} tensor per call and races across blocks, rms_kernel.cu:29-33,48-51). */
int sli_rmsnorm(const float* x, const float* w, float* y, int32_t dim, float eps, sli_stream_t stream);

/* kernel::rope_cache_cal_cuda (rope_kernel.cuh:5-6; CPU rope_kernel.cpp:4-19): the fp32 sin/cos table
 * [max_seq_len][head_dim/2] is computed on the host with libm powf/sinf/cosf (bit-identical to the
 * reference CPU table) and copied to sin_dev / cos_dev. */
int sli_rope_cache(int32_t head_dim, int32_t max_seq_len, float* sin_dev, float* cos_dev, float theta,
                   sli_stream_t stream);

/* kernel::rope_kernel_cuda (rope_kernel.cuh:7-8; CPU rope_kernel.cpp:22-41): rotate-half RoPE of q
 * (q_dim) and k (k_dim) at position pos_dev ? *pos_dev : pos. k is rotated over k_dim only. */
int sli_rope(float* q, float* k, int32_t pos, const int32_t* pos_dev, const float* sin_dev, const float* cos_dev,
             int32_t q_dim, int32_t k_dim, int32_t head_dim, sli_stream_t stream);

/* kernel::mha_kernel_cuda (mha_kernel.cuh:6-21; CPU mha_kernel.cpp:36-77): decode attention for one
 * layer at position pos over a KV cache in REFERENCE layout [L][T][KV] (fp32 or fp16). Split-context
 * flash-decoding: needs sli_mha_workspace_bytes() of device scratch (the reference's {hd,T} score
 * buffer is not needed). */
size_t sli_mha_workspace_bytes(int32_t max_seq_len, int32_t n_heads, int32_t head_dim);
int sli_mha(const float* q, const void* kcache, const void* vcache, int kv_dtype, float* out, int32_t layer,
            int32_t pos, int32_t max_seq_len, int32_t head_dim, int32_t n_heads, int32_t n_kv_heads,
            void* workspace, size_t workspace_bytes, sli_stream_t stream);

/* softmax_kernel_cpu (mha_kernel.cpp:7-20) as a standalone in-place op over n floats. */
int sli_softmax(float* x, int32_t n, sli_stream_t stream);

/* kernel::swiglu_kernel_cuda (swiglu_kernel.cuh:5; CPU swiglu_kernel.cpp:5-15): out = sigmoid(gate)*up
 * (the reference variant; see sli_model_config.act_mode for SiLU). */
int sli_swiglu(const float* up, const float* gate, float* out, int32_t n, sli_stream_t stream);

/* kernel::add_kernel_cuda (add_kernel.cuh:6; CPU add_kernel.cpp:5-14): out = a + b. */
int sli_add(const float* a, const float* b, float* out, int32_t n, sli_stream_t stream);

/* kernel::emb_kernel_cuda (emb_kernel.cuh:6-7; CPU emb_kernel.cpp:4-21): out = table[token] (row
 * dequantised for SLI_DT_I8 with row_scale). token = token_dev ? *token_dev : token. Returns
 * SLI_ERR_RANGE for a host token outside [0, vocab). A device token cannot be checked without a host
 * sync: outside [0, vocab) it fills `out` with quiet NaNs, so the failure (the reference's LOG-exit,
 * emb_kernel.cu:15-16) propagates loudly instead of as a plausible zero embedding. */
int sli_embedding(int32_t token, const int32_t* token_dev, const void* table, int dtype, const float* row_scale,
                  float* out, int32_t vocab, int32_t dim, sli_stream_t stream);

/* argmaxLayer::forward (source/op/argmax.cpp:7-17) on device: first index of the maximum. */
int sli_argmax(const float* logits, int32_t n, int32_t* out_dev, sli_stream_t stream);

/* ---------------------------------------------------------------- model level */
typedef struct {
    int32_t vocab, dim, n_heads, n_kv_heads, head_dim, ffn, n_layers, max_len;
    float eps, theta;
    int32_t w_dtype;  /* SLI_DT_F32 / SLI_DT_F16 / SLI_DT_I8 (per-row symmetric) */
    int32_t kv_dtype; /* SLI_DT_F32 / SLI_DT_F16 */
    int32_t act_mode; /* 0: reference sigmoid(gate)*up (swiglu_kernel.cpp:12-13); 1: SiLU(gate)*up */
    int32_t tp_rank, tp_size;
    int32_t device;
    int32_t batch;    /* sequences decoding in lockstep, <= 8 (0 or 1: batch 1, the reference's case).
                         batch > 1 runs the projections on MFMA (sli_matmul_batch) and needs fp16 weights */
} sli_model_config;

typedef struct sli_model sli_model;

/* Tensor-parallel shard plan (host only, no device needed): the window of the full reference-layout
 * tensor `kind` (sli_synth.h) that rank cfg->tp_rank holds, and where it lands in the rank's fused
 * buffer. Megatron split: wq/wk/wv/gate/up by output rows (heads / FFN columns),
 * wo/down by input columns, embedding and norms replicated, LM head = embedding rows [vocab_lo,
 * vocab_lo + vocab_n). */
typedef struct {
    int32_t row_lo, n_rows, col_lo, n_cols, full_cols;
    int32_t dst_row_off; /* first row inside the rank's fused buffer ([q;k;v] or [gate;up]) */
} sli_shard_window;
int sli_tp_plan(const sli_model_config* cfg, int32_t kind, sli_shard_window* out);
int sli_tp_vocab(const sli_model_config* cfg, int32_t* vocab_lo, int32_t* vocab_n);

/* One-shot all-reduce over xGMI (replaces the step's RCCL all-reduces; one process per GPU): every rank
 * exports its comm buffer (uncached device memory) with sli_model_comm_handle, the ranks exchange the
 * handles over any host transport, each opens all of them with sli_model_comm_open (handles [nranks][
 * sli_model_comm_handle_bytes()] in rank order) and switches with sli_model_set_allreduce. Each call
 * pushes the rank's partial to every rank, raises a flag per rank, waits (bounded) for all flags and
 * sums in rank order, so every rank holds bit-identical x; the argmax keys use the same exchange.
 * SLI_ALLREDUCE_FUSED (batch 1): the same exchange inside the wo / down GEMV launches — their epilogues
 * push the finished rows into the peers' slots and the launch's last workgroup waits and sums (no
 * separate all-reduce launch).
 * SLI_ALLREDUCE_FUSED_WG (ranks on distinct devices, any batch): the fused exchange per workgroup — workgroup w
 * (batch > 1: MFMA group g) of every rank owns the same rows, waits for the same workgroup of the peers and
 * sums its own rows (no launch-wide arrival, no single summing workgroup). Every workgroup waits, so ranks
 * sharing one device would starve each other of CUs unless their grids fit together
 * (SLI_DEBUG_GEMV_MAX_BLOCKS). The separate ONESHOT sum is sliced over workgroups the same way. */
enum { SLI_ALLREDUCE_RCCL = 0, SLI_ALLREDUCE_ONESHOT = 1, SLI_ALLREDUCE_FUSED = 2, SLI_ALLREDUCE_FUSED_WG = 3 };
int sli_model_comm_handle_bytes(void);
int sli_model_comm_handle(sli_model* m, void* out, int32_t n);
int sli_model_comm_open(sli_model* m, const void* handles, int32_t nranks);
int sli_model_set_allreduce(sli_model* m, int32_t mode);
/* RCCL unique id for tensor parallelism (broadcast it from rank 0 with any host transport). */
int sli_comm_id_bytes(void);
int sli_comm_get_id(void* out);

int sli_model_create(const sli_model_config* cfg, const void* comm_id, sli_model** out);
int sli_model_destroy(sli_model* m);
/* Seeded synthetic weights (include/sli_synth.h), generated on device in this rank's shard. */
int sli_model_init_synthetic(sli_model* m, uint32_t seed);
/* Place one full, unsharded, reference-layout fp32 tensor (kind/index from sli_synth.h). */
int sli_model_set_weight(sli_model* m, int32_t kind, int32_t index, const float* host, int64_t n);
/* Load the reference's flat fp32 weight file (model.cpp:204-245 read, :336-469 layout). */
int sli_model_load_flat(sli_model* m, const char* path);
/* Zero the KV cache and the decode state. */
int sli_model_reset(sli_model* m);
/* Fill K/V rows [0, upto) of every layer with the synthetic N(0,1) values (bench context fill); sequence b
 * of a batch uses seed + b. */
int sli_model_fill_kv_synthetic(sli_model* m, uint32_t seed, int32_t upto);
/* Decode state: the token fed at position pos. advance=1: after each step pos += 1 and the next token
 * is the teacher-forced prompt id or the greedy argmax (model.cpp:157-183); advance=0: the step is
 * idempotent (recomputes the same position; the bench mode). */
int sli_model_set_state(sli_model* m, int32_t token, int32_t pos, int32_t advance);
int sli_model_set_prompt(sli_model* m, const int32_t* ids, int32_t n);
int sli_model_get_state(sli_model* m, int32_t* pos, int32_t* token, int32_t* last_argmax, int32_t* error);
/* Per-sequence forms for batch > 1 (seq < batch). The sequence-less setters above act on every sequence,
 * the getters on sequence 0. */
int sli_model_set_state_seq(sli_model* m, int32_t seq, int32_t token, int32_t pos, int32_t advance);
int sli_model_set_prompt_seq(sli_model* m, int32_t seq, const int32_t* ids, int32_t n);
int sli_model_get_state_seq(sli_model* m, int32_t seq, int32_t* pos, int32_t* token, int32_t* last_argmax,
                            int32_t* error);
/* Prompt prefill (batch-1 models): positions 0 .. n-2 of the prompt run through the layers in chunks of up
 * to 256 positions, every projection one MFMA GEMM over the chunk and attention block-causal over the
 * cache (fp16 / int8 weights, head_dim 64 / 128; otherwise through the decode step, teacher-forced; under
 * multi-process tensor parallelism every rank calls it, the chunk's residual rows all-reduced over RCCL
 * twice per layer), filling the K/V cache; the state is left at
 * (token ids[n-1], position n-1, advancing, prompt = ids), so the next sli_model_step yields the first
 * greedy token exactly as the reference's token-by-token predict (model.cpp:157-165) would. */
int sli_model_prefill(sli_model* m, const int32_t* ids, int32_t n);
/* Which path sli_model_prefill takes for this model: 1 = chunked MFMA GEMMs (prefill.h), 0 = the decode step,
 * teacher-forced (fp32 weights, batch > 1, unsupported shapes, or a TP rank without an RCCL communicator). */
int sli_model_prefill_path(const sli_model* m);
/* 1: the batch-1 decode step runs each layer's q/k/v projection and attention as ONE launch (qkv_attn.h: the
 * attention's K/V rows below the position stream while the projection runs; q and this step's K/V row are
 * handed over inside the launch); 0: separate launches (model.cpp:70-84's matmul / rope / mha sequence either
 * way).
 * Taken where the shape qualifies (heads per kv head 1 or 2, head_dim 64 / 128, fp16 K/V cache, fp16 / int8
 * weights, an attention grid of at most a quarter of the CUs) and SLI_QKV_ATTN allows it
 * (1: always; 0: never; unset: single-rank models). */
int sli_model_fused_qkv_attn(sli_model* m);
/* sli_model_predict with the prompt prefilled: tokens_out[t] as sli_model_predict; logits_out rows for
 * positions < n_prompt - 1 (not computed by the prefill) are NaN. */
int sli_model_predict_prefill(sli_model* m, const int32_t* prompt, int32_t n_prompt, int32_t max_length,
                              int32_t* tokens_out, float* logits_out);
/* The tokens fed at positions [0, n) of sequence seq. */
int sli_model_get_history(sli_model* m, int32_t seq, int32_t n, int32_t* out);
/* Execution of the step: SLI_EXEC_LAUNCHES, one hipGraph of ~5 fused launches per layer (every configuration);
 * SLI_EXEC_PERSIST, the embedding, then EVERY layer as one persistent launch (csrc/tp_layers.h: one workgroup per
 * CU, each op's weight share in registers before its input arrives, the edges as tagged granules, the residual
 * exchange per workgroup inside the launch), then the LM head launches. Taken for batch-1 fp16 models at head_dim
 * 128 whose per-workgroup shares fit (the TP-4 / TP-8 shards of Llama-2-7B); otherwise SLI_ERR_STATE with the
 * reason. Under tensor parallelism it needs the one-shot buffers and SLI_ALLREDUCE_FUSED_WG (ranks on distinct
 * devices), or no communicator (SLI_DEBUG_NOCOMM). Not for the ranks of an in-process group.
 * (Round 5 removed the opt-in persistent one-launch step, mode 1; sli_model_set_exec(1) returns SLI_ERR_ARG.) */
enum { SLI_EXEC_LAUNCHES = 0, SLI_EXEC_PERSIST = 2 };
int sli_model_set_exec(sli_model* m, int32_t mode);
int sli_model_get_exec(sli_model* m, int32_t* mode);
/* One decode step (hipGraph replay; captured on first use). Asynchronous on the model's stream. */
int sli_model_step(sli_model* m);
/* Host waits (sync, logits / state / history reads, predict, prefill, the timing probes) of a rank whose step
 * carries RCCL collectives are bounded (csrc/comm_wait.h): they poll the stream, ncclCommGetAsyncError and a
 * deadline; a communicator error returns SLI_ERR_COMM, an expired deadline SLI_ERR_TIMEOUT, and either aborts the
 * communicator (ncclCommAbort), after which every call that would step returns SLI_ERR_COMM. The reference's
 * all-reduce-free equivalents: the logits copy at model.cpp:175-179. */
int sli_model_sync(sli_model* m);
/* logits of the last step: this rank's vocab shard [vocab_lo, vocab_lo+n) of every sequence, [batch][n]. */
int sli_model_get_logits(sli_model* m, float* host, int32_t n, int32_t* vocab_lo);
/* LlamaModel::predict on token ids: tokens_out[t] = token fed at position t; logits_out optional
 * [max_length][local vocab]. batch > 1: every sequence gets the prompt, tokens_out is [batch][max_length]
 * and logits_out [max_length][batch][local vocab]. */
int sli_model_predict(sli_model* m, const int32_t* prompt, int32_t n_prompt, int32_t max_length,
                      int32_t* tokens_out, float* logits_out);
/* predict for batch sequences with their own prompts: prompts [batch][ld] (sequence b's first lens[b]
 * ids), tokens_out [batch][max_length], logits_out optional [max_length][batch][local vocab]. */
int sli_model_predict_batch(sli_model* m, const int32_t* prompts, const int32_t* lens, int32_t ld, int32_t max_length,
                            int32_t* tokens_out, float* logits_out);
/* Copy one layer's K (which=0) or V (which=1) cache, positions [0, upto), to host as fp32 in reference
 * layout [upto][KV_local]. */
int sli_model_get_kv(sli_model* m, int32_t layer, int32_t which, int32_t upto, float* host);
int sli_model_get_kv_seq(sli_model* m, int32_t seq, int32_t layer, int32_t which, int32_t upto, float* host);
/* Read back this rank's shard of a weight (sli_tp_plan window, n = n_rows * n_cols) as fp32 (int8 is
 * dequantised with its row scales). */
int sli_model_get_weight(sli_model* m, int32_t kind, int32_t index, float* host, int64_t n);
int sli_model_stream(sli_model* m, sli_stream_t* out);
/* Algorithmic HBM bytes of one step on this rank (weights, KV at the current position) — SURVEY.md §8(d). */
int sli_model_step_bytes(sli_model* m, double* weight_bytes, double* kv_bytes);
/* ---------------------------------------------------------------- in-process tensor parallelism
 * The SURVEY.md §4 item-5 "fake communicator" (the reference drives one device, model.cpp:247-256):
 * tp_size rank models of cfg (cfg->tp_rank is ignored; rank r gets the sli_tp_plan shard of rank r)
 * on cfg->device, sharing one stream and stepped in lockstep by one captured hipGraph. Every all-reduce
 * of the multi-GPU step (the residual-stream sum after wo and down, the argmax-key MAX after the LM
 * head) is a device-side reduction over the ranks' buffers in rank order; the ranks' kernels are the
 * multi-GPU ones. Rank handles (sli_tp_group_rank) are borrowed: load weights, set state / prompts and
 * read logits through them; step and destroy only through the group. */
typedef struct sli_tp_group sli_tp_group;
int sli_tp_group_create(const sli_model_config* cfg, int32_t tp_size, sli_tp_group** out);
int sli_tp_group_destroy(sli_tp_group* g);
int sli_tp_group_rank(sli_tp_group* g, int32_t rank, sli_model** out);
int sli_tp_group_step(sli_tp_group* g);
int sli_tp_group_sync(sli_tp_group* g);
/* sli_model_predict_batch over the group: tokens_out [batch][max_length]; logits_out optional
 * [max_length][batch][vocab] with the ranks' vocab shards in place (the full vocabulary). */
int sli_tp_group_predict_batch(sli_tp_group* g, const int32_t* prompts, const int32_t* lens, int32_t ld,
                               int32_t max_length, int32_t* tokens_out, float* logits_out);
/* sli_model_prefill / sli_model_predict_prefill over the group (batch-1 groups): the ranks' prefill chunks
 * run in lockstep, the residual rows summed over the ranks after every wo and down GEMM. logits_out
 * [max_length][vocab] (rows < n_prompt - 1 NaN). */
int sli_tp_group_prefill(sli_tp_group* g, const int32_t* ids, int32_t n);
int sli_tp_group_predict_prefill(sli_tp_group* g, const int32_t* prompt, int32_t n_prompt, int32_t max_length,
                                 int32_t* tokens_out, float* logits_out);

/* Roofline probe: replays the step's weight-streaming (GEMV) kernels `iters` times between HIP events
 * on the model's stream; returns mean device time per GEMV launch, algorithmic bytes per launch and
 * the launches per step. */
int sli_model_time_gemv(sli_model* m, int32_t iters, double* avg_us, double* bytes_per_launch,
                        int32_t* launches_per_step);
/* Device time of one replayed step: `iters` graph launches between HIP events on the model's stream. */
int sli_model_time_steps(sli_model* m, int32_t iters, double* avg_us);
/* Per-kernel-family probe: for each family f (sli_kernel_family) replays that family's launches of one
 * step `iters` times between HIP events on the model's stream; us[f] = mean device time per launch,
 * bytes[f] = algorithmic HBM bytes per launch (the weight matrix (+ int8 row scales),
 * or K and V of the live context for attention), launches[f] = launches per step. Arrays of
 * SLI_FAM_COUNT. */
typedef enum { SLI_FAM_QKV = 0, SLI_FAM_ATTN, SLI_FAM_WO, SLI_FAM_GU, SLI_FAM_DOWN, SLI_FAM_LM, SLI_FAM_COUNT } sli_kernel_family;
int sli_model_time_families(sli_model* m, int32_t iters, double* us, double* bytes, int32_t* launches);
/* The measured streaming-read floor of the same launches: for each family, a pure read kernel (no
 * arithmetic, 16-byte non-temporal loads, one 1024-thread workgroup per CU) over exactly the buffers that
 * family's launches stream (each layer's weight matrix; K and V of the layer for attention, the
 * allocated context), replayed the same way; us[f] = mean device µs per launch (the
 * fraction of a measured stream-copy bandwidth). */
int sli_model_time_stream(sli_model* m, int32_t iters, double* us);
/* Test hook (no device needed): runs the bounded-wait policy of comm_wait.h against mocked probes. mode 0: a
 * query that completes on its 3rd poll (SLI_OK); 1: a query that never completes (SLI_ERR_TIMEOUT after
 * deadline_ms); 2: an async communicator error on the 2nd poll (SLI_ERR_COMM); 3: a failing query (SLI_ERR_HIP).
 * *waited_ms = the wall time the wait took. */
int sli_debug_bounded_wait(int32_t mode, double deadline_ms, double* waited_ms);

#ifdef __cplusplus
}
#endif
#endif
