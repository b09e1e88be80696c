// engine.hip — the model-level C ABI (include/sli.h): LlamaModel's decode step
// (source/model/model.cpp:40-140) and decode loop (:142-187) as a fused, graph-captured HIP step,
// sharded Megatron-style over tp_size ranks (one process per GPU) with RCCL all-reduces.
//
// Per layer, five streaming launches replace the reference's ~18:
//   1. RMSNorm ⊕ [wq;wk;wv] GEMV ⊕ RoPE ⊕ K/V cache write        (model.cpp:52-67)
//   2. attention partials (split context)   3. combine           (model.cpp:70-78)
//   4. wo GEMV ⊕ residual add  [+ all-reduce under TP]           (model.cpp:80-90)
//   5. RMSNorm ⊕ [gate;up] GEMV ⊕ SwiGLU                         (model.cpp:93-115)
//   6. down GEMV ⊕ residual add [+ all-reduce under TP]          (model.cpp:118-128)
// then RMSNorm ⊕ tied LM head ⊕ argmax keys, key reduce [+ all-reduce max], and a one-thread finalize
// that advances the on-device position/token (teacher forcing or greedy, model.cpp:157-183).
// Token and position live in device memory, so one captured hipGraph serves every step.
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <cstring>
#include <vector>

#include "../../include/sli_synth.h"
#include "attention.h"
#include "bgemm.h"
#include "comm_wait.h"
#include "common.h"
#include "gemv.h"
#include "oneshot.h"
#include "ops_internal.h"
#include "prefill.h"
#include "qkv_attn.h"
#include "rope_table.h"
#include "step_state.h"
#include "tp_layers.h"

namespace sli {

struct LayerW {
    void* qkv = nullptr;   // [(hq + 2 hkv) hd][D]
    float* qkv_s = nullptr;
    void* wo = nullptr;    // [D][hq hd]   (column slice of wo, re-laid contiguous)
    float* wo_s = nullptr;
    void* gu = nullptr;    // [2 Il][D]    (gate rows then up rows)
    float* gu_s = nullptr;
    void* down = nullptr;  // [D][Il]      (column slice of down)
    float* down_s = nullptr;
    // batch > 1, fp16: the same matrices in bgemm's fragment layout (bgemm.h BgIn::tiled), rows in each
    // epilogue's tile order; the decode step streams these, the row-major copies serve prefill-free readback
    void *qkv_t = nullptr, *wo_t = nullptr, *gu_t = nullptr, *down_t = nullptr;
};

}  // namespace sli

struct sli_model {
    sli_model_config c{};
    hipStream_t stream = nullptr;
    bool own_stream = true;  // false for the ranks of an in-process group (they share the group's stream)
    sli_tp_group* group = nullptr;  // in-process tensor-parallel group this rank belongs to (or null)
    ncclComm_t comm = nullptr;
    bool partial = false;    // wo/down write per-rank partials (+ residual on rank 0) into xpart
    bool collectives = false;  // all-reduce partials / argmax keys over RCCL inside the step
    // local (this rank's) geometry
    int D = 0, L = 0, T = 0, V = 0, hd = 0, hq = 0, hkv = 0, Il = 0;
    int v_lo = 0, v_n = 0;
    size_t wbytes = 4, kvbytes = 4;
    // device buffers
    void* emb = nullptr;
    float* emb_s = nullptr;
    void* lm_t = nullptr;     // batch > 1: this rank's LM-head rows of emb in the fragment layout (LayerW::*_t)
    bool bg_tiled = false;    // the batched projections stream the fragment-layout copies
    bool tiles_dirty = false; // a weight was placed since the copies were last built (bg_sync_tiles)
    float* norms = nullptr;
    std::vector<sli::LayerW> layers;
    void* kc = nullptr;
    void* vc = nullptr;
    float *x = nullptr, *xpart = nullptr, *q = nullptr, *attn = nullptr, *act = nullptr, *logits = nullptr;
    float* part = nullptr;
    unsigned* attn_count = nullptr;
    float* qa_kv = nullptr;       // batch 1: the fused q/k/v + attention launch's hand-off rows [2][hkv][hd] (qkv_attn.h)
    unsigned* qa_count = nullptr; // its per-kv-head counters (attention.h attn_hand_words; zero between launches)
    int wo_merge = 1;           // batch 1: 1 = the wo GEMV merges the attention's splits while staging its input,
                                // 0 = the attention's last-arriving workgroup merges them (wo_merges)
    int wo_ks = 1;              // batch-1 TP-1 wo split over its columns (wo_ksplit): partials [wo_ks][D]
    float* wo_part = nullptr;
    float *sin_t = nullptr, *cos_t = nullptr;
    unsigned long long* keys = nullptr;
    sli::DevState* st = nullptr;
    int32_t* prompt = nullptr;
    int32_t* hist = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    std::vector<void*> allocs;
    // batch > 1: B sequences decode in lockstep, the projections run on MFMA (bgemm.h)
    int B = 1;
    sli::BgPlan bp_qkv, bp_wo, bp_gu, bp_down, bp_lm;
    float* bg_ws = nullptr;               // split-K partials of the batched projections
    unsigned* bg_cnt = nullptr;           // their arrival counters (zero between launches)
    unsigned long long* bkeys = nullptr;  // [B] per-sequence argmax keys (all-reduced MAX under TP)
    int key_ld = 0;                       // per-sequence stride of the per-workgroup argmax keys
    // prompt prefill (sli_model_prefill, prefill.h): chunks of up to kPfMaxChunk prompt positions through
    // every layer per weight pass; one captured graph per chunk size (kPfSizes)
    struct Prefill {
        float *x = nullptr, *xpart = nullptr, *q = nullptr;  // [chunk][D], [chunk][D] (TP partials), [chunk][hq hd]
        __half *hhi = nullptr, *hlo = nullptr;  // [chunk][max(D, hq hd)]: normed x / attention out, fp16 hi + lo
        __half *ahi = nullptr, *alo = nullptr;  // [chunk][Il]: SwiGLU out, fp16 hi + lo
        sli::PfState* ps = nullptr;             // chunk start position + valid rows (device)
        hipGraph_t graph[4] = {};
        hipGraphExec_t exec[4] = {};
    } pf;
    // tensor-parallel all-reduce: SLI_ALLREDUCE_RCCL (ncclAllReduce) or SLI_ALLREDUCE_ONESHOT (oneshot.h)
    int ar_mode = SLI_ALLREDUCE_RCCL;
    char* os_buf = nullptr;                  // this rank's comm buffer (uncached device memory, IPC-exported)
    char* os_peer[sli::kOsMaxRanks] = {};    // every rank's buffer mapped here (own included)
    bool os_open = false;
    bool os_dead = false;                    // a one-shot wait timed out: set_allreduce(ONESHOT) is refused
    bool comm_dead = false;                  // a bounded host wait aborted the RCCL communicator (comm_wait.h)
    unsigned* os_epoch = nullptr;            // one-shot call counter; os_epoch[1..9]: fused-launch arrivals
    unsigned* os_wg_epoch = nullptr;         // per-(region, workgroup) epochs [kOsRegions][kOsMaxWg] (oneshot.h)
    int os_nmax = 0;
    bool os_loopback = false;                // debug: SLI_DEBUG_OS_LOOPBACK (oneshot.h OneShotArgs::loopback)
    char** os_peer_tab = nullptr;            // device copy of os_peer (oneshot.h EpiPush::peer_tab)
    size_t os_bytes = 0;
    int exec = SLI_EXEC_LAUNCHES;
    // SLI_EXEC_PERSIST: the layer stack as one persistent launch (tp_layers.h); its granule arrays, weight table,
    // launch counter and the device table of every rank's exchange granules (in the one-shot comm buffers)
    struct Tl {
        sli::tl_u2 *g_x = nullptr, *g_qkv = nullptr, *g_part = nullptr, *g_att = nullptr, *g_x1 = nullptr,
                   *g_act = nullptr;
        const __half** w = nullptr;
        unsigned* epoch = nullptr;
        sli::tl_u2** xg = nullptr;
    } tl;
};

// In-process tensor parallelism (the "fake communicator"): tp_size rank models on
// one device share one stream and one captured graph that steps them in lockstep; every all-reduce is a
// device-side reduction over the ranks' buffers in rank order (the ranks' kernels are the multi-GPU
// ones, so the sharded engine itself is what the group tests run).
constexpr int kMaxGroup = 8;
constexpr int kPfSizes[4] = {32, 64, 128, 256};  // prefill chunk sizes (the last is prefill.h kPfMaxChunk)
struct sli_tp_group {
    int n = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<sli_model*> ranks;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    hipGraph_t pf_graph[4] = {};  // the ranks' prefill chunks in lockstep, per chunk size
    hipGraphExec_t pf_exec[4] = {};
};

namespace sli {

static int model_alloc(sli_model* m, void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes ? bytes : 16);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc");
    m->allocs.push_back(*p);
    return SLI_OK;
}

#define SLI_TRY(expr)                   \
    do {                                \
        int rc_ = (expr);               \
        if (rc_ != SLI_OK) return rc_;  \
    } while (0)



#define SLI_NCCL(expr)                                                                          \
    do {                                                                                        \
        ncclResult_t r_ = (expr);                                                               \
        if (r_ != ncclSuccess) return fail(SLI_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// ---------------------------------------------------------------- weight placement
struct SrcSynth {
    uint32_t seed, stream;
    float c, offset;
    __device__ float operator()(uint64_t idx) const {
        const float v = __fmul_rn((float)sli_rng_ih4(seed, stream, idx), c);
        return offset != 0.0f ? __fadd_rn(offset, v) : v;  // sli_synth.h: one mul, one add, no FMA
    }
};

struct SrcBuf {
    const float* p;
    __device__ float operator()(uint64_t idx) const { return p[idx]; }
};

// Copy the [row_lo, row_lo+nrows) x [col_lo, col_lo+ncols) window of a full [*, full_cols] fp32
// tensor into dst (row stride ncols) as T. int8: per-row symmetric scale over the FULL row
// (max|w|/127, q = rint(w/s)), so column shards share the unsharded quantisation.
template <typename T, class Src>
__global__ void __launch_bounds__(256) place_kernel(T* dst, float* dst_scale, int nrows, int ncols, int row_lo,
                                                    int col_lo, int full_cols, Src src) {
    __shared__ float red[4];
    for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
        const uint64_t base = (uint64_t)(row_lo + r) * (uint64_t)full_cols;
        if constexpr (sizeof(T) == 1) {
            float mx = 0.0f;
            for (int c = threadIdx.x; c < full_cols; c += blockDim.x) mx = fmaxf(mx, fabsf(src(base + c)));
            mx = wave_max(mx);
            if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
            __syncthreads();
            mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
            __syncthreads();
            const float s = __fdiv_rn(mx, 127.0f);
            if (threadIdx.x == 0) dst_scale[r] = s;
            for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
                float q = s > 0.0f ? rintf(__fdiv_rn(src(base + col_lo + c), s)) : 0.0f;
                q = fminf(127.0f, fmaxf(-127.0f, q));
                dst[(size_t)r * ncols + c] = (T)(int)q;
            }
        } else {
            for (int c = threadIdx.x; c < ncols; c += blockDim.x)
                dst[(size_t)r * ncols + c] = from_f32<T>(src(base + col_lo + c));
        }
    }
}

template <class Src>
static int place(sli_model* m, void* dst, float* dst_scale, int nrows, int ncols, int row_lo, int col_lo, int full_cols,
                 const Src& src) {
    const int blocks = std::min(nrows, 4096);
    hipStream_t s = m->stream;
    switch (m->c.w_dtype) {
        case SLI_DT_F32:
            hipLaunchKernelGGL((place_kernel<float, Src>), dim3(blocks), dim3(256), 0, s, (float*)dst, dst_scale, nrows,
                               ncols, row_lo, col_lo, full_cols, src);
            break;
        case SLI_DT_F16:
            hipLaunchKernelGGL((place_kernel<__half, Src>), dim3(blocks), dim3(256), 0, s, (__half*)dst, dst_scale,
                               nrows, ncols, row_lo, col_lo, full_cols, src);
            break;
        default:
            hipLaunchKernelGGL((place_kernel<int8_t, Src>), dim3(blocks), dim3(256), 0, s, (int8_t*)dst, dst_scale,
                               nrows, ncols, row_lo, col_lo, full_cols, src);
    }
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

template <class Src>
static int place_f32(sli_model* m, float* dst, int n, const Src& src) {
    hipLaunchKernelGGL((place_kernel<float, Src>), dim3(1), dim3(256), 0, m->stream, dst, nullptr, 1, n, 0, 0, n, src);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

static char* wptr(void* base, size_t elem_bytes, size_t elems) { return (char*)base + elem_bytes * elems; }

// Place one full reference tensor (kind, index) from `src` into this rank's shard (sli_tp_plan).
template <class Src>
static int place_tensor(sli_model* m, int kind, int index, const Src& src) {
    const int D = m->D;
    if (kind == SLI_T_NORM) {
        if (index < 0 || index > 2 * m->L) return fail(SLI_ERR_RANGE, "norm index");
        return place_f32(m, m->norms + (size_t)index * D, D, src);
    }
    sli_shard_window w;
    SLI_TRY(sli_tp_plan(&m->c, kind, &w));
    m->tiles_dirty = m->bg_tiled;
    if (kind == SLI_T_EMB)
        return place(m, m->emb, m->emb_s, w.n_rows, w.n_cols, w.row_lo, w.col_lo, w.full_cols, src);
    if (index < 0 || index >= m->L) return fail(SLI_ERR_RANGE, "layer index");
    LayerW& L = m->layers[index];
    void* base = nullptr;
    float* sbase = nullptr;
    switch (kind) {
        case SLI_T_WQ: case SLI_T_WK: case SLI_T_WV: base = L.qkv; sbase = L.qkv_s; break;
        case SLI_T_WO: base = L.wo; sbase = L.wo_s; break;
        case SLI_T_GATE: case SLI_T_UP: base = L.gu; sbase = L.gu_s; break;
        case SLI_T_DOWN: base = L.down; sbase = L.down_s; break;
        default: return fail(SLI_ERR_ARG, "unknown tensor kind");
    }
    void* dst = wptr(base, m->wbytes, (size_t)w.dst_row_off * w.n_cols);
    return place(m, dst, sbase ? sbase + w.dst_row_off : nullptr, w.n_rows, w.n_cols, w.row_lo, w.col_lo,
                 w.full_cols, src);
}

static int64_t tensor_elems(const sli_model* m, int kind) {
    const int64_t D = m->c.dim, KV = (int64_t)m->c.n_kv_heads * m->c.head_dim, I = m->c.ffn, V = m->c.vocab;
    switch (kind) {
        case SLI_T_EMB: return V * D;
        case SLI_T_NORM: return D;
        case SLI_T_WQ: case SLI_T_WO: return D * D;
        case SLI_T_WK: case SLI_T_WV: return KV * D;
        case SLI_T_UP: case SLI_T_GATE: case SLI_T_DOWN: return I * D;
        default: return -1;
    }
}

static float synth_c(const sli_model* m, int kind) {
    switch (kind) {
        case SLI_T_EMB: return SLI_SYNTH_C(0.02);
        case SLI_T_NORM: return SLI_SYNTH_C(0.1);
        case SLI_T_DOWN: return SLI_SYNTH_C(1.0 / std::sqrt((double)m->c.ffn));
        default: return SLI_SYNTH_C(1.0 / std::sqrt((double)m->c.dim));
    }
}

// ---------------------------------------------------------------- small kernels of the step
// Second argmax stage (256 threads). FINALIZE: the step has no cross-rank key exchange, so the same
// thread that reduced the key also advances the state (one launch instead of keyreduce + finalize).
constexpr int kKeyThreads = 256;
template <bool FINALIZE>
__global__ void __launch_bounds__(kKeyThreads) keyreduce_kernel(const unsigned long long* __restrict__ keys, int n,
                                                                DevState* st, const int32_t* __restrict__ prompt,
                                                                int32_t* hist, int T) {
    unsigned long long b = 0;
    for (int i = threadIdx.x; i < n; i += kKeyThreads) b = keys[i] > b ? keys[i] : b;
    b = wave_max_u64(b);
    __shared__ unsigned long long red[kKeyThreads / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kKeyThreads / 64; ++w) b = red[w] > b ? red[w] : b;
        st->key = red[0] > b ? red[0] : b;
        if constexpr (FINALIZE) finalize_state(st, prompt, hist, T);
    }
}

__global__ void finalize_kernel(DevState* st, const int32_t* __restrict__ prompt, int32_t* hist, int T) {
    finalize_state(st, prompt, hist, T);
}

// ---- batch > 1: one sequence per block / thread
// emb_kernel.cpp:4-21 per sequence, token read on device (graph-capturable)
template <typename T>
__global__ void embedding_batch_kernel(const DevState* st, const T* __restrict__ table, const float* row_scale,
                                       float* __restrict__ out, int vocab, int dim) {
    const int b = blockIdx.y;
    const int token = st[b].token;
    const bool ok = token >= 0 && token < vocab;
    const float s = (ok && row_scale) ? row_scale[token] : 1.0f;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < dim; i += gridDim.x * blockDim.x)
        out[(size_t)b * dim + i] = ok ? to_f32(table[(size_t)token * dim + i]) * s : 0.0f;
}

// second argmax stage per sequence: block b reduces keys[b][0 .. n) into out[b]
__global__ void keyreduce_batch_kernel(const unsigned long long* __restrict__ keys, int ld, int n,
                                       unsigned long long* out) {
    const unsigned long long* k = keys + (size_t)blockIdx.x * ld;
    unsigned long long b = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) b = k[i] > b ? k[i] : b;
    b = wave_max_u64(b);
    __shared__ unsigned long long red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) b = red[w] > b ? red[w] : b;
        out[blockIdx.x] = b;
    }
}

__global__ void finalize_batch_kernel(DevState* st, const unsigned long long* __restrict__ keys,
                                      const int32_t* __restrict__ prompt, int32_t* hist, int T, int B) {
    const int b = threadIdx.x;
    if (b >= B) return;
    st[b].key = keys[b];
    finalize_state(st + b, prompt + (size_t)b * (T + 1), hist + (size_t)b * (T + 1), T);
}

template <typename KT>
__global__ void fill_kv_kernel(KT* kc, KT* vc, int L, int B, int hkv, int T, int hd, int upto, int kv_full,
                               int head_lo, uint32_t seed, float c) {
    const uint64_t n = (uint64_t)L * B * hkv * upto * hd;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int d = (int)(i % hd);
        uint64_t rest = i / hd;
        const int t = (int)(rest % upto);
        rest /= upto;
        const int h = (int)(rest % hkv);
        rest /= hkv;
        const int b = (int)(rest % B);
        const int l = (int)(rest / B);
        const uint64_t idx = (uint64_t)t * kv_full + (uint64_t)(head_lo + h) * hd + d;  // reference layout index
        const size_t off = ((((size_t)l * B + b) * hkv + h) * T + t) * hd + d;
        const uint32_t sb = seed + (uint32_t)b;  // sequence b = the oracle's fill with seed + b
        kc[off] = from_f32<KT>(__fmul_rn((float)sli_rng_ih4(sb, sli_stream_id(SLI_T_KCACHE, l), idx), c));
        vc[off] = from_f32<KT>(__fmul_rn((float)sli_rng_ih4(sb, sli_stream_id(SLI_T_VCACHE, l), idx), c));
    }
}

template <typename KT>
__global__ void get_kv_kernel(const KT* __restrict__ cache, float* out, int hkv, int T, int hd, int upto) {
    const int n = upto * hkv * hd;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int d = i % hd, h = (i / hd) % hkv, t = i / (hd * hkv);
        out[i] = to_f32(cache[((size_t)h * T + t) * hd + d]);
    }
}

// ---- in-process group collectives (sli_tp_group)
struct GroupSumArgs {
    const float* src[kMaxGroup];  // rank r's partial [B*D] (rank 0's includes the residual)
    float* dst[kMaxGroup];        // rank r's residual stream x
    int n_ranks, n;
    int f16_payload = 0;  // debug (SLI_DEBUG_AR_F16): each rank's contribution rounded to fp16 as an
                          // fp16 exchange would carry it (the residual stays fp32, added once locally)
};

// x_r = ((p_0 + p_1) + p_2) + ... for every rank r: one fixed order, so every rank holds the same x
__global__ void __launch_bounds__(256) group_sum_kernel(GroupSumArgs a) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
        float s;
        if (a.f16_payload) {  // x + sum_r fp16(p_r), p_0 = rank 0's partial without the residual it added
            const float x = a.dst[0][i];
            s = __half2float(__float2half(a.src[0][i] - x));
            for (int r = 1; r < a.n_ranks; ++r) s += __half2float(__float2half(a.src[r][i]));
            s = x + s;
        } else {
            s = a.src[0][i];
            for (int r = 1; r < a.n_ranks; ++r) s += a.src[r][i];
        }
        for (int r = 0; r < a.n_ranks; ++r) a.dst[r][i] = s;
    }
}

struct GroupKeyArgs {
    unsigned long long* key[kMaxGroup];  // rank r's per-sequence argmax keys [B] (batch 1: &st->key)
    DevState* st[kMaxGroup];
    const int32_t* prompt[kMaxGroup];
    int32_t* hist[kMaxGroup];
    int n_ranks, B, T;
};

// argmax-key MAX over the ranks' vocab shards (global first max), then every rank's state update
__global__ void group_finalize_kernel(GroupKeyArgs a) {
    const int b = threadIdx.x;
    if (b >= a.B) return;
    unsigned long long k = 0;
    for (int r = 0; r < a.n_ranks; ++r) k = a.key[r][b] > k ? a.key[r][b] : k;
    for (int r = 0; r < a.n_ranks; ++r) {
        DevState* st = a.st[r] + b;
        st->key = k;
        finalize_state(st, a.prompt[r] + (size_t)b * (a.T + 1), a.hist[r] + (size_t)b * (a.T + 1), a.T);
    }
}

// ---------------------------------------------------------------- the step
// launch_gemv_u / gemv_split: gemv.h (shared with the op-level sli_matmul)


// The fused q/k/v + attention launch (qkv_attn.h). SLI_QKV_ATTN=1: wherever the shape qualifies; 0: never;
// unset: single-rank models only (a rank process that may share its GPU with others keeps the two launches
// unless the launcher knows each rank has a device of its own: bench.py sets 1 then). In-process groups never
// (their ranks' launches share one device).
static bool qkv_attn_on(const sli_model* m) {
    static const int env = [] {
        const char* e = getenv("SLI_QKV_ATTN");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    if (m->group || env == 0) return false;
    return env == 1 || !m->partial;
}

// Batched decode: the register-staged attention (fp32 cache) leaves its split merge to attn_merge_kernel (its
// 1024 C4 workgroups run in two residency rounds, so a last-arriver merge inside the launch waits on the second
// round: profiles/r4_c4_merge_launch_ab.txt); the MFMA attention (fp16 cache) merges inside its one resident
// round (ops.hip attn_mfma_launch).
constexpr int kDeferBatched = 2;

// ---------------------------------------------------------------- the layer stack as one persistent launch
// (SLI_EXEC_PERSIST, tp_layers.h). Taken for batch-1 fp16 models at head_dim 128 whose per-workgroup shares fit the
// kernel's LDS partial buffer: the TP-4 / TP-8 shards of Llama-2-7B (C2), not the unsharded 7B.
static int tpl_nwg() { return gemv_max_blocks(); }

static int tpl_check(const sli_model* m, std::string* why) {
    auto no = [&](const char* r) {
        if (why) *why = r;
        return 0;
    };
    if (m->group) return no("the ranks of an in-process group step in lockstep launches (their exchange is between launches)");
    if (m->B != 1) return no("batch 1 only");
    if (m->c.w_dtype != SLI_DT_F16 || m->c.kv_dtype != SLI_DT_F16) return no("fp16 weights and K/V cache only");
    if (m->hd != kTlHD) return no("head_dim 128 only");
    const int G = m->hq / m->hkv;
    if (!(G == 1 || G == 2 || G == 4)) return no("1, 2 or 4 query heads per kv head");
    if (m->D % 8 || m->Il % 8 || m->D > kTlMaxD || m->Il > kTlMaxX || m->hq * kTlHD > kTlMaxX)
        return no("D at most 4096 and the local FFN width at most 8192, both multiples of 8");
    if ((m->T + kTlKS - 1) / kTlKS > kTlMaxSplits) return no("context at most 8192");
    auto pow2 = [](int k) { return k >= 8 && k <= 4096 && (k & (k - 1)) == 0; };
    if (!pow2(m->D) || !pow2(m->hq * kTlHD)) return no("D and the local q width must be powers of two (fixed column groups)");
    const int nwg = tpl_nwg();
    auto cdiv = [](long long a, long long b) { return (int)((a + b - 1) / b); };
    const int nrow = cdiv(m->D, nwg), nq = cdiv((long long)(m->hq + 2 * m->hkv) * (kTlHD / 2), nwg),
              ng = cdiv(m->Il, nwg);
    if (nrow > kTlMaxRows) return no("too many residual rows per workgroup");
    const long long need[] = {2LL * nq * (m->D / 8), (long long)nrow * m->hq * kTlHD / 8, 2LL * ng * (m->D / 8),
                              (long long)nrow * (m->Il / 8), (long long)kOsMaxRanks * nrow};
    for (long long n : need)
        if (n > kTlPartMax) return no("the per-workgroup shares exceed the kernel's LDS partial buffer (an unsharded 7B)");
    if (m->partial) {
        const bool wg = m->ar_mode == SLI_ALLREDUCE_FUSED_WG && m->os_open;
        const bool nocomm = !m->collectives && !m->os_open;
        if (!wg && !nocomm)
            return no("under tensor parallelism the exchange runs inside the launch: set_allreduce(fused_wg) first");
    }
    return 1;
}

static int tpl_alloc(sli_model* m) {
    if (m->tl.w) return SLI_OK;
    const int S = (m->T + kTlKS - 1) / kTlKS;
    const size_t n[6] = {(size_t)m->D, (size_t)(m->hq + 2 * m->hkv) * kTlHD, (size_t)m->hq * S * kTlPart,
                         (size_t)m->hq * kTlHD, (size_t)m->D, (size_t)m->Il};
    tl_u2** dst[6] = {&m->tl.g_x, &m->tl.g_qkv, &m->tl.g_part, &m->tl.g_att, &m->tl.g_x1, &m->tl.g_act};
    for (int i = 0; i < 6; ++i) {
        SLI_TRY(model_alloc(m, (void**)dst[i], 8 * n[i]));
        SLI_HIP(hipMemset(*dst[i], 0, 8 * n[i]));  // tag 0: never a launch's (epochs start at 1)
    }
    SLI_TRY(model_alloc(m, (void**)&m->tl.epoch, 16));
    SLI_HIP(hipMemset(m->tl.epoch, 0, 16));
    SLI_TRY(model_alloc(m, (void**)&m->tl.xg, sizeof(tl_u2*) * kOsMaxRanks));
    std::vector<const __half*> w(4 * (size_t)m->L);
    for (int l = 0; l < m->L; ++l) {
        w[4 * l + 0] = (const __half*)m->layers[l].qkv;
        w[4 * l + 1] = (const __half*)m->layers[l].wo;
        w[4 * l + 2] = (const __half*)m->layers[l].gu;
        w[4 * l + 3] = (const __half*)m->layers[l].down;
    }
    const __half** wd = nullptr;
    SLI_TRY(model_alloc(m, (void**)&wd, sizeof(void*) * w.size()));
    SLI_HIP(hipMemcpy(wd, w.data(), sizeof(void*) * w.size(), hipMemcpyHostToDevice));
    m->tl.w = wd;
    return SLI_OK;
}

// before a capture (no allocation or copy may run while the stream captures): buffers, and the device table of the
// ranks' exchange granules as currently mapped
static int tpl_prepare(sli_model* m) {
    std::string why;
    if (!tpl_check(m, &why)) return fail(SLI_ERR_STATE, "persistent layers: " + why);
    SLI_TRY(tpl_alloc(m));
    if (m->partial && m->os_open) {
        tl_u2* xg[kOsMaxRanks] = {};
        for (int r = 0; r < m->c.tp_size; ++r) xg[r] = (tl_u2*)(m->os_peer[r] + os_gran_off(m->os_nmax));
        SLI_HIP(hipMemcpy(m->tl.xg, xg, sizeof(xg), hipMemcpyHostToDevice));
    }
    return SLI_OK;
}

static int tpl_launch(sli_model* m) {
    std::string why;
    if (!tpl_check(m, &why) || !m->tl.w) return fail(SLI_ERR_STATE, "persistent layers: " + why);
    TlArgs a{};
    a.D = m->D;
    a.hq = m->hq;
    a.hkv = m->hkv;
    a.Il = m->Il;
    a.L = m->L;
    a.T = m->T;
    a.nwg = tpl_nwg();
    a.act_mode = m->c.act_mode;
    a.eps = m->c.eps;
    a.scale = 1.0f / sqrtf((float)kTlHD);
    a.w = m->tl.w;
    a.norms = m->norms;
    a.kc = (__half*)m->kc;
    a.vc = (__half*)m->vc;
    a.sin_t = m->sin_t;
    a.cos_t = m->cos_t;
    a.st = m->st;
    a.x = m->x;
    a.g_x = m->tl.g_x;
    a.g_qkv = m->tl.g_qkv;
    a.g_part = m->tl.g_part;
    a.g_att = m->tl.g_att;
    a.g_x1 = m->tl.g_x1;
    a.g_act = m->tl.g_act;
    a.epoch = m->tl.epoch;
    a.rank = m->c.tp_rank;
    a.nranks = m->c.tp_size;
    a.mode = !m->partial ? 0 : (m->os_open ? 2 : 1);
    a.loopback = m->os_loopback ? 1 : 0;
    a.xg = m->tl.xg;  // mode 2: every rank's exchange granules inside its comm buffer (tpl_prepare)
    const int G = m->hq / m->hkv;
    if (G == 1)
        hipLaunchKernelGGL(tp_layers_kernel<1>, dim3(a.nwg), dim3(kTlThreads), 0, m->stream, a);
    else if (G == 2)
        hipLaunchKernelGGL(tp_layers_kernel<2>, dim3(a.nwg), dim3(kTlThreads), 0, m->stream, a);
    else
        hipLaunchKernelGGL(tp_layers_kernel<4>, dim3(a.nwg), dim3(kTlThreads), 0, m->stream, a);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

template <typename WT, typename KT>
struct StepRecorder {
    static constexpr bool NT = true;  // streamed-once weights: non-temporal loads
    static int gemv_qkv(sli_model* m, int l) {
        const LayerW& w = m->layers[l];
        GemvIn in{m->x, m->norms + (size_t)(2 * l) * m->D, m->c.eps, m->D};
        KT* kc = (KT*)m->kc + (size_t)l * m->hkv * m->T * m->hd;
        KT* vc = (KT*)m->vc + (size_t)l * m->hkv * m->T * m->hd;
        EpiQKV<KT> e{m->q, kc, vc, w.qkv_s, &m->st->pos, m->sin_t, m->cos_t, m->hq, m->hkv, m->hd, m->T};
        SLI_HIP((launch_gemv_u<WT, 2, 4, NT>((const WT*)w.qkv, in, e, (m->hq + 2 * m->hkv) * (m->hd / 2), m->stream)));
        return SLI_OK;
    }
    // q/k/v + attention as one launch (qkv_attn.h) where the shape qualifies: *done = 1; 0: run the separate launches
    static int gemv_qkv_attn(sli_model* m, int l, int* done, bool dry = false) {
        *done = 0;
        if constexpr (std::is_same<KT, __half>::value && !std::is_same<WT, float>::value) {
            if (!m->qa_count || !qkv_attn_on(m)) return SLI_OK;
            const LayerW& w = m->layers[l];
            GemvIn in{m->x, m->norms + (size_t)(2 * l) * m->D, m->c.eps, m->D};
            const size_t lay = (size_t)l * m->hkv * m->T * m->hd;
            KT* kc = (KT*)m->kc + lay;
            KT* vc = (KT*)m->vc + lay;
            const int g = m->hq / m->hkv;
            EpiQKVHand<KT> e{{m->q, kc, vc, w.qkv_s, &m->st->pos, m->sin_t, m->cos_t, m->hq, m->hkv, m->hd, m->T},
                             m->qa_kv, m->qa_count, g};
            const int ppwg = attn_wg_positions(m->c.kv_dtype, m->hd);
            AttnArgs<KT> a{m->q, kc, vc, m->hd, (long long)m->T * m->hd, m->part, m->attn, m->attn_count, &m->st->pos, 0,
                           m->hkv, (m->T + ppwg - 1) / ppwg, 1.0f / sqrtf((float)m->hd), m->hkv, 0};
            a.defer_merge = m->wo_merge;
            a.hand_kv = m->qa_kv;
            a.hand_count = m->qa_count;
            a.hand_expect = (unsigned)((g + 2) * (m->hd / 2));
            a.hand_err = &m->st->error;
            const hipError_t r = launch_qkv_attn<WT, KT>((const WT*)w.qkv, in, e, a, (m->hq + 2 * m->hkv) * (m->hd / 2),
                                                         m->hd, m->stream, dry);
            if (r == hipErrorNotSupported) return SLI_OK;
            SLI_HIP(r);
            *done = 1;
        }
        return SLI_OK;
    }
    // wo + residual; its input is merged from the attention's split partials while it is staged
    // (attention launched with defer_merge, gemv.h XStageMerge)
    static int gemv_wo(sli_model* m, int l) {
        const LayerW& w = m->layers[l];
        if (m->wo_ks > 1) return gemv_wo_ks(m, l);
        const bool tp = m->partial;
        if (!m->wo_merge) {  // the attention merged its splits into attn: a plain input
            GemvIn in{m->attn, nullptr, 0.0f, m->hq * m->hd};
            if (fused_ar(m)) {
                SLI_HIP((launch_gemv_u<WT, 1, 2, NT>((const WT*)w.wo, in, push_epi(m, w.wo_s, 0), m->D, m->stream)));
                return SLI_OK;
            }
            EpiStore<1> e{tp ? m->xpart : m->x, (!tp || m->c.tp_rank == 0) ? m->x : nullptr, w.wo_s, 1.0f, m->D};
            SLI_HIP((launch_gemv_u<WT, 1, 2, NT>((const WT*)w.wo, in, e, m->D, m->stream)));
            return SLI_OK;
        }
        GemvIn in{m->attn, nullptr, 0.0f, m->hq * m->hd};
        EpiStore<1> e{tp ? m->xpart : m->x, (!tp || m->c.tp_rank == 0) ? m->x : nullptr, w.wo_s, 1.0f, m->D};
        const AttnMergeIn am{m->part, &m->st->pos, attn_max_splits(m), attn_wg_positions(m->c.kv_dtype, m->hd), m->hd};
        constexpr int UW = 2;  // int8 too (tools/gemv_lab i8: R1U2 7.5 us vs R1U1 7.95 on the 4096x4096 shape)
        if (fused_ar(m)) {
            const EpiPush<1> ep = push_epi(m, w.wo_s, 0);
            if (am.max_splits > 8)
                SLI_HIP((launch_gemv_merge<WT, 1, UW, NT, EpiPush<1>, 16>((const WT*)w.wo, in, ep, am, m->D, m->stream)));
            else
                SLI_HIP((launch_gemv_merge<WT, 1, UW, NT, EpiPush<1>>((const WT*)w.wo, in, ep, am, m->D, m->stream)));
            return SLI_OK;
        }
        // contexts past 8 splits (ctx > 2048 at hd 128 fp16): the 16-split input batch (ctx 4096 wo: 13.6 us
        // with splits 8..15 read one by one during the merge)
        if (am.max_splits > 8)
            SLI_HIP((launch_gemv_merge<WT, 1, UW, NT, EpiStore<1>, 16>((const WT*)w.wo, in, e, am, m->D, m->stream)));
        else
            SLI_HIP((launch_gemv_merge<WT, 1, UW, NT>((const WT*)w.wo, in, e, am, m->D, m->stream)));
        return SLI_OK;
    }
    // wo split over its columns (wo_ksplit): part[k][d] = wo[d][k-th column block] . attn[k-th block]
    static int gemv_wo_ks(sli_model* m, int l) {
        const LayerW& w = m->layers[l];
        const int ks = m->wo_ks;
        GemvIn in{m->attn, nullptr, 0.0f, m->hq * m->hd / ks};
        const EpiKPart e{m->wo_part, w.wo_s, m->D, ks};
        AttnMergeIn am{m->part, &m->st->pos, attn_max_splits(m), attn_wg_positions(m->c.kv_dtype, m->hd), m->hd};
        am.ksplit = ks;
        am.kunits = m->D;
        const int grid = gemv_ksplit_grid(m->D, ks);
        // U vectors per lane per step; NB steps in flight while the merge staging runs: fp16 4 (every step of the
        // wave's rows at C1: wo 9.42 -> 8.97 us, +0.4 % tok/s; 3 is slower, 9.66), int8 2 (4 measured no faster)
        // (profiles/r4_wo_nb_ab.txt)
        constexpr bool I8 = std::is_same<WT, int8_t>::value;
        constexpr int UK = I8 ? 1 : 2, NBK = I8 ? 2 : 4;
        if (am.max_splits > 8)
            SLI_HIP((launch_gemv_merge_ks<WT, 1, UK, NT, EpiKPart, 16, NBK>((const WT*)w.wo, in, e, am, grid, m->stream)));
        else
            SLI_HIP((launch_gemv_merge_ks<WT, 1, UK, NT, EpiKPart, 8, NBK>((const WT*)w.wo, in, e, am, grid, m->stream)));
        return SLI_OK;
    }
    static int attn_max_splits(sli_model* m) {
        const int ppwg = attn_wg_positions(m->c.kv_dtype, m->hd);
        return (m->T + ppwg - 1) / ppwg;
    }
    static int gemv_gu(sli_model* m, int l) {
        const LayerW& w = m->layers[l];
        GemvIn in{m->x, m->norms + (size_t)(2 * l + 1) * m->D, m->c.eps, m->D};
        EpiSwiGLU e{m->act, w.gu_s, m->Il, m->c.act_mode};
        if (m->wo_ks > 1) {  // stage x1 = x + the K-split wo's partials (XStageSum)
            constexpr int UG = std::is_same<WT, int8_t>::value ? 2 : 4;  // launch_gemv_u's unsplit U
            if (m->wo_ks == 2)
                SLI_HIP((launch_gemv_sum<WT, 2, UG, NT, EpiSwiGLU, 2>((const WT*)w.gu, in, e, m->wo_part, m->Il, m->stream)));
            else
                SLI_HIP((launch_gemv_sum<WT, 2, UG, NT, EpiSwiGLU, 4>((const WT*)w.gu, in, e, m->wo_part, m->Il, m->stream)));
            return SLI_OK;
        }
        SLI_HIP((launch_gemv_u<WT, 2, 4, NT>((const WT*)w.gu, in, e, m->Il, m->stream)));
        return SLI_OK;
    }
    static int gemv_down(sli_model* m, int l) {
        const LayerW& w = m->layers[l];
        const bool tp = m->partial;
        GemvIn in{m->act, nullptr, 0.0f, m->Il};
        if (fused_ar(m)) {
            const EpiPush<1> ep = push_epi(m, w.down_s, 1);
            if constexpr (std::is_same<WT, int8_t>::value)
                SLI_HIP((launch_gemv<WT, 1, 4, NT>((const WT*)w.down, in, ep, m->D, m->stream)));
            else
                SLI_HIP((launch_gemv_u<WT, 1, 6, NT>((const WT*)w.down, in, ep, m->D, m->stream)));
            return SLI_OK;
        }
        if (m->wo_ks == 2) return gemv_down_sum<2>(m, w, in);
        if (m->wo_ks == 4) return gemv_down_sum<4>(m, w, in);
        EpiStore<1> e{tp ? m->xpart : m->x, (!tp || m->c.tp_rank == 0) ? m->x : nullptr, w.down_s, 1.0f, m->D};
        if constexpr (std::is_same<WT, int8_t>::value)  // tools/gemv_lab i8: R1U4 11.66 us vs R1U3 11.74
            SLI_HIP((launch_gemv<WT, 1, 4, NT>((const WT*)w.down, in, e, m->D, m->stream)));
        else
            SLI_HIP((launch_gemv_u<WT, 1, 6, NT>((const WT*)w.down, in, e, m->D, m->stream)));
        return SLI_OK;
    }
    // down + residual x1 = x + the K-split wo's partials (EpiStoreSum: XStageSum's order), written to x
    template <int NP>
    static int gemv_down_sum(sli_model* m, const LayerW& w, const GemvIn& in) {
        const EpiStoreSum<1, NP> e{m->x, m->x, m->wo_part, w.down_s, m->D};
        if constexpr (std::is_same<WT, int8_t>::value)
            SLI_HIP((launch_gemv<WT, 1, 4, NT>((const WT*)w.down, in, e, m->D, m->stream)));
        else
            SLI_HIP((launch_gemv_u<WT, 1, 6, NT>((const WT*)w.down, in, e, m->D, m->stream)));
        return SLI_OK;
    }
    // the LM head launch's grid (its workgroups each write one argmax key): gemv_lm's split and blocks
    static int lm_head_blocks(sli_model* m) {
        const int units = (m->v_n + 1) / 2;
        const int cs = gemv_split<WT, 4>(units, m->D).cs;
        return cs == 1 ? gemv_balanced_blocks(units) : gemv_blocks(units, cs);  // launch_gemv's grid
    }
    static int gemv_lm(sli_model* m) {
        GemvIn in{m->x, m->norms + (size_t)(2 * m->L) * m->D, m->c.eps, m->D};
        EpiLogits<2> e{m->logits, m->keys, m->emb_s ? m->emb_s + m->v_lo : nullptr, m->v_n, m->v_lo, 0ull};
        const WT* w = (const WT*)m->emb + (size_t)m->v_lo * m->D;
        SLI_HIP((launch_gemv_u<WT, 2, 4, NT>(w, in, e, (m->v_n + 1) / 2, m->stream)));
        return SLI_OK;
    }
    // the residual all-reduce inside the wo / down launch (oneshot.h EpiPush), batch 1
    static bool fused_ar(const sli_model* m) {
        return m->partial && (m->ar_mode == SLI_ALLREDUCE_FUSED || m->ar_mode == SLI_ALLREDUCE_FUSED_WG);
    }
    // region: 0 for wo, 1 for down (FUSED_WG keeps their slots and per-workgroup epochs apart)
    static EpiPush<1> push_epi(sli_model* m, const float* rscale, int region) {
        OneShotArgs a{};
        for (int r = 0; r < m->c.tp_size; ++r) a.peers[r] = m->os_peer[r];
        a.rank = m->c.tp_rank;
        a.nranks = m->c.tp_size;
        a.n = m->D;
        a.nmax = m->os_nmax;
        a.src = nullptr;
        a.dst = m->x;
        a.epoch = m->os_epoch;
        a.st = m->st;
        a.loopback = m->os_loopback;
        EpiPush<1> e{m->c.tp_rank == 0 ? m->x : nullptr, rscale, 1.0f, m->D, a, m->os_epoch + 1, m->os_peer_tab};
        e.wg_mode = m->ar_mode == SLI_ALLREDUCE_FUSED_WG ? 1 : 0;
        e.region = region;
        e.wg_epoch = m->os_wg_epoch;
        return e;
    }
    static int oneshot(sli_model* m, const void* src, void* dst, int n, bool max_u64) {
        OneShotArgs a{};
        for (int r = 0; r < m->c.tp_size; ++r) a.peers[r] = m->os_peer[r];
        a.rank = m->c.tp_rank;
        a.nranks = m->c.tp_size;
        a.n = n;
        a.nmax = m->os_nmax;
        a.src = (const float*)src;
        a.dst = (float*)dst;
        a.epoch = m->os_epoch;
        a.st = m->st;
        a.loopback = m->os_loopback;
        if (max_u64)  // the argmax keys: 2 * B u64s, one workgroup
            hipLaunchKernelGGL(oneshot_kernel<1>, dim3(1), dim3(1024), 0, m->stream, a);
        else  // the residual sums: sliced over kOsSliceWgs workgroups
            hipLaunchKernelGGL(oneshot_sliced_kernel, dim3(std::min(kOsSliceWgs, std::max(1, n / 64))), dim3(256), 0,
                               m->stream, a, m->os_peer_tab, m->os_wg_epoch);
        SLI_HIP(hipGetLastError());
        return SLI_OK;
    }
    static int allreduce_x(sli_model* m) {
        const size_t n = (size_t)m->B * m->D;
        if (fused_ar(m)) return SLI_OK;  // done inside the wo / down launch
        if (m->ar_mode == SLI_ALLREDUCE_ONESHOT) return oneshot(m, m->xpart, m->x, (int)n, false);
        if (m->collectives)
            SLI_NCCL(ncclAllReduce(m->xpart, m->x, n, ncclFloat32, ncclSum, m->comm, m->stream));
        else if (m->partial)  // debug no-comm mode: keep the local partial as the residual stream
            SLI_HIP(hipMemcpyAsync(m->x, m->xpart, sizeof(float) * n, hipMemcpyDeviceToDevice, m->stream));
        return SLI_OK;
    }

    // ---- batch > 1: the same step for B sequences, projections on MFMA (bgemm.h)
    static constexpr int kPosStride = (int)(sizeof(DevState) / sizeof(int32_t));
    template <class Epi>
    static int bg(sli_model* m, const void* W, const BgIn& in, const Epi& e, const BgPlan& p) {
        if constexpr (std::is_same<WT, __half>::value) {
            SLI_HIP(launch_bgemm((const __half*)W, in, e, p, m->stream));
            return SLI_OK;
        } else {
            return fail(SLI_ERR_ARG, "batch > 1 needs fp16 weights");
        }
    }
    template <class Epi, bool NORM>
    static int allow(sli_model*) {
        if constexpr (std::is_same<WT, __half>::value) SLI_HIP((bg_allow_lds<Epi, NORM>()));
        return SLI_OK;
    }
    // raise the LDS limit of every batched kernel once, before any capture
    static int prepare(sli_model* m) {
        SLI_TRY((allow<BgEpiQKV<KT>, true>(m)));
        SLI_TRY((allow<BgEpiStore, false>(m)));
        SLI_TRY((allow<BgEpiPush, false>(m)));
        SLI_TRY((allow<BgEpiSwiGLU, true>(m)));
        SLI_TRY((allow<BgEpiLogits, true>(m)));
        return SLI_OK;
    }
    static BgIn bin(sli_model* m, const float* x, const float* norm, int K) {
        BgIn in{};
        in.x = x;
        in.norm_w = norm;
        in.eps = m->c.eps;
        in.K = K;
        in.B = m->B;
        in.ws = m->bg_ws;
        in.counters = m->bg_cnt;
        in.tiled = m->bg_tiled ? 1 : 0;
        return in;
    }
    static int b_qkv(sli_model* m, int l) {
        const size_t lay = (size_t)l * m->B * m->hkv * m->T * m->hd;
        BgEpiQKV<KT> e{m->q, (KT*)m->kc + lay, (KT*)m->vc + lay, &m->st->pos, kPosStride, m->sin_t, m->cos_t,
                       m->hq, m->hkv, m->hd, m->T};
        return bg(m, m->bg_tiled ? m->layers[l].qkv_t : m->layers[l].qkv, bin(m, m->x, m->norms + (size_t)(2 * l) * m->D, m->D), e, m->bp_qkv);
    }
    // batched wo / down with the exchange per group (oneshot.h BgEpiPush; region 3: wo, 4: down)
    static BgEpiPush push_bg(sli_model* m, int region, const BgPlan& p) {
        BgEpiPush e{};
        e.resid = m->c.tp_rank == 0 ? m->x : nullptr;
        for (int r = 0; r < m->c.tp_size; ++r) e.os.peers[r] = m->os_peer[r];
        e.os.rank = m->c.tp_rank;
        e.os.nranks = m->c.tp_size;
        e.os.n = m->B * m->D;
        e.os.nmax = m->os_nmax;
        e.os.dst = m->x;
        e.os.epoch = m->os_epoch;
        e.os.st = m->st;
        e.os.loopback = m->os_loopback;
        e.peer_tab = m->os_peer_tab;
        e.wg_epoch = m->os_wg_epoch;
        e.region = region;
        e.nrows = m->D;
        e.ld = m->D;
        e.B = m->B;
        e.tpw = p.tpw;
        e.ntiles = p.ntiles;
        return e;
    }
    static int b_wo(sli_model* m, int l) {
        const bool tp = m->partial;
        const void* w = m->bg_tiled ? m->layers[l].wo_t : m->layers[l].wo;
        if (fused_ar(m)) return bg(m, w, bin(m, m->attn, nullptr, m->hq * m->hd), push_bg(m, 3, m->bp_wo), m->bp_wo);
        BgEpiStore e{tp ? m->xpart : m->x, (!tp || m->c.tp_rank == 0) ? m->x : nullptr, nullptr, 1.0f, m->D, m->D};
        return bg(m, w, bin(m, m->attn, nullptr, m->hq * m->hd), e, m->bp_wo);
    }
    static int b_gu(sli_model* m, int l) {
        BgEpiSwiGLU e{m->act, m->Il, m->c.act_mode};
        return bg(m, m->bg_tiled ? m->layers[l].gu_t : m->layers[l].gu, bin(m, m->x, m->norms + (size_t)(2 * l + 1) * m->D, m->D), e, m->bp_gu);
    }
    static int b_down(sli_model* m, int l) {
        const bool tp = m->partial;
        const void* w = m->bg_tiled ? m->layers[l].down_t : m->layers[l].down;
        if (fused_ar(m)) return bg(m, w, bin(m, m->act, nullptr, m->Il), push_bg(m, 4, m->bp_down), m->bp_down);
        BgEpiStore e{tp ? m->xpart : m->x, (!tp || m->c.tp_rank == 0) ? m->x : nullptr, nullptr, 1.0f, m->D, m->D};
        return bg(m, w, bin(m, m->act, nullptr, m->Il), e, m->bp_down);
    }
    static int b_lm(sli_model* m) {
        BgEpiLogits e{m->logits, m->keys, m->v_n, m->v_n, m->v_lo, m->key_ld};
        const void* w = m->bg_tiled ? m->lm_t : wptr(m->emb, m->wbytes, (size_t)m->v_lo * m->D);
        return bg(m, w, bin(m, m->x, m->norms + (size_t)(2 * m->L) * m->D, m->D), e, m->bp_lm);
    }
    // ---- one step = phases 0 .. 2L (model.cpp:48-139). Phase 2l: [embedding when l = 0,] qkv(l),
    // attention(l), wo(l); phase 2l+1: gate/up(l), down(l); phase 2L: LM head + first argmax stage.
    // Under tensor parallelism phases 0 .. 2L-1 end with the sum all-reduce of the residual stream and
    // phase 2L with the argmax-key MAX exchange; the communicator's recorder (record: none / RCCL;
    // record_group: the in-process group) places those between the phases.
    static int record_phase(sli_model* m, int p) {
        hipStream_t s = m->stream;
        const bool batched = m->B > 1;
        if (p == 0) {
            if (batched) {
                const int eb = std::min(64, (m->D + 255) / 256);
                hipLaunchKernelGGL(embedding_batch_kernel<WT>, dim3(eb, m->B), dim3(256), 0, s, m->st,
                                   (const WT*)m->emb, m->emb_s, m->x, m->V, m->D);
                SLI_HIP(hipGetLastError());
            } else {
                SLI_TRY(embedding_launch(0, &m->st->token, m->emb, m->c.w_dtype, m->emb_s, m->x, m->V, m->D, s));
            }
        }
        if (p >= 2 * m->L) return record_head(m, true);
        const int l = p / 2;
        if (p % 2 == 0) {
            const long long ps = m->hd, hs = (long long)m->T * m->hd;
            const long long ls = (long long)m->B * m->hkv * m->T * m->hd;
            int fused = 0;
            if (!batched) SLI_TRY(gemv_qkv_attn(m, l, &fused));
            if (fused == 1) return gemv_wo(m, l);
            SLI_TRY(batched ? b_qkv(m, l) : gemv_qkv(m, l));
            // a batch is B * hkv kv heads of one layer: sequence b owns kv heads [b*hkv, (b+1)*hkv)
            SLI_TRY(mha_launch<KT>(m->q, (const KT*)m->kc, (const KT*)m->vc, m->attn, l, 0, &m->st->pos, m->T, m->hd,
                                   m->B * m->hq, m->B * m->hkv, ps, hs, ls, m->part, m->attn_count, s,
                                   batched ? m->hkv : 0, batched ? kPosStride : 0, 0, batched ? kDeferBatched : m->wo_merge));
            return batched ? b_wo(m, l) : gemv_wo(m, l);
        }
        SLI_TRY(batched ? b_gu(m, l) : gemv_gu(m, l));
        return batched ? b_down(m, l) : gemv_down(m, l);
    }
    // LM head + first argmax stage. exchange = false: the step has no cross-rank key exchange, so batch 1
    // fuses the key reduce with the state update (one launch).
    static int record_head(sli_model* m, bool exchange) {
        hipStream_t s = m->stream;
        if (m->B > 1) {
            SLI_TRY(b_lm(m));
            hipLaunchKernelGGL(keyreduce_batch_kernel, dim3(m->B), dim3(256), 0, s, m->keys, m->key_ld,
                               m->bp_lm.groups, m->bkeys);
            SLI_HIP(hipGetLastError());
            return SLI_OK;
        }
        SLI_TRY(gemv_lm(m));
        if (exchange)
            hipLaunchKernelGGL(keyreduce_kernel<false>, dim3(1), dim3(kKeyThreads), 0, s, m->keys, lm_head_blocks(m),
                               m->st, m->prompt, m->hist, m->T);
        else
            hipLaunchKernelGGL(keyreduce_kernel<true>, dim3(1), dim3(kKeyThreads), 0, s, m->keys, lm_head_blocks(m),
                               m->st, m->prompt, m->hist, m->T);
        SLI_HIP(hipGetLastError());
        return SLI_OK;
    }
    // state update after the (exchanged) argmax keys: position, next token, history (model.cpp:157-183)
    static int record_finalize(sli_model* m) {
        hipStream_t s = m->stream;
        if (m->B > 1)
            hipLaunchKernelGGL(finalize_batch_kernel, dim3(1), dim3(64), 0, s, m->st, m->bkeys, m->prompt, m->hist,
                               m->T, m->B);
        else
            hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(1), 0, s, m->st, m->prompt, m->hist, m->T);
        SLI_HIP(hipGetLastError());
        return SLI_OK;
    }

    // one model and its own communicator (none, RCCL, or the debug modes)
    static int record(sli_model* m) {
        if (m->exec == SLI_EXEC_PERSIST) {  // embedding, then every layer in one persistent launch (tp_layers.h)
            if constexpr (!std::is_same<WT, __half>::value || !std::is_same<KT, __half>::value)
                return fail(SLI_ERR_STATE, "persistent layers: fp16 weights and K/V cache only");
            SLI_TRY(embedding_launch(0, &m->st->token, m->emb, m->c.w_dtype, m->emb_s, m->x, m->V, m->D, m->stream));
            SLI_TRY(tpl_launch(m));
        } else {
            for (int p = 0; p < 2 * m->L; ++p) {
                SLI_TRY(record_phase(m, p));
                SLI_TRY(allreduce_x(m));
            }
        }
        if (m->ar_mode != SLI_ALLREDUCE_RCCL) {  // the argmax keys through the one-shot exchange
            SLI_TRY(record_head(m, true));
            void* k = m->B > 1 ? (void*)m->bkeys : (void*)&m->st->key;
            SLI_TRY(oneshot(m, k, k, 2 * m->B, true));
            return record_finalize(m);
        }
        if (!m->collectives) {
            SLI_TRY(record_head(m, m->B > 1));
            return m->B > 1 ? record_finalize(m) : SLI_OK;
        }
        SLI_TRY(record_head(m, true));
        if (m->B > 1)
            SLI_NCCL(ncclAllReduce(m->bkeys, m->bkeys, m->B, ncclUint64, ncclMax, m->comm, m->stream));
        else
            SLI_NCCL(ncclAllReduce(&m->st->key, &m->st->key, 1, ncclUint64, ncclMax, m->comm, m->stream));
        return record_finalize(m);
    }
    // the in-process group: phase p of every rank, then the device-side collective (sli_tp_group)
    static int record_group(sli_tp_group* g) {
        sli_model* m0 = g->ranks[0];
        const int n = g->n;
        GroupSumArgs sa{};
        sa.n_ranks = n;
        sa.n = m0->B * m0->D;
        sa.f16_payload = getenv("SLI_DEBUG_AR_F16") ? 1 : 0;
        GroupKeyArgs ka{};
        ka.n_ranks = n;
        ka.B = m0->B;
        ka.T = m0->T;
        for (int r = 0; r < n; ++r) {
            sli_model* m = g->ranks[r];
            sa.src[r] = m->xpart;
            sa.dst[r] = m->x;
            ka.key[r] = m->B > 1 ? m->bkeys : &m->st->key;
            ka.st[r] = m->st;
            ka.prompt[r] = m->prompt;
            ka.hist[r] = m->hist;
        }
        const int blocks = std::min(64, (sa.n + 255) / 256);
        for (int p = 0; p < 2 * m0->L; ++p) {
            for (int r = 0; r < n; ++r) SLI_TRY(record_phase(g->ranks[r], p));
            hipLaunchKernelGGL(group_sum_kernel, dim3(blocks), dim3(256), 0, g->stream, sa);
            SLI_HIP(hipGetLastError());
        }
        for (int r = 0; r < n; ++r) SLI_TRY(record_head(g->ranks[r], true));
        hipLaunchKernelGGL(group_finalize_kernel, dim3(1), dim3(64), 0, g->stream, ka);
        SLI_HIP(hipGetLastError());
        return SLI_OK;
    }
    // ---- prompt prefill (model.cpp:157-165 runs the prompt one token per forward; prefill.h): a chunk of
    // M prompt positions runs through every layer together, each projection one MFMA GEMM over the chunk
    // (weights read once per BM positions), attention block-causal over the cache rows the chunk's own qkv
    // GEMM just wrote. No LM head: the prompt's logits are not used (teacher forcing); the last prompt
    // position runs as an ordinary decode step. Phases as record_phase: 2l = qkv, attention, wo; 2l+1 =
    // gate/up, down; under tensor parallelism each ends with the all-reduce of the chunk's residual rows.
    template <class Epi, class Cfg>
    static int pg_cfg(sli_model* m, const void* W, int N, int K, const __half* hi, const __half* lo, const Epi& e,
                      int M) {
        if constexpr (std::is_same<WT, float>::value) {
            return fail(SLI_ERR_ARG, "prefill needs fp16 or int8 weights");
        } else {
            const PgIn<WT> in{(const WT*)W, hi, lo, N, K, M};
            SLI_HIP((launch_pgemm<Epi, Cfg, WT>(in, e, m->pf.ps, m->stream)));
            return SLI_OK;
        }
    }
    // The GEMM tiling (prefill.h PgCfg<BM, WR, S, AT, PIPE>) per weight type, projection role and chunk size: the
    // fastest of the tools/pgemm_lab sweeps on the 7B shapes (profiles/r3_pgemm_lab.txt; round 6: the pipelined
    // fragment reads, 5-20 % faster at every tiling, the M = 128 choices, profiles/r6b_pg_pipe.txt, and the M = 256
    // ones re-timed with the weights streamed from HBM as in the engine, profiles/r6b_pg_cold.txt).
    // role 0: qkv, 1: gate/up, 2: wo / down (N = D: few row blocks, so small chunk blocks for a full grid).
    // f(PgCfg<...>{}) is called with the chosen tiling (pg launches it, allow_pg sets its LDS limit).
    template <class F>
    static int pg_pick(int M, int role, F&& f) {
        if constexpr (std::is_same<WT, int8_t>::value) {
            if (M == 32) return f(PgCfg<32, 2, 4, 2, true>{});
            if (role == 2) return M == 256 ? f(PgCfg<64, 2, 2, 2, true>{}) : f(PgCfg<32, 2, 4, 2, true>{});
            if (role == 1) return M == 128 ? f(PgCfg<128, 4, 2, 2, true>{}) : f(PgCfg<64, 4, 2, 2, true>{});
            return M == 256 ? f(PgCfg<128, 4, 2, 2, true>{}) : f(PgCfg<64, 4, 2, 2, true>{});
        } else {
            if (M == 32) return f(PgCfg<32, 2, 4, 2, true>{});
            if (role == 2) return M == 256 ? f(PgCfg<64, 2, 3, 2, true>{}) : f(PgCfg<32, 2, 4, 2, true>{});
            if (M == 64 || (M == 128 && role == 0)) return f(PgCfg<64, 2, 3, 2, true>{});
            // M = 256 with the weights streamed from HBM (profiles/r6b_pg_cold.txt): 8-wave workgroups
            // (q/k/v: the weights in a 4-deep ring of their own, profiles/r6b_pg_split.txt)
            if (M == 256) return role == 0 ? f(PgCfg<128, 4, 2, 2, true, 4>{}) : f(PgCfg<64, 4, 3, 2, true>{});
            return f(PgCfg<128, 2, 2, 2, true>{});
        }
    }
    template <class Epi>
    static int pg(sli_model* m, const void* W, int N, int K, const __half* hi, const __half* lo, const Epi& e, int M,
                  int role) {
        return pg_pick(M, role, [&](auto cfg) { return pg_cfg<Epi, decltype(cfg)>(m, W, N, K, hi, lo, e, M); });
    }
    template <class Epi>
    static int allow_pg(sli_model*) {
        if constexpr (std::is_same<WT, int8_t>::value || std::is_same<WT, __half>::value) {
            for (int M : {32, 64, 128, 256})
                for (int role = 0; role < 3; ++role)
                    SLI_TRY(pg_pick(M, role, [&](auto cfg) -> int {
                        SLI_HIP((pgemm_allow_lds<Epi, decltype(cfg), WT>()));
                        return SLI_OK;
                    }));
        }
        return SLI_OK;
    }
    static int prepare_prefill(sli_model* m) {
        SLI_TRY(allow_pg<PgEpiQKV<KT>>(m));
        SLI_TRY(allow_pg<PgEpiResid>(m));
        SLI_TRY(allow_pg<PgEpiSwiGLU>(m));
        return SLI_OK;
    }
    static int record_pf_phase(sli_model* m, int p, int M) {
        auto& f = m->pf;
        hipStream_t s = m->stream;
        const int D = m->D, hd = m->hd, QD = m->hq * hd;
        if (p == 0) {
            hipLaunchKernelGGL(pf_embed_kernel<WT>, dim3(M), dim3(256), 0, s, f.ps, m->prompt, (const WT*)m->emb,
                               m->emb_s, f.x, D);
            SLI_HIP(hipGetLastError());
        }
        const int l = p / 2;
        const LayerW& w = m->layers[l];
        const bool tp = m->partial;
        PgEpiResid er{tp ? f.xpart : f.x, (!tp || m->c.tp_rank == 0) ? f.x : nullptr, nullptr, D, D};
        hipLaunchKernelGGL(pf_norm_split_kernel, dim3(M), dim3(256), 0, s, f.x, m->norms + (size_t)p * D, f.hhi, f.hlo,
                           D, m->c.eps);
        SLI_HIP(hipGetLastError());
        if (p % 2 == 0) {
            const size_t ls = (size_t)l * m->hkv * m->T * hd;
            PgEpiQKV<KT> eq{f.q, (KT*)m->kc + ls, (KT*)m->vc + ls, w.qkv_s, m->sin_t, m->cos_t, m->hq, m->hkv, hd, m->T};
            SLI_TRY(pg(m, w.qkv, (m->hq + 2 * m->hkv) * hd, D, f.hhi, f.hlo, eq, M, 0));
            PfAttnArgs<KT> aa{f.q, (const KT*)m->kc + ls, (const KT*)m->vc + ls, f.hhi, f.hlo, m->hq, m->hkv, m->T,
                              1.0f / sqrtf((float)hd)};
            if constexpr (std::is_same<KT, __half>::value) {  // MFMA, 16 chunk rows per workgroup
                const dim3 ag(M / 16, m->hq);
                if (hd == 128)
                    hipLaunchKernelGGL((pf_attn_mfma_kernel<128>), ag, dim3(256), 0, s, aa, f.ps);
                else
                    hipLaunchKernelGGL((pf_attn_mfma_kernel<64>), ag, dim3(256), 0, s, aa, f.ps);
            } else {  // fp32 cache: fp32 VALU, 64 chunk rows per workgroup
                const dim3 ag((M + kPaQB - 1) / kPaQB, m->hq);
                if (hd == 128)
                    hipLaunchKernelGGL((pf_attn_kernel<KT, 128>), ag, dim3(256), 0, s, aa, f.ps);
                else
                    hipLaunchKernelGGL((pf_attn_kernel<KT, 64>), ag, dim3(256), 0, s, aa, f.ps);
            }
            SLI_HIP(hipGetLastError());
            er.rscale = w.wo_s;
            return pg(m, w.wo, D, QD, f.hhi, f.hlo, er, M, 2);
        }
        PgEpiSwiGLU eg{f.ahi, f.alo, w.gu_s, m->Il, m->c.act_mode};
        SLI_TRY(pg(m, w.gu, 2 * m->Il, D, f.hhi, f.hlo, eg, M, 1));
        er.rscale = w.down_s;
        return pg(m, w.down, D, m->Il, f.ahi, f.alo, er, M, 2);
    }
    static int record_prefill(sli_model* m, int M) {
        for (int p = 0; p < 2 * m->L; ++p) {
            SLI_TRY(record_pf_phase(m, p, M));
            const size_t n = (size_t)M * m->D;
            if (m->collectives)
                SLI_NCCL(ncclAllReduce(m->pf.xpart, m->pf.x, n, ncclFloat32, ncclSum, m->comm, m->stream));
            else if (m->partial)  // debug no-comm mode: keep the local partial as the residual stream
                SLI_HIP(hipMemcpyAsync(m->pf.x, m->pf.xpart, sizeof(float) * n, hipMemcpyDeviceToDevice, m->stream));
        }
        return SLI_OK;
    }
    static int record_group_prefill(sli_tp_group* g, int M) {
        sli_model* m0 = g->ranks[0];
        GroupSumArgs sa{};
        sa.n_ranks = g->n;
        sa.n = M * m0->D;
        for (int r = 0; r < g->n; ++r) {
            sa.src[r] = g->ranks[r]->pf.xpart;
            sa.dst[r] = g->ranks[r]->pf.x;
        }
        const int blocks = std::min(256, (sa.n + 255) / 256);
        for (int p = 0; p < 2 * m0->L; ++p) {
            for (int r = 0; r < g->n; ++r) SLI_TRY(record_pf_phase(g->ranks[r], p, M));
            hipLaunchKernelGGL(group_sum_kernel, dim3(blocks), dim3(256), 0, g->stream, sa);
            SLI_HIP(hipGetLastError());
        }
        return SLI_OK;
    }
    // All weight-streaming launches of one step (for the roofline probe).
    static int gemvs(sli_model* m) {
        if (m->B > 1) {
            for (int l = 0; l < m->L; ++l) {
                SLI_TRY(b_qkv(m, l));
                SLI_TRY(b_wo(m, l));
                SLI_TRY(b_gu(m, l));
                SLI_TRY(b_down(m, l));
            }
            return b_lm(m);
        }
        for (int l = 0; l < m->L; ++l) {
            SLI_TRY(gemv_qkv(m, l));
            SLI_TRY(gemv_wo(m, l));
            SLI_TRY(gemv_gu(m, l));
            SLI_TRY(gemv_down(m, l));
        }
        return gemv_lm(m);
    }
    // The launches of one kernel family in one step (for the per-family timing probe): every layer's
    // qkv / attention / wo / gate-up / down launch, or the LM head.
    static int family(sli_model* m, int f) {
        const bool batched = m->B > 1;
        if (f == SLI_FAM_LM) return batched ? b_lm(m) : gemv_lm(m);
        for (int l = 0; l < m->L; ++l) {
            switch (f) {
                case SLI_FAM_QKV: SLI_TRY(batched ? b_qkv(m, l) : gemv_qkv(m, l)); break;
                case SLI_FAM_ATTN: {
                    const long long ps = m->hd, hs = (long long)m->T * m->hd;
                    const long long ls = (long long)m->B * m->hkv * m->T * m->hd;
                    SLI_TRY(mha_launch<KT>(m->q, (const KT*)m->kc, (const KT*)m->vc, m->attn, l, 0, &m->st->pos, m->T,
                                           m->hd, m->B * m->hq, m->B * m->hkv, ps, hs, ls, m->part, m->attn_count,
                                           m->stream, batched ? m->hkv : 0, batched ? kPosStride : 0, 0,
                                           batched ? kDeferBatched : m->wo_merge));
                    break;
                }
                case SLI_FAM_WO: SLI_TRY(batched ? b_wo(m, l) : gemv_wo(m, l)); break;
                case SLI_FAM_GU: SLI_TRY(batched ? b_gu(m, l) : gemv_gu(m, l)); break;
                case SLI_FAM_DOWN: SLI_TRY(batched ? b_down(m, l) : gemv_down(m, l)); break;
                default: return fail(SLI_ERR_ARG, "unknown kernel family");
            }
        }
        return SLI_OK;
    }
    static int fill_kv(sli_model* m, uint32_t seed, int upto) {
        const uint64_t n = (uint64_t)m->L * m->B * m->hkv * upto * m->hd;
        const int blocks = (int)std::min<uint64_t>(4096, (n + 255) / 256);
        hipLaunchKernelGGL(fill_kv_kernel<KT>, dim3(blocks), dim3(256), 0, m->stream, (KT*)m->kc, (KT*)m->vc, m->L,
                           m->B, m->hkv, m->T, m->hd, upto, m->c.n_kv_heads * m->hd, m->c.tp_rank * m->hkv, seed,
                           SLI_SYNTH_C(1.0));
        SLI_HIP(hipGetLastError());
        return SLI_OK;
    }
    static int get_kv(sli_model* m, int seq, int layer, int which, int upto, float* tmp) {
        const KT* base = (const KT*)(which == 0 ? m->kc : m->vc) + ((size_t)layer * m->B + seq) * m->hkv * m->T * m->hd;
        hipLaunchKernelGGL(get_kv_kernel<KT>, dim3(256), dim3(256), 0, m->stream, base, tmp, m->hkv, m->T, m->hd, upto);
        SLI_HIP(hipGetLastError());
        return SLI_OK;
    }
};

#define SLI_DISPATCH(m, FN, ...)                                                                        \
    ([&]() -> int {                                                                                     \
        const int wd = (m)->c.w_dtype, kd = (m)->c.kv_dtype;                                            \
        if (wd == SLI_DT_F16 && kd == SLI_DT_F16) return StepRecorder<__half, __half>::FN(__VA_ARGS__); \
        if (wd == SLI_DT_F16 && kd == SLI_DT_F32) return StepRecorder<__half, float>::FN(__VA_ARGS__);  \
        if (wd == SLI_DT_F32 && kd == SLI_DT_F16) return StepRecorder<float, __half>::FN(__VA_ARGS__);  \
        if (wd == SLI_DT_F32 && kd == SLI_DT_F32) return StepRecorder<float, float>::FN(__VA_ARGS__);   \
        if (wd == SLI_DT_I8 && kd == SLI_DT_F16) return StepRecorder<int8_t, __half>::FN(__VA_ARGS__);  \
        return StepRecorder<int8_t, float>::FN(__VA_ARGS__);                                            \
    })()

template <class Rec>
static int capture_graph(hipStream_t stream, hipGraph_t& graph, hipGraphExec_t& exec, Rec record) {
    if (exec) return SLI_OK;
    SLI_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed));
    int rc = record();
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(stream, &g);
    if (rc != SLI_OK) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (e != hipSuccess) return hip_fail(e, "hipStreamEndCapture");
    graph = g;
    SLI_HIP(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
    return SLI_OK;
}

// (Re)build the fragment-layout copies of the batched projections from the row-major matrices after weights
// were placed (bgemm.h bg_tile_kernel; each epilogue's row order), on the model's stream before any use
static int bg_sync_tiles(sli_model* m) {
    if (!m->bg_tiled || !m->tiles_dirty) return SLI_OK;
    const int D = m->D, hd = m->hd, QD = m->hq * hd;
    hipStream_t s = m->stream;
    BgEpiQKV<__half> eq{};
    eq.hq = m->hq;
    eq.hkv = m->hkv;
    eq.hd = hd;
    BgEpiStore eo{};
    eo.nrows = D;
    BgEpiSwiGLU eg{};
    eg.inter = m->Il;
    BgEpiLogits el{};
    el.nrows = m->v_n;
    for (const LayerW& w : m->layers) {
        SLI_HIP(launch_bg_tile((const __half*)w.qkv, D, m->bp_qkv.ntiles, eq, w.qkv_t, s));
        SLI_HIP(launch_bg_tile((const __half*)w.wo, QD, m->bp_wo.ntiles, eo, w.wo_t, s));
        SLI_HIP(launch_bg_tile((const __half*)w.gu, D, m->bp_gu.ntiles, eg, w.gu_t, s));
        SLI_HIP(launch_bg_tile((const __half*)w.down, m->Il, m->bp_down.ntiles, eo, w.down_t, s));
    }
    SLI_HIP(launch_bg_tile((const __half*)m->emb + (size_t)m->v_lo * D, D, m->bp_lm.ntiles, el, m->lm_t, s));
    m->tiles_dirty = false;
    return SLI_OK;
}

static int capture(sli_model* m) {
    if (m->comm_dead) return fail(SLI_ERR_COMM, "the RCCL communicator was aborted by an earlier bounded wait");
    SLI_TRY(bg_sync_tiles(m));
    if (m->exec == SLI_EXEC_PERSIST && !m->graph_exec) SLI_TRY(tpl_prepare(m));
    return capture_graph(m->stream, m->graph, m->graph_exec, [&]() { return SLI_DISPATCH(m, record, m); });
}

// The ranks share the group's stream, so a tile rebuild (bg_sync_tiles, only after a weight was placed) is ordered
// after any group graph still running on it and before the next one; nothing to wait for on a plain step.
static int capture_group(sli_tp_group* g) {
    sli_model* m0 = g->ranks[0];
    for (sli_model* r : g->ranks) SLI_TRY(bg_sync_tiles(r));
    return capture_graph(g->stream, g->graph, g->exec, [&]() { return SLI_DISPATCH(m0, record_group, g); });
}

// ---- bounded host waits (comm_wait.h): a rank whose step holds RCCL collectives never blocks in
// hipStreamSynchronize on a wedged peer; it polls the stream / event, ncclCommGetAsyncError and a deadline, and on
// failure aborts the communicator (its kernels and proxy threads end) and reports which rank gave up and why.
static int comm_abort(sli_model* m, int code, const std::string& why) {
    if (m->comm) (void)ncclCommAbort(m->comm);
    m->comm = nullptr;
    m->comm_dead = true;
    return fail(code, "tp rank " + std::to_string(m->c.tp_rank) + "/" + std::to_string(m->c.tp_size) + ": " + why);
}
template <class Query>
static int wait_bounded(sli_model* m, Query query) {
    std::string why;
    const int rc = bounded_wait(
        [&] {
            const hipError_t e = query();
            return e == hipSuccess ? WaitPoll::Done : e == hipErrorNotReady ? WaitPoll::Pending : WaitPoll::Failed;
        },
        [&](std::string& msg) {
            ncclResult_t r = ncclSuccess;
            if (ncclCommGetAsyncError(m->comm, &r) != ncclSuccess) {
                msg = "ncclCommGetAsyncError failed";
                return true;
            }
            if (r == ncclSuccess || r == ncclInProgress) return false;
            msg = ncclGetErrorString(r);
            return true;
        },
        steady_ms, comm_timeout_ms(), why);
    if (rc == SLI_OK) return SLI_OK;
    if (rc == SLI_ERR_HIP) return hip_fail(query(), why.c_str());
    return comm_abort(m, rc, why);
}
static int wait_stream(sli_model* m) {
    if (m->comm_dead) return fail(SLI_ERR_COMM, "the RCCL communicator was aborted by an earlier bounded wait");
    if (!m->comm) {
        SLI_HIP(hipStreamSynchronize(m->stream));
        return SLI_OK;
    }
    return wait_bounded(m, [&] { return hipStreamQuery(m->stream); });
}
static int wait_event(sli_model* m, hipEvent_t e) {
    if (m->comm_dead) return fail(SLI_ERR_COMM, "the RCCL communicator was aborted by an earlier bounded wait");
    if (!m->comm) {
        SLI_HIP(hipEventSynchronize(e));
        return SLI_OK;
    }
    return wait_bounded(m, [&] { return hipEventQuery(e); });
}

static int upload_states(sli_model* m, const std::vector<DevState>& h) {
    SLI_HIP(hipMemcpyAsync(m->st, h.data(), sizeof(DevState) * m->B, hipMemcpyHostToDevice, m->stream));
    SLI_TRY(wait_stream(m));
    return SLI_OK;
}

static int download_states(sli_model* m, std::vector<DevState>& h) {
    h.resize(m->B);
    SLI_HIP(hipMemcpyAsync(h.data(), m->st, sizeof(DevState) * m->B, hipMemcpyDeviceToHost, m->stream));
    SLI_TRY(wait_stream(m));
    return SLI_OK;
}

// Device-side error bits (DevState::error: a bounded spin of the one-shot all-reduce or of the fused q/k/v +
// attention hand-off gave up, leaving stale outputs) surfaced as a status: every predict path calls this after its
// final stream sync, so a step that returned early never yields SLI_OK with garbage tokens.
static int check_device_errors(sli_model* m) {
    std::vector<DevState> h;
    SLI_TRY(download_states(m, h));
    int bits = 0;
    for (const DevState& d : h) bits |= d.error;
    if (bits == 0) return SLI_OK;
    if (bits & kOsErrTimeout) m->os_dead = true;  // epochs may disagree across ranks from here on
    if (bits & kAttnErrHand) {
        // a hand-off wait gave up: late q/k/v workgroups may have added their counts after the head's last attention
        // workgroup reset them, and the next step's waits would pass early on that residue. Start them from zero.
        if (m->qa_count) (void)hipMemsetAsync(m->qa_count, 0, sizeof(unsigned) * attn_hand_words(m->hkv), m->stream);
        (void)hipMemsetAsync(m->attn_count, 0, sizeof(unsigned) * m->B * m->hkv, m->stream);
        (void)hipStreamSynchronize(m->stream);
    }
    std::string why;
    if (bits & kOsErrTimeout) why += " one-shot all-reduce timed out (the one-shot path is now refused);";
    if (bits & kAttnErrHand) why += " fused q/k/v + attention hand-off wait timed out;";
    if (bits & kTlErrWait) why += " a persistent-layer wait timed out (a peer or a workgroup never arrived);";
    return fail(SLI_ERR_STATE, "device error bits 0x" + std::to_string(bits) + ":" + why + " outputs are stale");
}

static void destroy(sli_model* m) {
    if (!m) return;
    (void)hipSetDevice(m->c.device);
    if (m->comm_dead) {
        // an aborted communicator: work may still sit on the stream behind a wedged peer, so nothing is freed (the
        // process is about to exit on that error; freeing under running kernels would be worse than the leak)
        delete m;
        return;
    }
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    if (m->graph_exec) (void)hipGraphExecDestroy(m->graph_exec);
    if (m->graph) (void)hipGraphDestroy(m->graph);
    for (int b = 0; b < 4; ++b) {
        if (m->pf.exec[b]) (void)hipGraphExecDestroy(m->pf.exec[b]);
        if (m->pf.graph[b]) (void)hipGraphDestroy(m->pf.graph[b]);
    }
    if (m->comm) ncclCommDestroy(m->comm);
    for (int r = 0; r < sli::kOsMaxRanks; ++r)
        if (m->os_peer[r] && m->os_peer[r] != m->os_buf) (void)hipIpcCloseMemHandle(m->os_peer[r]);
    if (m->os_buf) (void)hipFree(m->os_buf);
    for (void* p : m->allocs) (void)hipFree(p);
    if (m->stream && m->own_stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

}  // namespace sli

using namespace sli;

extern "C" {

int sli_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int sli_comm_get_id(void* out) {
    SLI_CHECK(out, SLI_ERR_ARG, "sli_comm_get_id: null");
    ncclUniqueId id;
    SLI_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
    return SLI_OK;
}

// group != null: rank cfg->tp_rank of an in-process group (shares the group's stream, no communicator)
// Where the batch-1 attention's context splits are merged. Up to 8 splits per head the wo GEMV merges them
// while it stages its input (gemv.h XStageMerge: no serial tail in the attention launch). Past 8 (ctx > 2048
// at head_dim 128, fp16 K/V) the 16-split register batch spills (128 VGPRs + scratch) and wo took 17 us at
// ctx 4096 against 9 at 2048, so there the attention's last-arriving workgroup merges and wo stages a plain
// input. SLI_WO_MERGE=0|1 forces it (A/B, profiles/r4_wo_merge_ab.txt).
static int wo_merges(const sli_model* m) {
    const char* e = getenv("SLI_WO_MERGE");
    if (e && (e[0] == '0' || e[0] == '1')) return e[0] - '0';
    const int ppwg = attn_wg_positions(m->c.kv_dtype, m->hd);
    return (m->T + ppwg - 1) / ppwg > 8 ? 0 : 1;
}

// The batch-1 wo GEMV split over its input columns (gemv.h EpiKPart): ks workgroup blocks, block k streams columns
// [k QD / ks, (k + 1) QD / ks) of every row and merges only those heads' attention split partials, so a workgroup
// stages 1/ks of the 32 heads x 8 splits it reads unsplit (C1: 133 KB per workgroup, as many bytes as its weight
// rows at int8). The ks partial row sums go to wo_part; the gate/up GEMV stages x + sum(parts) (XStageSum) and
// the down GEMV's residual is the same sum (EpiStoreSum). Batch 1, TP 1 (a TP rank's wo feeds the exchange),
// D <= 4096 (XStageSum's one round). SLI_WO_KSPLIT=1 / 2 / 4 (A/B; default 2: C1 wo 10.0 -> 9.45 us, C3 int8 wo
// 8.32 -> 7.43 us, +0.6 % / +1.9 % tok/s; 4 is no faster).
static int wo_ksplit(const sli_model* m) {
    const char* e = getenv("SLI_WO_KSPLIT");  // read per model (tests switch it between models)
    const int env = e ? atoi(e) : 2;  // measured (profiles/r4_wo_ksplit_ab.txt): 2 best at C1 and C3
    const int ks = env == 2 || env == 4 ? env : 1;
    if (ks == 1 || m->B != 1 || m->partial || m->group || m->D > 4 * sli::kGemvThreads || m->hq % ks) return 1;
    if (!m->wo_merge) return 1;  // the split pays off in the merge staging it shrinks
    const int cols = m->hq * m->hd / ks;
    const int epv = 16 / (int)m->wbytes;  // weight elements per 16-byte vector
    if (cols % epv || cols % 4 || sli::gemv_ksplit_grid(m->D, ks) == 0) return 1;
    return ks;
}

// The batched projections' fragment-layout weight copies (bgemm.h BgIn::tiled: one contiguous KiB per wave load;
// C4 1742 -> 1988 tok/s, profiles/r4_bg_tiled_ab.txt). They double the projection weights in HBM (C4: +15 GB), so
// they are allocated last and only when they fit beside everything else with 1 GiB to spare; otherwise (or if an
// allocation fails) the model keeps streaming the row-major matrices (16 rows x 64 B per wave load), which is
// correct, only slower. SLI_DEBUG_BG_ROWMAJOR=1 forces that fallback (tests).
static void bg_alloc_tiles(sli_model* m) {
    m->bg_tiled = false;
    if (m->c.w_dtype != SLI_DT_F16 || std::getenv("SLI_DEBUG_BG_ROWMAJOR")) return;
    const int D = m->D, QD = m->hq * m->hd;
    std::vector<std::pair<void**, size_t>> want;
    for (auto& w : m->layers) {
        want.push_back({&w.qkv_t, bg_tiled_bytes(m->bp_qkv.ntiles, D)});
        want.push_back({&w.wo_t, bg_tiled_bytes(m->bp_wo.ntiles, QD)});
        want.push_back({&w.gu_t, bg_tiled_bytes(m->bp_gu.ntiles, D)});
        want.push_back({&w.down_t, bg_tiled_bytes(m->bp_down.ntiles, m->Il)});
    }
    want.push_back({&m->lm_t, bg_tiled_bytes(m->bp_lm.ntiles, D)});
    size_t need = 0, free_b = 0, total_b = 0;
    for (const auto& p : want) need += p.second;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b < need + ((size_t)1 << 30)) return;
    const size_t n0 = m->allocs.size();
    for (const auto& p : want) {
        if (hipMalloc(p.first, p.second) != hipSuccess) {  // undo: free the copies made so far, stay row-major
            (void)hipGetLastError();
            for (size_t i = n0; i < m->allocs.size(); ++i) (void)hipFree(m->allocs[i]);
            m->allocs.resize(n0);
            for (const auto& q : want) *q.first = nullptr;
            return;
        }
        m->allocs.push_back(*p.first);
    }
    m->bg_tiled = true;
}

static int create_model(const sli_model_config* cfg, const void* comm_id, sli_tp_group* group, sli_model** out) {
    SLI_CHECK(cfg && out, SLI_ERR_ARG, "sli_model_create: null");
    const sli_model_config& c = *cfg;
    SLI_CHECK(c.vocab > 0 && c.dim > 0 && c.n_heads > 0 && c.n_kv_heads > 0 && c.head_dim > 0 && c.ffn > 0 &&
                  c.n_layers > 0 && c.max_len > 0,
              SLI_ERR_SHAPE, "sli_model_create: non-positive dimension");
    SLI_CHECK(c.head_dim == 64 || c.head_dim == 128, SLI_ERR_SHAPE, "head_dim must be 64 or 128");
    SLI_CHECK(c.n_heads * c.head_dim == c.dim, SLI_ERR_SHAPE, "n_heads * head_dim must equal dim");
    SLI_CHECK(c.n_heads % c.n_kv_heads == 0, SLI_ERR_SHAPE, "n_heads must be a multiple of n_kv_heads");
    const int g = c.n_heads / c.n_kv_heads;
    SLI_CHECK(g == 1 || g == 2 || g == 4 || g == 8, SLI_ERR_SHAPE, "heads per kv head must be 1, 2, 4 or 8");
    SLI_CHECK(c.tp_size >= 1 && c.tp_rank >= 0 && c.tp_rank < c.tp_size, SLI_ERR_ARG, "bad tp rank/size");
    SLI_CHECK(c.n_kv_heads % c.tp_size == 0 && c.ffn % c.tp_size == 0, SLI_ERR_SHAPE,
              "kv heads and ffn must divide by tp_size");
    SLI_CHECK((c.ffn / c.tp_size) % 2 == 0, SLI_ERR_SHAPE, "local ffn must be even");
    SLI_CHECK(c.w_dtype >= SLI_DT_F32 && c.w_dtype <= SLI_DT_I8, SLI_ERR_ARG, "bad w_dtype");
    SLI_CHECK(c.kv_dtype == SLI_DT_F32 || c.kv_dtype == SLI_DT_F16, SLI_ERR_ARG, "bad kv_dtype");
    SLI_CHECK(c.tp_size == 1 || comm_id || group || std::getenv("SLI_DEBUG_NOCOMM"), SLI_ERR_ARG,
              "tensor parallel needs a comm id");
    const size_t wb = c.w_dtype == SLI_DT_F32 ? 4 : c.w_dtype == SLI_DT_F16 ? 2 : 1;
    SLI_CHECK(((size_t)c.dim * wb) % 16 == 0 && ((size_t)(c.ffn / c.tp_size) * wb) % 16 == 0 &&
                  ((size_t)(c.dim / c.tp_size) * wb) % 16 == 0,
              SLI_ERR_SHAPE, "row bytes must be multiples of 16");
    SLI_CHECK(c.dim <= kGemvMaxCols && c.ffn / c.tp_size <= kGemvMaxCols, SLI_ERR_SHAPE, "row too long for LDS staging");
    const int B = c.batch > 0 ? c.batch : 1;
    SLI_CHECK(B <= kBgMaxBatch, SLI_ERR_SHAPE, "batch must be at most 8");
    if (B > 1) {
        SLI_CHECK(c.w_dtype == SLI_DT_F16, SLI_ERR_ARG, "batch > 1 needs fp16 weights (MFMA projections)");
        SLI_CHECK(c.dim % 32 == 0 && (c.ffn / c.tp_size) % 32 == 0 && ((c.n_heads / c.tp_size) * c.head_dim) % 32 == 0,
                  SLI_ERR_SHAPE, "batch > 1: projection inputs must be multiples of 32");
        SLI_CHECK(c.dim <= kBgMaxStageK, SLI_ERR_SHAPE, "batch > 1: dim must be at most 4096 (RMS staging)");
    }

    SLI_HIP(hipSetDevice(c.device));
    sli_model* m = new sli_model();
    m->c = c;
    auto bail = [&](int rc) {
        destroy(m);
        return rc;
    };
    if (group) {
        m->stream = group->stream;
        m->own_stream = false;
        m->group = group;
    } else if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess) {
        return bail(fail(SLI_ERR_HIP, "hipStreamCreate"));
    }
    m->B = B;
    m->D = c.dim;
    m->L = c.n_layers;
    m->T = c.max_len;
    m->V = c.vocab;
    m->hd = c.head_dim;
    m->hq = c.n_heads / c.tp_size;
    m->hkv = c.n_kv_heads / c.tp_size;
    m->Il = c.ffn / c.tp_size;
    int32_t vlo = 0, vn = 0;
    if (sli_tp_vocab(&c, &vlo, &vn) != SLI_OK) return bail(SLI_ERR_ARG);
    m->v_lo = vlo;
    m->v_n = vn;
    if (m->v_n <= 0) return bail(fail(SLI_ERR_SHAPE, "vocab shard is empty"));
    m->wbytes = wb;
    m->kvbytes = c.kv_dtype == SLI_DT_F32 ? 4 : 2;
    const bool i8 = c.w_dtype == SLI_DT_I8;
    const int D = m->D, hd = m->hd, qkv_rows = (m->hq + 2 * m->hkv) * hd;

    int rc = SLI_OK;
    auto A = [&](void** p, size_t bytes) {
        if (rc == SLI_OK) rc = model_alloc(m, p, bytes);
    };
    A(&m->emb, (size_t)m->V * D * wb);
    if (i8) A((void**)&m->emb_s, sizeof(float) * m->V);
    A((void**)&m->norms, sizeof(float) * (size_t)(2 * m->L + 1) * D);
    m->layers.resize(m->L);
    for (auto& w : m->layers) {
        A(&w.qkv, (size_t)qkv_rows * D * wb);
        A(&w.wo, (size_t)D * m->hq * hd * wb);
        A(&w.gu, (size_t)2 * m->Il * D * wb);
        A(&w.down, (size_t)D * m->Il * wb);
        if (i8) {
            A((void**)&w.qkv_s, sizeof(float) * qkv_rows);
            A((void**)&w.wo_s, sizeof(float) * D);
            A((void**)&w.gu_s, sizeof(float) * 2 * m->Il);
            A((void**)&w.down_s, sizeof(float) * D);
        }
    }
    const size_t kv_elems = (size_t)m->L * B * m->hkv * m->T * hd;
    A(&m->kc, kv_elems * m->kvbytes);
    A(&m->vc, kv_elems * m->kvbytes);
    A((void**)&m->x, sizeof(float) * B * D);
    A((void**)&m->xpart, sizeof(float) * B * D);
    A((void**)&m->q, sizeof(float) * B * m->hq * hd);
    A((void**)&m->attn, sizeof(float) * B * m->hq * hd);
    A((void**)&m->act, sizeof(float) * B * m->Il);
    A((void**)&m->logits, sizeof(float) * B * m->v_n);
    A((void**)&m->part, mha_part_bytes(m->T, B * m->hq, hd));  // split-context partials
    A((void**)&m->attn_count, sizeof(unsigned) * B * m->hkv);   // per-kv-head arrival counters (kept zero)
    if (B == 1) {
        A((void**)&m->qa_kv, sizeof(float) * 2 * m->hkv * hd);
        A((void**)&m->qa_count, sizeof(unsigned) * attn_hand_words(m->hkv));
    }
    size_t bg_part = 0;
    int bg_groups = 1;
    const int cus = gemv_max_blocks();  // device_cus(), or the tests' SLI_DEBUG_GEMV_MAX_BLOCKS cap
    m->key_ld = gemv_max_blocks();  // LM-head argmax keys: one per GEMV workgroup
    if (B > 1) {  // tilings of the batched projections (bgemm.h)
        m->bp_qkv = bg_plan(qkv_rows / 16, D, B, true, cus);
        m->bp_wo = bg_plan((D + 15) / 16, m->hq * hd, B, false, cus);
        m->bp_gu = bg_plan(m->Il / 8, D, B, true, cus);
        m->bp_down = bg_plan((D + 15) / 16, m->Il, B, false, cus);
        m->bp_lm = bg_plan((m->v_n + 15) / 16, D, B, true, cus);
        for (const BgPlan* p : {&m->bp_qkv, &m->bp_wo, &m->bp_gu, &m->bp_down, &m->bp_lm}) {
            if (p->groups <= 0) return bail(fail(SLI_ERR_SHAPE, "batched projection: no tiling fits"));
            bg_part = std::max(bg_part, bg_part_bytes(*p));
            bg_groups = std::max(bg_groups, p->groups);
        }
        m->key_ld = std::max(m->key_ld, m->bp_lm.groups);
        A((void**)&m->bg_ws, bg_part + 256);
        A((void**)&m->bg_cnt, sizeof(unsigned) * bg_groups);
    }
    A((void**)&m->bkeys, sizeof(unsigned long long) * B);

    A((void**)&m->sin_t, sizeof(float) * (size_t)m->T * (hd / 2));
    A((void**)&m->cos_t, sizeof(float) * (size_t)m->T * (hd / 2));
    A((void**)&m->keys, sizeof(unsigned long long) * B * m->key_ld);
    A((void**)&m->st, sizeof(DevState) * B);
    A((void**)&m->prompt, sizeof(int32_t) * B * (m->T + 1));
    A((void**)&m->hist, sizeof(int32_t) * B * (m->T + 1));
    if (rc != SLI_OK) return bail(rc);
    if (B > 1) bg_alloc_tiles(m);

    std::vector<float> s, co;
    rope_table_host(hd, m->T, c.theta, s, co);  // rope_kernel.cpp:4-19, model.cpp:309-316
    if (hipMemcpy(m->sin_t, s.data(), s.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(m->cos_t, co.data(), co.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(SLI_ERR_HIP, "rope table upload"));
    if (hipMemset(m->prompt, 0, sizeof(int32_t) * B * (m->T + 1)) != hipSuccess ||
        hipMemset(m->attn_count, 0, sizeof(unsigned) * B * m->hkv) != hipSuccess ||
        (m->qa_count && hipMemset(m->qa_count, 0, sizeof(unsigned) * attn_hand_words(m->hkv)) != hipSuccess) ||
        hipMemset(m->hist, 0, sizeof(int32_t) * B * (m->T + 1)) != hipSuccess ||
        (m->bg_cnt && hipMemset(m->bg_cnt, 0, sizeof(unsigned) * bg_groups) != hipSuccess))
        return bail(fail(SLI_ERR_HIP, "memset"));
    if (B > 1 && (rc = SLI_DISPATCH(m, prepare, m)) != SLI_OK) return bail(rc);
    if ((rc = sli_model_reset(m)) != SLI_OK) return bail(rc);

    // Debug switches (tests only): SLI_DEBUG_FORCE_COMM=1 runs the tensor-parallel step
    // (partials + RCCL all-reduces) on a 1-rank communicator; SLI_DEBUG_NOCOMM=1 builds a tp_size>1
    // shard without a communicator (weight-placement checks; its logits are not meaningful).
    const bool force_comm = !group && c.tp_size == 1 && std::getenv("SLI_DEBUG_FORCE_COMM") != nullptr;
    const bool no_comm = !group && c.tp_size > 1 && std::getenv("SLI_DEBUG_NOCOMM") != nullptr;
    m->partial = c.tp_size > 1 || force_comm || group;
    m->collectives = !group && ((c.tp_size > 1 && !no_comm) || force_comm);  // a group's are its own kernels
    if (m->collectives) {
        ncclUniqueId id;
        if (comm_id) {
            std::memcpy(&id, comm_id, sizeof(id));
        } else if (ncclGetUniqueId(&id) != ncclSuccess) {
            return bail(fail(SLI_ERR_COMM, "ncclGetUniqueId"));
        }
        ncclResult_t r = ncclCommInitRank(&m->comm, c.tp_size, id, c.tp_rank);
        if (r != ncclSuccess) return bail(fail(SLI_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)));
    }
    m->wo_merge = m->B == 1 ? wo_merges(m) : 1;
    m->wo_ks = wo_ksplit(m);
    if (m->wo_ks > 1 && (rc = model_alloc(m, (void**)&m->wo_part, sizeof(float) * m->wo_ks * D)) != SLI_OK) return bail(rc);
    *out = m;
    return SLI_OK;
}

int sli_model_create(const sli_model_config* cfg, const void* comm_id, sli_model** out) {
    return create_model(cfg, comm_id, nullptr, out);
}

int sli_model_destroy(sli_model* m) {
    SLI_CHECK(!m || !m->group, SLI_ERR_STATE, "a rank of an in-process tp group is destroyed with its group");
    destroy(m);
    return SLI_OK;
}

int sli_model_init_synthetic(sli_model* m, uint32_t seed) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    SLI_HIP(hipSetDevice(m->c.device));
    auto src = [&](int kind, int index) {
        return SrcSynth{seed, sli_stream_id((uint32_t)kind, (uint32_t)index), synth_c(m, kind),
                        kind == SLI_T_NORM ? 1.0f : 0.0f};
    };
    SLI_TRY(place_tensor(m, SLI_T_EMB, 0, src(SLI_T_EMB, 0)));
    for (int i = 0; i < 2 * m->L + 1; ++i) SLI_TRY(place_tensor(m, SLI_T_NORM, i, src(SLI_T_NORM, i)));
    const int kinds[] = {SLI_T_WQ, SLI_T_WK, SLI_T_WV, SLI_T_WO, SLI_T_UP, SLI_T_GATE, SLI_T_DOWN};
    for (int l = 0; l < m->L; ++l)
        for (int k : kinds) SLI_TRY(place_tensor(m, k, l, src(k, l)));
    SLI_TRY(wait_stream(m));
    return SLI_OK;
}

int sli_model_set_weight(sli_model* m, int32_t kind, int32_t index, const float* host, int64_t n) {
    SLI_CHECK(m && host, SLI_ERR_ARG, "null argument");
    const int64_t want = tensor_elems(m, kind);
    SLI_CHECK(want > 0, SLI_ERR_ARG, "unknown tensor kind");
    SLI_CHECK(n == want, SLI_ERR_SHAPE, "tensor element count does not match the config");
    SLI_HIP(hipSetDevice(m->c.device));
    float* tmp = nullptr;
    SLI_HIP(hipMalloc(&tmp, sizeof(float) * (size_t)n));
    int rc = SLI_OK;
    if (hipMemcpy(tmp, host, sizeof(float) * (size_t)n, hipMemcpyHostToDevice) != hipSuccess)
        rc = fail(SLI_ERR_HIP, "hipMemcpy weight");
    if (rc == SLI_OK) rc = place_tensor(m, kind, index, SrcBuf{tmp});
    if (rc == SLI_OK) rc = wait_stream(m);
    (void)hipFree(tmp);
    return rc;
}

int sli_model_load_flat(sli_model* m, const char* path) {
    SLI_CHECK(m && path, SLI_ERR_ARG, "null argument");
    const int fd = open(path, O_RDONLY);
    SLI_CHECK(fd >= 0, SLI_ERR_ARG, std::string("Fail to open the weight file: ") + path);
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
        close(fd);
        return fail(SLI_ERR_ARG, "fstat failed");
    }
    const int L = m->L;
    int64_t total = tensor_elems(m, SLI_T_EMB) + (int64_t)(2 * L + 1) * m->D;
    const int kinds[] = {SLI_T_WQ, SLI_T_WK, SLI_T_WV, SLI_T_WO, SLI_T_UP, SLI_T_GATE, SLI_T_DOWN};
    for (int k : kinds) total += (int64_t)L * tensor_elems(m, k);
    if ((int64_t)sb.st_size < total * 4) {
        close(fd);
        return fail(SLI_ERR_SHAPE, "weight file smaller than the config requires");
    }
    void* map = mmap(nullptr, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (map == MAP_FAILED) return fail(SLI_ERR_ARG, "mmap failed");  // (the reference tests !ptr, model.cpp:242)
    const float* p = (const float*)map;
    int rc = sli_model_set_weight(m, SLI_T_EMB, 0, p, tensor_elems(m, SLI_T_EMB));  // model.cpp:343-358
    p += tensor_elems(m, SLI_T_EMB);
    for (int i = 0; rc == SLI_OK && i < 2 * L + 1; ++i, p += m->D)  // :360-364
        rc = sli_model_set_weight(m, SLI_T_NORM, i, p, m->D);
    for (int k : kinds) {  // :366-468
        const int64_t n = tensor_elems(m, k);
        for (int l = 0; rc == SLI_OK && l < L; ++l, p += n) rc = sli_model_set_weight(m, k, l, p, n);
    }
    munmap(map, (size_t)sb.st_size);
    return rc;
}

int sli_model_reset(sli_model* m) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    SLI_HIP(hipSetDevice(m->c.device));
    const size_t kv = (size_t)m->L * m->B * m->hkv * m->T * m->hd * m->kvbytes;
    SLI_HIP(hipMemsetAsync(m->kc, 0, kv, m->stream));
    SLI_HIP(hipMemsetAsync(m->vc, 0, kv, m->stream));
    std::vector<DevState> h(m->B);
    for (auto& d : h) d.advance = 1;
    return upload_states(m, h);
}

int sli_model_fill_kv_synthetic(sli_model* m, uint32_t seed, int32_t upto) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    SLI_CHECK(upto >= 0 && upto <= m->T, SLI_ERR_RANGE, "upto out of range");
    if (upto == 0) return SLI_OK;
    SLI_HIP(hipSetDevice(m->c.device));
    SLI_TRY(SLI_DISPATCH(m, fill_kv, m, seed, upto));
    SLI_TRY(wait_stream(m));
    return SLI_OK;
}

// seq < 0: every sequence
static int set_state(sli_model* m, int seq, int32_t token, int32_t pos, int32_t advance) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    SLI_CHECK(seq < m->B, SLI_ERR_RANGE, "sequence index out of range");
    SLI_CHECK(token >= 0 && token < m->V, SLI_ERR_RANGE, "Token index is greater than vocab size.");
    SLI_CHECK(pos >= 0 && pos < m->T, SLI_ERR_RANGE, "position out of range");
    std::vector<DevState> h;
    SLI_TRY(download_states(m, h));
    for (int b = 0; b < m->B; ++b) {
        if (seq >= 0 && b != seq) continue;
        h[b].token = token;
        h[b].pos = pos;
        h[b].advance = advance ? 1 : 0;
        h[b].key = 0;
        h[b].error = 0;
        SLI_HIP(hipMemcpyAsync(m->hist + (size_t)b * (m->T + 1) + pos, &token, sizeof(int32_t), hipMemcpyHostToDevice,
                               m->stream));
    }
    return upload_states(m, h);
}

static int set_prompt(sli_model* m, int seq, const int32_t* ids, int32_t n) {
    SLI_CHECK(m && ids, SLI_ERR_ARG, "null argument");
    SLI_CHECK(seq < m->B, SLI_ERR_RANGE, "sequence index out of range");
    SLI_CHECK(n >= 1 && n <= m->T, SLI_ERR_RANGE, "prompt length out of range");
    SLI_CHECK(!m->comm_dead, SLI_ERR_COMM, "the RCCL communicator was aborted by an earlier bounded wait");
    for (int i = 0; i < n; ++i)
        SLI_CHECK(ids[i] >= 0 && ids[i] < m->V, SLI_ERR_RANGE, "Token index is greater than vocab size.");
    std::vector<DevState> h;
    SLI_TRY(download_states(m, h));
    for (int b = 0; b < m->B; ++b) {
        if (seq >= 0 && b != seq) continue;
        SLI_HIP(hipMemcpyAsync(m->prompt + (size_t)b * (m->T + 1), ids, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                               m->stream));
        h[b].n_forced = n;
    }
    return upload_states(m, h);
}

static int get_state(sli_model* m, int seq, int32_t* pos, int32_t* token, int32_t* last_argmax, int32_t* error) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    SLI_CHECK(seq >= 0 && seq < m->B, SLI_ERR_RANGE, "sequence index out of range");
    std::vector<DevState> h;
    SLI_TRY(download_states(m, h));
    if (pos) *pos = h[seq].pos;
    if (token) *token = h[seq].token;
    if (last_argmax) *last_argmax = h[seq].last_argmax;
    if (error) *error = h[seq].error;
    return SLI_OK;
}

}  // extern "C" (reopened below)

// ---------------------------------------------------------------- prompt prefill
// The GEMM prefill (prefill.h) needs fp16 or int8 weights, batch 1, head_dim 64 or 128 and 64-multiple
// projection depths; otherwise the prompt runs through the decode step itself (teacher forcing), which gives
// the same tokens.
// The chunked MFMA prefill (prefill.h) takes GEMM depths that are multiples of 64 (int8: 128-deep stages with a
// half last stage). A multi-process TP rank without an RCCL communicator (SLI_DEBUG_NOCOMM, with or without the
// one-shot exchange) has no all-reduce for a chunk's M x D residual rows, so it prefills through the decode step,
// whose exchange it does have; an in-process group sums the chunk rows itself (record_group_prefill).
static bool pf_supported(const sli_model* m) {
    if (m->partial && !m->collectives && !m->group) return false;
    return m->c.w_dtype != SLI_DT_F32 && m->B == 1 && (m->hd == 64 || m->hd == 128) && m->D % 64 == 0 &&
           m->D <= 8192 && m->Il % 64 == 0 && (m->hq * m->hd) % 64 == 0;
}

static int pf_bucket(int nv) {
    for (int b = 0; b < 3; ++b)
        if (nv <= kPfSizes[b]) return b;
    return 3;
}

static int pf_alloc(sli_model* m) {
    auto& p = m->pf;
    if (p.x) return SLI_OK;
    const size_t M = kPfMaxChunk, D = m->D, QD = (size_t)m->hq * m->hd;
    int rc = SLI_OK;
    auto A = [&](void** ptr, size_t bytes) {
        if (rc == SLI_OK) rc = model_alloc(m, ptr, bytes);
    };
    A((void**)&p.x, sizeof(float) * M * D);
    if (m->partial) A((void**)&p.xpart, sizeof(float) * M * D);
    A((void**)&p.q, sizeof(float) * M * QD);
    A((void**)&p.hhi, sizeof(__half) * M * std::max(D, QD));
    A((void**)&p.hlo, sizeof(__half) * M * std::max(D, QD));
    A((void**)&p.ahi, sizeof(__half) * M * m->Il);
    A((void**)&p.alo, sizeof(__half) * M * m->Il);
    A((void**)&p.ps, sizeof(PfState));
    if (rc != SLI_OK) return rc;
    return SLI_DISPATCH(m, prepare_prefill, m);
}

// chunk c of the prompt's n - 1 prefilled positions
static std::vector<PfState> pf_chunks(int n) {
    std::vector<PfState> cs;
    for (int p0 = 0; p0 < n - 1; p0 += kPfMaxChunk) cs.push_back(PfState{p0, std::min(kPfMaxChunk, n - 1 - p0)});
    return cs;
}

extern "C" int sli_model_prefill_path(const sli_model* m) { return m && m->B == 1 && pf_supported(m) ? 1 : 0; }

extern "C" int sli_model_fused_qkv_attn(sli_model* m) {
    if (!m || m->B != 1) return 0;
    int done = 0;
    if (SLI_DISPATCH(m, gemv_qkv_attn, m, 0, &done, true) != SLI_OK) return 0;
    return done;
}

extern "C" int sli_model_prefill(sli_model* m, const int32_t* ids, int32_t n) {
    SLI_CHECK(m && ids, SLI_ERR_ARG, "null argument");
    SLI_CHECK(m->B == 1, SLI_ERR_STATE, "prefill: batch-1 models (a batch prefills through predict_batch)");
    SLI_CHECK(!m->group, SLI_ERR_STATE, "prefill: ranks of an in-process group prefill through sli_tp_group_prefill");
    SLI_CHECK(n >= 1 && n <= m->T, SLI_ERR_RANGE, "prompt length out of range");
    for (int i = 0; i < n; ++i)
        SLI_CHECK(ids[i] >= 0 && ids[i] < m->V, SLI_ERR_RANGE, "Token index is greater than vocab size.");
    SLI_HIP(hipSetDevice(m->c.device));
    SLI_TRY(set_prompt(m, 0, ids, n));
    SLI_HIP(hipMemcpyAsync(m->hist, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice, m->stream));
    if (n > 1 && pf_supported(m)) {
        SLI_TRY(pf_alloc(m));
        const std::vector<PfState> cs = pf_chunks(n);
        for (const PfState& c : cs) {  // capture before anything is enqueued behind the capture
            const int b = pf_bucket(c.nv);
            SLI_TRY(capture_graph(m->stream, m->pf.graph[b], m->pf.exec[b],
                                  [&]() { return SLI_DISPATCH(m, record_prefill, m, kPfSizes[b]); }));
        }
        for (const PfState& c : cs) {  // each copy reads its own element of cs: enqueued back to back
            SLI_HIP(hipMemcpyAsync(m->pf.ps, &c, sizeof(PfState), hipMemcpyHostToDevice, m->stream));
            SLI_HIP(hipGraphLaunch(m->pf.exec[pf_bucket(c.nv)], m->stream));
        }
        SLI_TRY(wait_stream(m));
    } else {
        for (int p = 0; p < n - 1; ++p) {  // the decode step, teacher-forced (model.cpp:159-165)
            SLI_TRY(set_state(m, 0, ids[p], p, 0));
            SLI_TRY(sli_model_step(m));
        }
    }
    // the last prompt position is an ordinary decode step: it yields the first greedy token
    return set_state(m, 0, ids[n - 1], n - 1, 1);
}

extern "C" int sli_tp_group_prefill(sli_tp_group* g, const int32_t* ids, int32_t n) {
    SLI_CHECK(g && ids, SLI_ERR_ARG, "null argument");
    sli_model* m0 = g->ranks[0];
    SLI_CHECK(m0->B == 1, SLI_ERR_STATE, "prefill: batch-1 groups (a batch prefills through predict_batch)");
    SLI_CHECK(n >= 1 && n <= m0->T, SLI_ERR_RANGE, "prompt length out of range");
    SLI_HIP(hipSetDevice(g->device));
    for (sli_model* m : g->ranks) {
        SLI_TRY(set_prompt(m, 0, ids, n));
        SLI_HIP(hipMemcpyAsync(m->hist, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice, m->stream));
    }
    if (n > 1 && pf_supported(m0)) {
        for (sli_model* m : g->ranks) SLI_TRY(pf_alloc(m));
        const std::vector<PfState> cs = pf_chunks(n);
        for (const PfState& c : cs) {
            const int b = pf_bucket(c.nv);
            SLI_TRY(capture_graph(g->stream, g->pf_graph[b], g->pf_exec[b],
                                  [&]() { return SLI_DISPATCH(m0, record_group_prefill, g, kPfSizes[b]); }));
        }
        for (const PfState& c : cs) {
            for (sli_model* m : g->ranks)
                SLI_HIP(hipMemcpyAsync(m->pf.ps, &c, sizeof(PfState), hipMemcpyHostToDevice, g->stream));
            SLI_HIP(hipGraphLaunch(g->pf_exec[pf_bucket(c.nv)], g->stream));
        }
        SLI_HIP(hipStreamSynchronize(g->stream));
    } else {
        for (int p = 0; p < n - 1; ++p) {
            for (sli_model* m : g->ranks) SLI_TRY(set_state(m, 0, ids[p], p, 0));
            SLI_TRY(sli_tp_group_step(g));
        }
    }
    for (sli_model* m : g->ranks) SLI_TRY(set_state(m, 0, ids[n - 1], n - 1, 1));
    return SLI_OK;
}

extern "C" int sli_model_predict_prefill(sli_model* m, const int32_t* prompt, int32_t n_prompt, int32_t max_length,
                                         int32_t* tokens_out, float* logits_out) {
    SLI_CHECK(m && prompt && tokens_out, SLI_ERR_ARG, "null argument");
    SLI_CHECK(max_length >= n_prompt && max_length <= m->T, SLI_ERR_RANGE, "max_length must be in [n_prompt, max_len]");
    SLI_TRY(sli_model_prefill(m, prompt, n_prompt));
    const size_t per_step = (size_t)m->v_n;
    if (logits_out)  // positions the prefill computes no logits for
        for (size_t i = 0; i < (size_t)(n_prompt - 1) * per_step; ++i) logits_out[i] = NAN;
    for (int t = n_prompt - 1; t < max_length; ++t) {
        SLI_TRY(sli_model_step(m));
        if (logits_out) SLI_TRY(sli_model_get_logits(m, logits_out + (size_t)t * per_step, (int32_t)per_step, nullptr));
    }
    SLI_HIP(hipMemcpyAsync(tokens_out, m->hist, sizeof(int32_t) * max_length, hipMemcpyDeviceToHost, m->stream));
    SLI_TRY(wait_stream(m));
    return check_device_errors(m);
}

extern "C" {

int sli_model_set_state(sli_model* m, int32_t token, int32_t pos, int32_t advance) {
    return set_state(m, -1, token, pos, advance);
}

int sli_model_set_state_seq(sli_model* m, int32_t seq, int32_t token, int32_t pos, int32_t advance) {
    SLI_CHECK(seq >= 0, SLI_ERR_RANGE, "sequence index out of range");
    return set_state(m, seq, token, pos, advance);
}

int sli_model_set_prompt(sli_model* m, const int32_t* ids, int32_t n) { return set_prompt(m, -1, ids, n); }

int sli_model_set_prompt_seq(sli_model* m, int32_t seq, const int32_t* ids, int32_t n) {
    SLI_CHECK(seq >= 0, SLI_ERR_RANGE, "sequence index out of range");
    return set_prompt(m, seq, ids, n);
}

int sli_model_get_state(sli_model* m, int32_t* pos, int32_t* token, int32_t* last_argmax, int32_t* error) {
    return get_state(m, 0, pos, token, last_argmax, error);
}

int sli_model_get_state_seq(sli_model* m, int32_t seq, int32_t* pos, int32_t* token, int32_t* last_argmax,
                            int32_t* error) {
    return get_state(m, seq, pos, token, last_argmax, error);
}

int sli_model_get_history(sli_model* m, int32_t seq, int32_t n, int32_t* out) {
    SLI_CHECK(m && out, SLI_ERR_ARG, "null argument");
    SLI_CHECK(seq >= 0 && seq < m->B && n >= 0 && n <= m->T, SLI_ERR_RANGE, "sequence / length out of range");
    SLI_HIP(hipMemcpyAsync(out, m->hist + (size_t)seq * (m->T + 1), sizeof(int32_t) * n, hipMemcpyDeviceToHost,
                           m->stream));
    SLI_TRY(wait_stream(m));
    return SLI_OK;
}

int sli_model_set_exec(sli_model* m, int32_t mode) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    SLI_CHECK(mode == SLI_EXEC_LAUNCHES || mode == SLI_EXEC_PERSIST, SLI_ERR_ARG,
              "unknown execution mode (the persistent one-launch step, mode 1, was removed in round 5: DESIGN.md §9)");
    if (mode == SLI_EXEC_PERSIST) {
        std::string why;
        SLI_CHECK(tpl_check(m, &why), SLI_ERR_STATE, "persistent layers: " + why);
    }
    SLI_HIP(hipSetDevice(m->c.device));
    if (mode != m->exec) {  // re-capture the step graph on the next step
        SLI_TRY(wait_stream(m));
        if (m->graph_exec) (void)hipGraphExecDestroy(m->graph_exec);
        if (m->graph) (void)hipGraphDestroy(m->graph);
        m->graph_exec = nullptr;
        m->graph = nullptr;
        m->exec = mode;
    }
    return SLI_OK;
}

int sli_model_get_exec(sli_model* m, int32_t* mode) {
    SLI_CHECK(m && mode, SLI_ERR_ARG, "null argument");
    *mode = m->exec;
    return SLI_OK;
}

int sli_model_step(sli_model* m) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    SLI_CHECK(!m->group, SLI_ERR_STATE, "a rank of an in-process tp group steps with its group (sli_tp_group_step)");
    SLI_TRY(capture(m));
    SLI_HIP(hipGraphLaunch(m->graph_exec, m->stream));
    return SLI_OK;
}

int sli_model_sync(sli_model* m) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    SLI_TRY(wait_stream(m));
    return SLI_OK;
}

int sli_model_get_logits(sli_model* m, float* host, int32_t n, int32_t* vocab_lo) {
    SLI_CHECK(m && host, SLI_ERR_ARG, "null argument");
    SLI_CHECK(n >= m->B * m->v_n, SLI_ERR_SHAPE, "host buffer smaller than the local vocab shard x batch");
    SLI_HIP(hipMemcpyAsync(host, m->logits, sizeof(float) * m->B * m->v_n, hipMemcpyDeviceToHost, m->stream));
    SLI_TRY(wait_stream(m));
    if (vocab_lo) *vocab_lo = m->v_lo;
    return SLI_OK;
}

int sli_model_predict_batch(sli_model* m, const int32_t* prompts, const int32_t* lens, int32_t ld, int32_t max_length,
                            int32_t* tokens_out, float* logits_out) {
    SLI_CHECK(m && prompts && lens && tokens_out, SLI_ERR_ARG, "null argument");
    SLI_CHECK(max_length >= 1 && max_length <= m->T, SLI_ERR_RANGE, "max_length must be in [1, max_len]");
    for (int b = 0; b < m->B; ++b) {
        SLI_CHECK(lens[b] >= 1 && lens[b] <= ld, SLI_ERR_RANGE, "prompt length out of range");
        SLI_TRY(set_prompt(m, b, prompts + (size_t)b * ld, lens[b]));
        SLI_TRY(set_state(m, b, prompts[(size_t)b * ld], 0, 1));
    }
    const size_t per_step = (size_t)m->B * m->v_n;
    for (int t = 0; t < max_length; ++t) {  // model.cpp:157
        SLI_TRY(sli_model_step(m));
        if (logits_out) SLI_TRY(sli_model_get_logits(m, logits_out + (size_t)t * per_step, (int32_t)per_step, nullptr));
    }
    for (int b = 0; b < m->B; ++b)
        SLI_HIP(hipMemcpyAsync(tokens_out + (size_t)b * max_length, m->hist + (size_t)b * (m->T + 1),
                               sizeof(int32_t) * max_length, hipMemcpyDeviceToHost, m->stream));
    SLI_TRY(wait_stream(m));
    return check_device_errors(m);
}

int sli_model_predict(sli_model* m, const int32_t* prompt, int32_t n_prompt, int32_t max_length, int32_t* tokens_out,
                      float* logits_out) {
    SLI_CHECK(m && prompt && tokens_out, SLI_ERR_ARG, "null argument");
    SLI_CHECK(n_prompt >= 1, SLI_ERR_RANGE, "prompt length out of range");
    std::vector<int32_t> ps((size_t)m->B * n_prompt), lens(m->B, n_prompt);
    for (int b = 0; b < m->B; ++b) std::memcpy(ps.data() + (size_t)b * n_prompt, prompt, sizeof(int32_t) * n_prompt);
    return sli_model_predict_batch(m, ps.data(), lens.data(), n_prompt, max_length, tokens_out, logits_out);
}

int sli_model_get_kv(sli_model* m, int32_t layer, int32_t which, int32_t upto, float* host) {
    return sli_model_get_kv_seq(m, 0, layer, which, upto, host);
}

int sli_model_get_kv_seq(sli_model* m, int32_t seq, int32_t layer, int32_t which, int32_t upto, float* host) {
    SLI_CHECK(m && host, SLI_ERR_ARG, "null argument");
    SLI_CHECK(layer >= 0 && layer < m->L && upto > 0 && upto <= m->T && (which == 0 || which == 1) && seq >= 0 &&
                  seq < m->B,
              SLI_ERR_RANGE, "seq/layer/which/upto out of range");
    const size_t n = (size_t)upto * m->hkv * m->hd;
    float* tmp = nullptr;
    SLI_HIP(hipMalloc(&tmp, n * 4));
    int rc = SLI_DISPATCH(m, get_kv, m, seq, layer, which, upto, tmp);
    if (rc == SLI_OK && hipMemcpyAsync(host, tmp, n * 4, hipMemcpyDeviceToHost, m->stream) != hipSuccess)
        rc = fail(SLI_ERR_HIP, "copy kv");
    if (rc == SLI_OK) rc = wait_stream(m);
    (void)hipFree(tmp);
    return rc;
}

int sli_model_get_weight(sli_model* m, int32_t kind, int32_t index, float* host, int64_t n) {
    SLI_CHECK(m && host, SLI_ERR_ARG, "null argument");
    const void* src = nullptr;
    const float* scale = nullptr;
    int64_t rows = 0, cols = 0;
    if (kind == SLI_T_NORM) {
        SLI_CHECK(index >= 0 && index <= 2 * m->L, SLI_ERR_RANGE, "norm index");
        SLI_CHECK(n == m->D, SLI_ERR_SHAPE, "host buffer size");
        SLI_HIP(hipMemcpy(host, m->norms + (size_t)index * m->D, sizeof(float) * m->D, hipMemcpyDeviceToHost));
        return SLI_OK;
    }
    sli_shard_window w;
    SLI_TRY(sli_tp_plan(&m->c, kind, &w));
    rows = w.n_rows;
    cols = w.n_cols;
    if (kind == SLI_T_EMB) {
        src = m->emb;
        scale = m->emb_s;
    } else {
        SLI_CHECK(index >= 0 && index < m->L, SLI_ERR_RANGE, "layer index");
        const LayerW& L = m->layers[index];
        switch (kind) {
            case SLI_T_WQ: case SLI_T_WK: case SLI_T_WV: src = L.qkv; scale = L.qkv_s; break;
            case SLI_T_WO: src = L.wo; scale = L.wo_s; break;
            case SLI_T_GATE: case SLI_T_UP: src = L.gu; scale = L.gu_s; break;
            case SLI_T_DOWN: src = L.down; scale = L.down_s; break;
            default: return fail(SLI_ERR_ARG, "unknown tensor kind");
        }
        src = wptr(const_cast<void*>(src), m->wbytes, (size_t)w.dst_row_off * w.n_cols);
        if (scale) scale += w.dst_row_off;
    }
    SLI_CHECK(n == rows * cols, SLI_ERR_SHAPE, "host buffer size must be the local shard's rows*cols");
    std::vector<unsigned char> raw((size_t)(rows * cols) * m->wbytes);
    SLI_HIP(hipMemcpy(raw.data(), src, raw.size(), hipMemcpyDeviceToHost));
    std::vector<float> sc;
    if (scale) {
        sc.resize(rows);
        SLI_HIP(hipMemcpy(sc.data(), scale, sizeof(float) * rows, hipMemcpyDeviceToHost));
    }
    for (int64_t i = 0; i < rows * cols; ++i) {
        float v;
        if (m->wbytes == 4) {
            std::memcpy(&v, &raw[4 * i], 4);
        } else if (m->wbytes == 2) {
            __half h;
            std::memcpy(&h, &raw[2 * i], 2);
            v = __half2float(h);
        } else {
            v = (float)(int8_t)raw[i] * sc[i / cols];
        }
        host[i] = v;
    }
    return SLI_OK;
}


int sli_model_stream(sli_model* m, sli_stream_t* out) {
    SLI_CHECK(m && out, SLI_ERR_ARG, "null argument");
    *out = m->stream;
    return SLI_OK;
}

int sli_model_step_bytes(sli_model* m, double* weight_bytes, double* kv_bytes) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    std::vector<DevState> h;
    SLI_TRY(download_states(m, h));
    const double wb = (double)m->wbytes, D = m->D, hd = m->hd;
    const double per_layer = ((m->hq + 2.0 * m->hkv) * hd * D + D * m->hq * hd + 3.0 * m->Il * D) * wb;
    double w = m->L * per_layer + (double)m->v_n * D * wb;
    if (m->c.w_dtype == SLI_DT_I8) w += 4.0 * (m->L * ((m->hq + 2.0 * m->hkv) * hd + 2.0 * D + 2.0 * m->Il) + m->v_n);
    if (weight_bytes) *weight_bytes = w;
    double ctx = 0.0;
    for (const DevState& d : h) ctx += d.pos + 1.0;
    if (kv_bytes) *kv_bytes = 2.0 * m->L * ctx * m->hkv * hd * (double)m->kvbytes;
    return SLI_OK;
}

// ---------------------------------------------------------------- one-shot all-reduce (oneshot.h)
int sli_model_comm_handle(sli_model* m, void* out, int32_t n) {
    SLI_CHECK(m && out, SLI_ERR_ARG, "null argument");
    SLI_CHECK(n >= (int32_t)sizeof(hipIpcMemHandle_t), SLI_ERR_ARG, "handle buffer too small");
    SLI_CHECK(m->c.tp_size > 1 && m->c.tp_size <= kOsMaxRanks && !m->group, SLI_ERR_STATE,
              "one-shot all-reduce: 2..8 ranks, one process per rank");
    SLI_HIP(hipSetDevice(m->c.device));
    if (!m->os_buf) {
        m->os_nmax = (std::max(m->B * m->D, 2 * m->B) + 3) & ~3;
        m->os_bytes = os_buffer_bytes(m->os_nmax);
        SLI_HIP(hipExtMallocWithFlags((void**)&m->os_buf, m->os_bytes, hipDeviceMallocUncached));
        SLI_HIP(hipMemset(m->os_buf, 0, m->os_bytes));
        SLI_TRY(model_alloc(m, (void**)&m->os_epoch, 16 * sizeof(unsigned)));
        SLI_HIP(hipMemset(m->os_epoch, 0, 16 * sizeof(unsigned)));
        SLI_TRY(model_alloc(m, (void**)&m->os_wg_epoch, kOsRegions * kOsMaxWg * sizeof(unsigned)));
        SLI_HIP(hipMemset(m->os_wg_epoch, 0, kOsRegions * kOsMaxWg * sizeof(unsigned)));
        SLI_TRY(model_alloc(m, (void**)&m->os_peer_tab, sizeof(char*) * kOsMaxRanks));
    }
    hipIpcMemHandle_t h;
    SLI_HIP(hipIpcGetMemHandle(&h, m->os_buf));
    std::memcpy(out, &h, sizeof(h));
    return SLI_OK;
}

int sli_model_comm_handle_bytes(void) { return (int)sizeof(hipIpcMemHandle_t); }

int sli_model_comm_open(sli_model* m, const void* handles, int32_t nranks) {
    SLI_CHECK(m && handles, SLI_ERR_ARG, "null argument");
    SLI_CHECK(m->os_buf, SLI_ERR_STATE, "call sli_model_comm_handle first");
    SLI_CHECK(nranks == m->c.tp_size, SLI_ERR_ARG, "one handle per rank");
    SLI_HIP(hipSetDevice(m->c.device));
    if (m->os_open) return SLI_OK;
    for (int r = 0; r < nranks; ++r) {
        if (r == m->c.tp_rank) {
            m->os_peer[r] = m->os_buf;
            continue;
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, (const char*)handles + (size_t)r * sizeof(h), sizeof(h));
        void* p = nullptr;
        SLI_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        m->os_peer[r] = (char*)p;
    }
    SLI_HIP(hipMemcpy(m->os_peer_tab, m->os_peer, sizeof(char*) * kOsMaxRanks, hipMemcpyHostToDevice));
    m->os_open = true;
    return SLI_OK;
}

int sli_model_set_allreduce(sli_model* m, int32_t mode) {
    SLI_CHECK(m, SLI_ERR_ARG, "null model");
    if (mode != SLI_ALLREDUCE_RCCL && !m->os_open && getenv("SLI_DEBUG_OS_LOOPBACK") && m->partial && !m->collectives) {
        // debug timing on one GPU without peers (with SLI_DEBUG_NOCOMM): every peer slot is this rank's own
        // buffer and the rank raises every flag itself; the sums are not a model
        char h[256];
        SLI_TRY(sli_model_comm_handle(m, h, (int32_t)sizeof(h)));
        for (int r = 0; r < m->c.tp_size; ++r) m->os_peer[r] = m->os_buf;
        SLI_HIP(hipMemcpy(m->os_peer_tab, m->os_peer, sizeof(char*) * kOsMaxRanks, hipMemcpyHostToDevice));
        m->os_open = true;
        m->os_loopback = true;
    }
    SLI_CHECK(mode == SLI_ALLREDUCE_RCCL || mode == SLI_ALLREDUCE_ONESHOT || mode == SLI_ALLREDUCE_FUSED ||
                  mode == SLI_ALLREDUCE_FUSED_WG,
              SLI_ERR_ARG, "unknown all-reduce mode");
    SLI_CHECK(mode != SLI_ALLREDUCE_FUSED || m->B == 1, SLI_ERR_STATE,
              "the launch-level fused all-reduce rides the batch-1 GEMV epilogues (batch > 1: fused_wg, oneshot or rccl)");
    SLI_CHECK(mode != SLI_ALLREDUCE_FUSED_WG ||
                  (gemv_max_blocks() <= kOsMaxWg && m->bp_wo.groups <= kOsMaxWg && m->bp_down.groups <= kOsMaxWg),
              SLI_ERR_SHAPE, "per-workgroup exchange: more workgroups than flag slots");
    SLI_CHECK(mode == SLI_ALLREDUCE_RCCL || m->os_open, SLI_ERR_STATE, "one-shot all-reduce: open the peers first");
    SLI_CHECK(mode == SLI_ALLREDUCE_RCCL || !m->os_dead, SLI_ERR_STATE,
              "one-shot all-reduce: a wait timed out earlier, the ranks' epochs may disagree");
    // the fp32 sum moves float4s and the key exchange 2*B floats: both must fit the slot exactly
    SLI_CHECK(mode == SLI_ALLREDUCE_RCCL || ((m->B * m->D) % 4 == 0 && m->B * m->D <= m->os_nmax && 2 * m->B <= m->os_nmax),
              SLI_ERR_SHAPE, "one-shot all-reduce: B*D must be a multiple of 4 within the comm slot");
    SLI_CHECK(m->exec == SLI_EXEC_LAUNCHES || mode == SLI_ALLREDUCE_FUSED_WG, SLI_ERR_STATE,
              "the persistent layers exchange per workgroup inside the launch: fused_wg (set_exec(launches) first)");
    if (mode != m->ar_mode) {
        SLI_TRY(wait_stream(m));
        if (m->graph_exec) (void)hipGraphExecDestroy(m->graph_exec);
        if (m->graph) (void)hipGraphDestroy(m->graph);
        m->graph_exec = nullptr;
        m->graph = nullptr;
        m->ar_mode = mode;
    }
    return SLI_OK;
}

int sli_debug_bounded_wait(int32_t mode, double deadline_ms, double* waited_ms) {
    SLI_CHECK(mode >= 0 && mode <= 3 && deadline_ms >= 0.0 && waited_ms, SLI_ERR_ARG, "bad argument");
    int polls = 0;
    std::string why;
    const double t0 = steady_ms();
    const int rc = bounded_wait(
        [&] {
            ++polls;
            if (mode == 3) return WaitPoll::Failed;
            return mode == 0 && polls >= 3 ? WaitPoll::Done : WaitPoll::Pending;
        },
        [&](std::string& msg) {
            if (mode != 2 || polls < 2) return false;
            msg = "mocked remote error";
            return true;
        },
        steady_ms, deadline_ms, why);
    *waited_ms = steady_ms() - t0;
    return rc == SLI_OK ? SLI_OK : fail(rc, why);
}

int sli_model_time_steps(sli_model* m, int32_t iters, double* avg_us) {
    SLI_CHECK(m && iters > 0 && avg_us, SLI_ERR_ARG, "bad argument");
    SLI_CHECK(!m->group, SLI_ERR_STATE, "time a group through its own stream");
    SLI_HIP(hipSetDevice(m->c.device));
    struct Guard {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        ~Guard() {
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
        }
    } g;
    SLI_HIP(hipEventCreate(&g.e0));
    SLI_HIP(hipEventCreate(&g.e1));
    SLI_TRY(sli_model_step(m));  // captured and warm
    SLI_HIP(hipEventRecord(g.e0, m->stream));
    for (int i = 0; i < iters; ++i) SLI_HIP(hipGraphLaunch(m->graph_exec, m->stream));
    SLI_HIP(hipEventRecord(g.e1, m->stream));
    SLI_TRY(wait_event(m, g.e1));
    float ms = 0.0f;
    SLI_HIP(hipEventElapsedTime(&ms, g.e0, g.e1));
    *avg_us = 1000.0 * ms / iters;
    return SLI_OK;
}

int sli_model_time_families(sli_model* m, int32_t iters, double* us, double* bytes, int32_t* launches) {
    SLI_CHECK(m && iters > 0 && us && bytes && launches, SLI_ERR_ARG, "bad argument");
    SLI_CHECK(!m->group, SLI_ERR_STATE, "time a group's ranks through a standalone model");
    SLI_HIP(hipSetDevice(m->c.device));
    SLI_TRY(bg_sync_tiles(m));
    // Like sli_model_time_gemv: x is saved and restored; the qkv family rewrites each layer's K/V row at
    // the current position, which the next real step at that position rewrites again.
    struct Guard {
        float* xsave = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        ~Guard() {
            if (xsave) (void)hipFree(xsave);
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
        }
    } g;
    const size_t xb = sizeof(float) * m->B * m->D;
    SLI_HIP(hipMalloc(&g.xsave, xb));
    SLI_HIP(hipMemcpyAsync(g.xsave, m->x, xb, hipMemcpyDeviceToDevice, m->stream));
    SLI_HIP(hipEventCreate(&g.e0));
    SLI_HIP(hipEventCreate(&g.e1));
    std::vector<DevState> h;
    SLI_TRY(download_states(m, h));
    double ctx = 0.0;
    for (const DevState& d : h) ctx += d.pos + 1.0;
    const double wb = (double)m->wbytes, D = m->D, hd = m->hd, i8 = m->c.w_dtype == SLI_DT_I8 ? 4.0 : 0.0;
    const double qkv_rows = (m->hq + 2.0 * m->hkv) * hd;
    bytes[SLI_FAM_QKV] = qkv_rows * (D * wb + i8);
    bytes[SLI_FAM_ATTN] = 2.0 * ctx * m->hkv * hd * (double)m->kvbytes;
    bytes[SLI_FAM_WO] = D * (m->hq * hd * wb + i8);
    bytes[SLI_FAM_GU] = 2.0 * m->Il * (D * wb + i8);
    bytes[SLI_FAM_DOWN] = D * (m->Il * wb + i8);
    bytes[SLI_FAM_LM] = (double)m->v_n * (D * wb + i8);
    int rc = SLI_OK;
    for (int f = 0; rc == SLI_OK && f < SLI_FAM_COUNT; ++f) {
        launches[f] = f == SLI_FAM_LM ? 1 : m->L;
        rc = SLI_DISPATCH(m, family, m, f);  // warm-up
        if (rc == SLI_OK && hipEventRecord(g.e0, m->stream) != hipSuccess) rc = fail(SLI_ERR_HIP, "event");
        for (int i = 0; rc == SLI_OK && i < iters; ++i) rc = SLI_DISPATCH(m, family, m, f);
        if (rc == SLI_OK && hipEventRecord(g.e1, m->stream) != hipSuccess) rc = fail(SLI_ERR_HIP, "event");
        float ms = 0.0f;
        if (rc == SLI_OK &&
            (rc = wait_event(m, g.e1)) == SLI_OK && hipEventElapsedTime(&ms, g.e0, g.e1) != hipSuccess)
            rc = fail(SLI_ERR_HIP, "event timing");
        us[f] = 1000.0 * ms / ((double)iters * launches[f]);
    }
    if (hipMemcpyAsync(m->x, g.xsave, xb, hipMemcpyDeviceToDevice, m->stream) != hipSuccess) {
        if (rc == SLI_OK) rc = fail(SLI_ERR_HIP, "restore x");
    } else if (rc == SLI_OK) {
        rc = wait_stream(m);
    }
    return rc;
}

namespace sli {
// pure streaming read of up to three byte ranges (the stream floor of sli_model_time_stream): workgroup b
// reads its contiguous 1/grid share of each range, 8 x 16 B per lane in flight
__global__ void __launch_bounds__(1024) stream_read_kernel(const char* a, long long na, const char* b, long long nb,
                                                           const char* c, long long nc, float* sink) {
    float acc = 0.0f;
    for (int r = 0; r < 3; ++r) {
        const char* base = r == 0 ? a : r == 1 ? b : c;
        const long long n = r == 0 ? na : r == 1 ? nb : nc;
        if (!base || n < 16) continue;
        const long long per = (n / 16 + gridDim.x - 1) / gridDim.x;  // 16-B vectors per workgroup
        const long long v0 = per * blockIdx.x, v1 = min(v0 + per, n / 16);
        for (long long v = v0 + threadIdx.x; v < v1; v += 8 * 1024) {
            u32x4 w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = load16<true>(base + min(v + j * 1024, v1 - 1) * 16);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += __uint_as_float(w[j].x ^ w[j].w);
        }
    }
    if (acc == 1.2345f) sink[threadIdx.x] = acc;  // never: keeps the loads
}
}  // namespace sli

int sli_model_time_stream(sli_model* m, int32_t iters, double* us) {
    SLI_CHECK(m && iters > 0 && us, SLI_ERR_ARG, "bad argument");
    SLI_CHECK(!m->group, SLI_ERR_STATE, "time a group's ranks through a standalone model");
    SLI_HIP(hipSetDevice(m->c.device));
    struct Guard {
        float* sink = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        ~Guard() {
            if (sink) (void)hipFree(sink);
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
        }
    } g;
    SLI_HIP(hipMalloc(&g.sink, 4096));
    SLI_HIP(hipEventCreate(&g.e0));
    SLI_HIP(hipEventCreate(&g.e1));
    const long long wb = m->wbytes, D = m->D, hd = m->hd;
    const long long kvl = (long long)m->B * m->hkv * m->T * hd * m->kvbytes;  // one layer's K (or V)
    const int grid = device_cus();
    auto launch = [&](int f, int l) {
        const char *a = nullptr, *b = nullptr, *c = nullptr;
        long long na = 0, nb = 0, nc = 0;
        const LayerW& w = m->layers[f == SLI_FAM_LM ? 0 : l];
        switch (f) {
            case SLI_FAM_QKV: a = (const char*)w.qkv; na = (m->hq + 2LL * m->hkv) * hd * D * wb; break;
            case SLI_FAM_ATTN:
                a = (const char*)m->kc + l * kvl;
                b = (const char*)m->vc + l * kvl;
                na = nb = kvl;
                break;
            case SLI_FAM_WO: a = (const char*)w.wo; na = D * m->hq * hd * wb; break;
            case SLI_FAM_GU: a = (const char*)w.gu; na = 2LL * m->Il * D * wb; break;
            case SLI_FAM_DOWN: a = (const char*)w.down; na = D * m->Il * wb; break;
            default: a = (const char*)m->emb + (long long)m->v_lo * D * wb; na = (long long)m->v_n * D * wb; break;
        }
        hipLaunchKernelGGL(stream_read_kernel, dim3(grid), dim3(1024), 0, m->stream, a, na, b, nb, c, nc, g.sink);
    };
    for (int f = 0; f < SLI_FAM_COUNT; ++f) {
        const int n = f == SLI_FAM_LM ? 1 : m->L;
        for (int l = 0; l < n; ++l) launch(f, l);  // warm-up
        SLI_HIP(hipEventRecord(g.e0, m->stream));
        for (int i = 0; i < iters; ++i)
            for (int l = 0; l < n; ++l) launch(f, l);
        SLI_HIP(hipEventRecord(g.e1, m->stream));
        SLI_HIP(hipGetLastError());
        float ms = 0.0f;
        SLI_TRY(wait_event(m, g.e1));
        SLI_HIP(hipEventElapsedTime(&ms, g.e0, g.e1));
        us[f] = 1000.0 * ms / ((double)iters * n);
    }
    return SLI_OK;
}

int sli_model_time_gemv(sli_model* m, int32_t iters, double* avg_us, double* bytes_per_launch,
                        int32_t* launches_per_step) {
    SLI_CHECK(m && iters > 0, SLI_ERR_ARG, "bad argument");
    SLI_HIP(hipSetDevice(m->c.device));
    SLI_TRY(bg_sync_tiles(m));  // the batched launches stream the fragment-layout copies
    // The probe re-runs the step's weight-streaming launches in place. It saves and restores the residual
    // stream x; its QKV launches rewrite each layer's K/V row at the current position (from the final x),
    // which the next real step at that position overwrites again (the bench's idempotent step does).
    struct Guard {  // every exit path frees the save buffer and both events
        float* xsave = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        ~Guard() {
            if (xsave) (void)hipFree(xsave);
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
        }
    } g;
    const size_t xb = sizeof(float) * m->B * m->D;
    SLI_HIP(hipMalloc(&g.xsave, xb));
    SLI_HIP(hipMemcpyAsync(g.xsave, m->x, xb, hipMemcpyDeviceToDevice, m->stream));
    SLI_HIP(hipEventCreate(&g.e0));
    SLI_HIP(hipEventCreate(&g.e1));
    int rc = SLI_DISPATCH(m, gemvs, m);  // warm-up
    if (rc == SLI_OK) rc = hipEventRecord(g.e0, m->stream) == hipSuccess ? SLI_OK : fail(SLI_ERR_HIP, "event");
    for (int i = 0; rc == SLI_OK && i < iters; ++i) rc = SLI_DISPATCH(m, gemvs, m);
    if (rc == SLI_OK) rc = hipEventRecord(g.e1, m->stream) == hipSuccess ? SLI_OK : fail(SLI_ERR_HIP, "event");
    float ms = 0.0f;
    if (rc == SLI_OK && (rc = wait_event(m, g.e1)) == SLI_OK && hipEventElapsedTime(&ms, g.e0, g.e1) != hipSuccess)
        rc = fail(SLI_ERR_HIP, "event timing");
    if (hipMemcpyAsync(m->x, g.xsave, xb, hipMemcpyDeviceToDevice, m->stream) != hipSuccess) {
        if (rc == SLI_OK) rc = fail(SLI_ERR_HIP, "restore x");
    } else if (rc == SLI_OK) {
        rc = wait_stream(m);
    }
    if (rc != SLI_OK) return rc;
    const int n_launch = 4 * m->L + 1;
    double wbytes = 0.0;
    SLI_TRY(sli_model_step_bytes(m, &wbytes, nullptr));
    if (avg_us) *avg_us = 1000.0 * ms / ((double)iters * n_launch);
    if (bytes_per_launch) *bytes_per_launch = wbytes / n_launch;
    if (launches_per_step) *launches_per_step = n_launch;
    return SLI_OK;
}

// ---------------------------------------------------------------- in-process tensor-parallel group
int sli_tp_group_create(const sli_model_config* cfg, int32_t tp_size, sli_tp_group** out) {
    SLI_CHECK(cfg && out, SLI_ERR_ARG, "sli_tp_group_create: null");
    SLI_CHECK(tp_size >= 1 && tp_size <= kMaxGroup, SLI_ERR_ARG, "tp group size must be in [1, 8]");
    SLI_HIP(hipSetDevice(cfg->device));
    sli_tp_group* g = new sli_tp_group();
    g->n = tp_size;
    g->device = cfg->device;
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
        delete g;
        return fail(SLI_ERR_HIP, "hipStreamCreate");
    }
    for (int r = 0; r < tp_size; ++r) {
        sli_model_config c = *cfg;
        c.tp_rank = r;
        c.tp_size = tp_size;
        sli_model* m = nullptr;
        const int rc = create_model(&c, nullptr, g, &m);
        if (rc != SLI_OK) {
            const std::string err = sli_last_error();
            sli_tp_group_destroy(g);
            return fail(rc, err);
        }
        g->ranks.push_back(m);
    }
    *out = g;
    return SLI_OK;
}

int sli_tp_group_destroy(sli_tp_group* g) {
    if (!g) return SLI_OK;
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    if (g->graph) (void)hipGraphDestroy(g->graph);
    for (int b = 0; b < 4; ++b) {
        if (g->pf_exec[b]) (void)hipGraphExecDestroy(g->pf_exec[b]);
        if (g->pf_graph[b]) (void)hipGraphDestroy(g->pf_graph[b]);
    }
    for (sli_model* m : g->ranks) destroy(m);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
    return SLI_OK;
}

int sli_tp_group_rank(sli_tp_group* g, int32_t rank, sli_model** out) {
    SLI_CHECK(g && out, SLI_ERR_ARG, "null argument");
    SLI_CHECK(rank >= 0 && rank < g->n, SLI_ERR_RANGE, "rank out of range");
    *out = g->ranks[rank];
    return SLI_OK;
}

int sli_tp_group_step(sli_tp_group* g) {
    SLI_CHECK(g, SLI_ERR_ARG, "null group");
    SLI_HIP(hipSetDevice(g->device));
    SLI_TRY(capture_group(g));
    SLI_HIP(hipGraphLaunch(g->exec, g->stream));
    return SLI_OK;
}

int sli_tp_group_sync(sli_tp_group* g) {
    SLI_CHECK(g, SLI_ERR_ARG, "null group");
    SLI_HIP(hipStreamSynchronize(g->stream));
    return SLI_OK;
}

int sli_tp_group_predict_prefill(sli_tp_group* g, const int32_t* prompt, int32_t n_prompt, int32_t max_length,
                                 int32_t* tokens_out, float* logits_out) {
    SLI_CHECK(g && prompt && tokens_out, SLI_ERR_ARG, "null argument");
    sli_model* m0 = g->ranks[0];
    SLI_CHECK(max_length >= n_prompt && max_length <= m0->T, SLI_ERR_RANGE,
              "max_length must be in [n_prompt, max_len]");
    SLI_TRY(sli_tp_group_prefill(g, prompt, n_prompt));
    const size_t V = (size_t)m0->V;
    if (logits_out)
        for (size_t i = 0; i < (size_t)(n_prompt - 1) * V; ++i) logits_out[i] = NAN;
    for (int t = n_prompt - 1; t < max_length; ++t) {
        SLI_TRY(sli_tp_group_step(g));
        if (!logits_out) continue;
        for (sli_model* m : g->ranks)
            SLI_HIP(hipMemcpyAsync(logits_out + (size_t)t * V + m->v_lo, m->logits, sizeof(float) * m->v_n,
                                   hipMemcpyDeviceToHost, g->stream));
        SLI_HIP(hipStreamSynchronize(g->stream));
    }
    SLI_HIP(hipMemcpyAsync(tokens_out, m0->hist, sizeof(int32_t) * max_length, hipMemcpyDeviceToHost, g->stream));
    SLI_HIP(hipStreamSynchronize(g->stream));
    for (sli_model* m : g->ranks) SLI_TRY(check_device_errors(m));
    return SLI_OK;
}

int sli_tp_group_predict_batch(sli_tp_group* g, const int32_t* prompts, const int32_t* lens, int32_t ld,
                               int32_t max_length, int32_t* tokens_out, float* logits_out) {
    SLI_CHECK(g && prompts && lens && tokens_out, SLI_ERR_ARG, "null argument");
    sli_model* m0 = g->ranks[0];
    SLI_CHECK(max_length >= 1 && max_length <= m0->T, SLI_ERR_RANGE, "max_length must be in [1, max_len]");
    for (sli_model* m : g->ranks) {
        for (int b = 0; b < m->B; ++b) {
            SLI_CHECK(lens[b] >= 1 && lens[b] <= ld, SLI_ERR_RANGE, "prompt length out of range");
            SLI_TRY(set_prompt(m, b, prompts + (size_t)b * ld, lens[b]));
            SLI_TRY(set_state(m, b, prompts[(size_t)b * ld], 0, 1));
        }
    }
    const int B = m0->B, V = m0->V;
    for (int t = 0; t < max_length; ++t) {  // model.cpp:157
        SLI_TRY(sli_tp_group_step(g));
        if (!logits_out) continue;
        for (sli_model* m : g->ranks)  // [t][b][v_lo .. v_lo + v_n) <- rank's [b][v_n]
            SLI_HIP(hipMemcpy2DAsync(logits_out + ((size_t)t * B) * V + m->v_lo, sizeof(float) * V, m->logits,
                                     sizeof(float) * m->v_n, sizeof(float) * m->v_n, B, hipMemcpyDeviceToHost,
                                     g->stream));
        SLI_HIP(hipStreamSynchronize(g->stream));
    }
    for (int b = 0; b < B; ++b)
        SLI_HIP(hipMemcpyAsync(tokens_out + (size_t)b * max_length, m0->hist + (size_t)b * (m0->T + 1),
                               sizeof(int32_t) * max_length, hipMemcpyDeviceToHost, g->stream));
    SLI_HIP(hipStreamSynchronize(g->stream));
    for (sli_model* m : g->ranks) SLI_TRY(check_device_errors(m));
    return SLI_OK;
}

}  // extern "C"
