// ops.hip — kernel-level C ABI (include/sli.h): one entry point per reference CUDA launcher in
// include/kernel/cuda/*.cuh, with the reference CPU kernels' semantics (the oracle).
#include <cmath>
#include <type_traits>
#include <vector>

#include "attention.h"
#include "attn_mfma.h"
#include "bgemm.h"
#include "common.h"
#include "gemv.h"
#include "ops_internal.h"
#include "rope_table.h"

namespace sli {

// ---------------------------------------------------------------- RMSNorm (rms_kernel.cpp:5-23)
// One workgroup: the whole vector is one reduction, so no cross-block atomics (the reference CUDA
// kernel's multi-block atomicAdd has no grid barrier, rms_kernel.cu:29-33).
__global__ void __launch_bounds__(1024) rmsnorm_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                      float* __restrict__ y, int dim, float eps) {
    __shared__ float red[16];
    __shared__ float inv_s;
    float ss = 0.0f;
    for (int i = threadIdx.x; i < dim; i += blockDim.x) {
        float v = x[i];
        ss += v * v;
    }
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.0f;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
        float tep = t / (float)dim;
        float rms = sqrtf(tep + eps);
        inv_s = 1.0f / rms;
    }
    __syncthreads();
    const float inv = inv_s;
    for (int i = threadIdx.x; i < dim; i += blockDim.x) y[i] = (x[i] * inv) * w[i];
}

// ---------------------------------------------------------------- RoPE (rope_kernel.cpp:22-41)
__global__ void rope_kernel(float* __restrict__ q, float* __restrict__ k, int pos_host, const int32_t* pos_dev,
                            const float* __restrict__ sin_t, const float* __restrict__ cos_t, int q_dim, int k_dim,
                            int head_dim) {
    const int half = head_dim / 2;
    const int pos = pos_dev ? *pos_dev : pos_host;
    const int nq = q_dim / 2, nk = k_dim / 2;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nq + nk; i += gridDim.x * blockDim.x) {
        float* vec = i < nq ? q : k;
        const int j = i < nq ? i : i - nq;
        const int head = j / half, d = j - head * half;
        const float fci = sin_t[pos * half + d], fcr = cos_t[pos * half + d];
        float* p = vec + head * head_dim;
        const float v0 = p[d], v1 = p[d + half];
        p[d] = v0 * fcr - v1 * fci;
        p[d + half] = v1 * fcr + v0 * fci;
    }
}

// ---------------------------------------------------------------- softmax (mha_kernel.cpp:7-20)
__global__ void __launch_bounds__(1024) softmax_kernel(float* __restrict__ x, int n) {
    __shared__ float red[16];
    __shared__ float bc;
    float m = -INFINITY;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, x[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = -INFINITY;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t = fmaxf(t, red[i]);
        bc = t;
    }
    __syncthreads();
    m = bc;
    float s = 0.0f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        float e = expf(x[i] - m);
        x[i] = e;
        s += e;
    }
    s = wave_sum(s);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.0f;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
        bc = t;
    }
    __syncthreads();
    s = bc;
    for (int i = threadIdx.x; i < n; i += blockDim.x) x[i] /= s;
}

// ---------------------------------------------------------------- SwiGLU / add (elementwise)
__global__ void swiglu_kernel(const float* __restrict__ up, const float* __restrict__ gate, float* __restrict__ out,
                              int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float t = 1.0f / (1.0f + expf(-gate[i]));  // swiglu_kernel.cpp:12
        out[i] = t * up[i];                               // :13
    }
}

__global__ void add_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ out, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = a[i] + b[i];
}

// ---------------------------------------------------------------- embedding (emb_kernel.cpp:4-21)
template <typename T>
__global__ void embedding_kernel(int token_host, const int32_t* token_dev, const T* __restrict__ table,
                                 const float* row_scale, float* __restrict__ out, int vocab, int dim) {
    const int token = token_dev ? *token_dev : token_host;
    const bool ok = token >= 0 && token < vocab;
    const float s = (ok && row_scale) ? row_scale[token] : 1.0f;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < dim; i += gridDim.x * blockDim.x)
        out[i] = ok ? to_f32(table[(size_t)token * dim + i]) * s : __int_as_float(0x7FC00000);  // poison: NaN
}

// ---------------------------------------------------------------- argmax (argmax.cpp:7-17)
__global__ void __launch_bounds__(1024) argmax_kernel(const float* __restrict__ x, int n, int32_t* out) {
    __shared__ unsigned long long red[16];
    unsigned long long best = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        unsigned long long k = argmax_key(x[i], (unsigned)i);
        best = k > best ? k : best;
    }
    best = wave_max_u64(best);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) b = red[i] > b ? red[i] : b;
        *out = (int32_t)argmax_key_index(b);
    }
}

// ---------------------------------------------------------------- dispatch helpers
template <typename WT>
static int matmul_dispatch(const float* x, const WT* w, const float* rscale, float* y, int rows, int cols, float scale,
                           hipStream_t s) {
    const bool vec_ok = ((uintptr_t)w % 16 == 0) && ((uintptr_t)x % 16 == 0) && (cols % 4 == 0) &&
                        (((size_t)cols * sizeof(WT)) % 16 == 0) && cols <= kGemvMaxCols;
    if (vec_ok) {
        EpiStore<2> epi{y, nullptr, rscale, scale, rows};
        GemvIn in{x, nullptr, 0.0f, cols};
        SLI_HIP((launch_gemv_u<WT, 2, 4, true>(w, in, epi, (rows + 1) / 2, s)));  // column split below 4096 units
    } else {
        const int blocks = std::min(gemv_max_blocks(), (rows + 3) / 4);
        hipLaunchKernelGGL(gemv_scalar_kernel<WT>, dim3(blocks), dim3(kGemvThreads), 0, s, w, x, rscale, y, rows,
                           cols, scale);
        SLI_HIP(hipGetLastError());
    }
    return SLI_OK;
}

int attn_wg_positions(int kv_dtype, int head_dim) {
    const int epv = kv_dtype == SLI_DT_F16 ? 8 : 4;
    return kAttnSlots * (64 / (head_dim / epv));
}

// The MFMA decode attention (attn_mfma.h) for an fp16 cache. SLI_ATTN_MFMA=0 at build time keeps the
// register-staged kernel (attention.h) everywhere, for an A/B variant build.
#ifndef SLI_ATTN_MFMA
#define SLI_ATTN_MFMA 1
#endif
static bool attn_mfma_ok(const AttnArgs<__half>& a, int g) {
    // the batch-1 MHA step (C1 / C3) merges its splits in the wo GEMV's input staging (defer_merge 1), where the
    // register-staged kernel's 8.5 us stays ahead (tools/attn_mfma_lab: 9.1 vs 10.6 us at C1, both ramp-bound: 131 KB
    // per CU); every other fp16 attention (GQA batches and shards, op level) runs on the matrix cores
    if (!SLI_ATTN_MFMA || a.cache_heads != 0 || !(g == 1 || g == 2 || g == 4 || g == 8) || a.defer_merge == 1)
        return false;
    // every 16-byte DMA piece aligned: cache bases, row and head strides, q
    return (uintptr_t)a.k % 16 == 0 && (uintptr_t)a.v % 16 == 0 && (uintptr_t)a.q % 16 == 0 && a.pos_stride % 8 == 0 &&
           a.head_stride % 8 == 0;
}
template <int HD, int G>
static void attn_mfma_go(const AttnArgs<__half>& a, int blocks, int nbuf, hipStream_t s) {
    if (nbuf == 1)
        hipLaunchKernelGGL((attn_mfma_kernel<HD, G, 1>), dim3(blocks), dim3(64 * kAmWaves), 0, s, a);
    else
        hipLaunchKernelGGL((attn_mfma_kernel<HD, G, 2>), dim3(blocks), dim3(64 * kAmWaves), 0, s, a);
}
// Split geometry: one workgroup per CU over the whole context (attn_mfma_tpw), its splits merged by the head's
// last-arriving workgroup inside the launch (a requested merge launch, defer_merge 2, becomes that in-launch
// merge: the same result in out).
template <int HD>
static int attn_mfma_launch(AttnArgs<__half> a, int g, int T, hipStream_t s) {
    // the partial buffer (mha_part_bytes) holds ceil(T / pf) splits per head, pf = the fp32 kernel's positions per
    // workgroup; at head_dim 64 that is 256 keys, so one tile per wave (128 keys) over a longer context would store
    // past it (the round-5 fault record): the split is never shorter than pf
    const int pf = attn_wg_positions(SLI_DT_F32, HD);
    const int tpw = std::max(attn_mfma_tpw(a.n_kv_heads, T, device_cus()), (pf + kAmWgKeys - 1) / kAmWgKeys);
    a.ppwg = kAmWgKeys * tpw;
    a.max_splits = (T + a.ppwg - 1) / a.ppwg;
    if (a.max_splits > kAttnMaxWgSplits) return fail(SLI_ERR_SHAPE, "mha: context too long for the split merge");
    if (a.max_splits > (T + pf - 1) / pf) return fail(SLI_ERR_SHAPE, "mha: more splits than the partial buffer holds");
    if (a.defer_merge == 2) a.defer_merge = 0;
    const int blocks = a.n_kv_heads * a.max_splits, nbuf = tpw > 1 ? 2 : 1;
    switch (g) {
        case 1: attn_mfma_go<HD, 1>(a, blocks, nbuf, s); break;
        case 2: attn_mfma_go<HD, 2>(a, blocks, nbuf, s); break;
        case 4: attn_mfma_go<HD, 4>(a, blocks, nbuf, s); break;
        default: attn_mfma_go<HD, 8>(a, blocks, nbuf, s); break;
    }
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

template <typename KT, int HD>
static int mha_launch_hd(const float* q, const KT* kc, const KT* vc, float* out, int layer, int pos, const int32_t* pos_dev,
                         int T, int H, int Hkv, long long pos_stride, long long head_stride, long long layer_stride,
                         float* part, unsigned* counters, hipStream_t s, int seq_heads, int pos_seq_stride,
                         int cache_heads, int defer_merge) {
    using Geo = AttnGeom<KT, HD>;
    constexpr int ppw_wg = Geo::PPWG;
    const int wg_splits = (T + ppw_wg - 1) / ppw_wg;
    if (wg_splits > kAttnMaxWgSplits) return fail(SLI_ERR_SHAPE, "mha: context too long for the split merge");
    AttnArgs<KT> a{q,    kc + (long long)layer * layer_stride, vc + (long long)layer * layer_stride, pos_stride,
                   head_stride, part, out, counters, pos_dev, pos, Hkv, wg_splits, 1.0f / sqrtf((float)HD),
                   seq_heads > 0 ? seq_heads : Hkv, pos_seq_stride};
    a.cache_heads = cache_heads;
    a.defer_merge = defer_merge;
    int g = H / Hkv;
    if constexpr (std::is_same<KT, __half>::value) {
        if (attn_mfma_ok(a, g)) return attn_mfma_launch<HD>(a, g, T, s);
    }
    // GQA-4 as two GQA-2 groups per kv head: the 59-VGPR GQA-2 kernel at 8 waves/SIMD instead of the 128-VGPR GQA-4
    // one at 4; the two groups of a kv head are wg_splits blocks apart and read the same K/V rows. Deferred merges
    // only (partials are indexed by q head; the counters by kv head), where the unsplit grid fills at most half the
    // chip. Measured (profiles/r4_gqa_split_ab.txt): Llama-3-8B batch 1 (8 kv heads x 16 splits = 128 workgroups)
    // attention 10.7 -> 8.1 us; C4 (1024 workgroups) 34.5 -> 41 us, so off there.
    if (g == 4 && defer_merge && cache_heads == 0 && 2 * Hkv * wg_splits <= device_cus()) {
        g = 2;
        a.kv_group = 2;
        a.n_kv_heads = 2 * Hkv;
        a.seq_heads *= 2;
        Hkv *= 2;
    }
    const int blocks = Hkv * wg_splits;
    switch (g) {
        case 1: hipLaunchKernelGGL((attn_partial_kernel<KT, HD, 1>), dim3(blocks), dim3(64 * attn_waves(1)), 0, s, a); break;
        case 2: hipLaunchKernelGGL((attn_partial_kernel<KT, HD, 2>), dim3(blocks), dim3(64 * attn_waves(2)), 0, s, a); break;
        case 4: hipLaunchKernelGGL((attn_partial_kernel<KT, HD, 4>), dim3(blocks), dim3(64 * attn_waves(4)), 0, s, a); break;
        case 8: hipLaunchKernelGGL((attn_partial_kernel<KT, HD, 8>), dim3(blocks), dim3(64 * attn_waves(8)), 0, s, a); break;
        default: return fail(SLI_ERR_SHAPE, "mha: heads per kv head must be 1, 2, 4 or 8");
    }
    SLI_HIP(hipGetLastError());
    if (defer_merge == 2) {
        const dim3 mb(kAttnMergeThreads);
        switch (g) {
            case 1: hipLaunchKernelGGL((attn_merge_kernel<KT, HD, 1>), dim3(Hkv * attn_merge_wgs(HD)), mb, 0, s, a); break;
            case 2: hipLaunchKernelGGL((attn_merge_kernel<KT, HD, 2>), dim3(Hkv * attn_merge_wgs(2 * HD)), mb, 0, s, a); break;
            case 4: hipLaunchKernelGGL((attn_merge_kernel<KT, HD, 4>), dim3(Hkv * attn_merge_wgs(4 * HD)), mb, 0, s, a); break;
            default: hipLaunchKernelGGL((attn_merge_kernel<KT, HD, 8>), dim3(Hkv * attn_merge_wgs(8 * HD)), mb, 0, s, a); break;
        }
        SLI_HIP(hipGetLastError());
    }
    return SLI_OK;
}

template <typename KT>
int mha_launch(const float* q, const KT* kc, const KT* vc, float* out, int layer, int pos, const int32_t* pos_dev,
               int T, int hd, int H, int Hkv, long long pos_stride, long long head_stride, long long layer_stride,
               float* part, unsigned* counters, hipStream_t s, int seq_heads, int pos_seq_stride, int cache_heads,
               int defer_merge) {
    if (hd == 128)
        return mha_launch_hd<KT, 128>(q, kc, vc, out, layer, pos, pos_dev, T, H, Hkv, pos_stride, head_stride,
                                      layer_stride, part, counters, s, seq_heads, pos_seq_stride, cache_heads, defer_merge);
    if (hd == 64)
        return mha_launch_hd<KT, 64>(q, kc, vc, out, layer, pos, pos_dev, T, H, Hkv, pos_stride, head_stride,
                                     layer_stride, part, counters, s, seq_heads, pos_seq_stride, cache_heads, defer_merge);
    return fail(SLI_ERR_SHAPE, "mha: head_dim must be 64 or 128");
}

template int mha_launch<float>(const float*, const float*, const float*, float*, int, int, const int32_t*, int, int,
                               int, int, long long, long long, long long, float*, unsigned*, hipStream_t, int, int,
                               int, int);
template int mha_launch<__half>(const float*, const __half*, const __half*, float*, int, int, const int32_t*, int,
                                int, int, int, long long, long long, long long, float*, unsigned*, hipStream_t, int,
                                int, int, int);

size_t mha_part_bytes(int T, int H, int hd) {
    const int ppw_wg_min = attn_wg_positions(SLI_DT_F32, hd);
    const size_t splits = (size_t)((T + ppw_wg_min - 1) / ppw_wg_min);
    return (sizeof(float) * (size_t)H * splits * (size_t)(hd + kAttnPartPad) + 255) & ~(size_t)255;
}

// split partials, then one arrival counter per kv head (<= H)
size_t mha_workspace_bytes(int T, int H, int hd) { return mha_part_bytes(T, H, hd) + sizeof(unsigned) * (size_t)H; }

int embedding_launch(int token, const int32_t* token_dev, const void* table, int dtype, const float* row_scale,
                     float* out, int vocab, int dim, hipStream_t s) {
    const int blocks = std::min(64, (dim + 255) / 256);
    if (dtype == SLI_DT_F32)
        hipLaunchKernelGGL(embedding_kernel<float>, dim3(blocks), dim3(256), 0, s, token, token_dev,
                           (const float*)table, row_scale, out, vocab, dim);
    else if (dtype == SLI_DT_F16)
        hipLaunchKernelGGL(embedding_kernel<__half>, dim3(blocks), dim3(256), 0, s, token, token_dev,
                           (const __half*)table, row_scale, out, vocab, dim);
    else if (dtype == SLI_DT_I8)
        hipLaunchKernelGGL(embedding_kernel<int8_t>, dim3(blocks), dim3(256), 0, s, token, token_dev,
                           (const int8_t*)table, row_scale, out, vocab, dim);
    else
        return fail(SLI_ERR_ARG, "embedding: bad dtype");
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

}  // namespace sli

using namespace sli;

extern "C" {

int sli_matmul(const float* x, const void* w, int w_dtype, const float* w_row_scale, float* y, int32_t rows,
               int32_t cols, float scale, sli_stream_t stream) {
    SLI_CHECK(x && w && y, SLI_ERR_ARG, "sli_matmul: null pointer");
    SLI_CHECK(rows > 0 && cols > 0, SLI_ERR_SHAPE, "sli_matmul: Tensor with Wrong Dim!");
    hipStream_t s = as_stream(stream);
    switch (w_dtype) {
        case SLI_DT_F32: return matmul_dispatch<float>(x, (const float*)w, w_row_scale, y, rows, cols, scale, s);
        case SLI_DT_F16: return matmul_dispatch<__half>(x, (const __half*)w, w_row_scale, y, rows, cols, scale, s);
        case SLI_DT_I8:
            SLI_CHECK(w_row_scale, SLI_ERR_ARG, "sli_matmul: int8 weights need row scales");
            return matmul_dispatch<int8_t>(x, (const int8_t*)w, w_row_scale, y, rows, cols, scale, s);
        default: return fail(SLI_ERR_ARG, "sli_matmul: bad dtype");
    }
}

size_t sli_matmul_batch_workspace_bytes(int32_t rows, int32_t cols, int32_t batch) {
    if (rows <= 0 || cols <= 0 || batch <= 0 || batch > kBgMaxBatch || cols % 32 != 0) return 0;
    return bg_ws_bytes(bg_plan((rows + 15) / 16, cols, batch, false, device_cus()));
}

int sli_matmul_batch(const float* x, const void* w, int w_dtype, float* y, int32_t rows, int32_t cols, int32_t batch,
                     void* workspace, size_t workspace_bytes, sli_stream_t stream) {
    SLI_CHECK(x && w && y && workspace, SLI_ERR_ARG, "sli_matmul_batch: null pointer");
    SLI_CHECK(w_dtype == SLI_DT_F16, SLI_ERR_ARG, "sli_matmul_batch: fp16 weights only");
    SLI_CHECK(rows > 0 && cols > 0 && cols % 32 == 0, SLI_ERR_SHAPE, "sli_matmul_batch: cols must be a multiple of 32");
    SLI_CHECK(batch >= 1 && batch <= kBgMaxBatch, SLI_ERR_SHAPE, "sli_matmul_batch: batch must be in [1, 8]");
    SLI_CHECK((uintptr_t)x % 16 == 0 && (uintptr_t)w % 16 == 0, SLI_ERR_ARG, "sli_matmul_batch: 16-byte alignment");
    const BgPlan p = bg_plan((rows + 15) / 16, cols, batch, false, device_cus());
    SLI_CHECK(p.groups > 0, SLI_ERR_SHAPE, "sli_matmul_batch: no tiling fits");
    SLI_CHECK(workspace_bytes >= bg_ws_bytes(p), SLI_ERR_ARG, "sli_matmul_batch: workspace too small");
    hipStream_t s = as_stream(stream);
    unsigned* cnt = (unsigned*)((char*)workspace + bg_part_bytes(p));
    SLI_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned) * p.groups, s));
    SLI_HIP((bg_allow_lds<BgEpiStore, false>()));
    BgIn in{x, nullptr, 0.0f, cols, batch, 0, 0, 0, (float*)workspace, cnt};
    BgEpiStore e{y, nullptr, nullptr, 1.0f, rows, rows};
    SLI_HIP(launch_bgemm((const __half*)w, in, e, p, s));
    return SLI_OK;
}

int sli_rmsnorm(const float* x, const float* w, float* y, int32_t dim, float eps, sli_stream_t stream) {
    SLI_CHECK(x && w && y, SLI_ERR_ARG, "sli_rmsnorm: null pointer");
    SLI_CHECK(dim > 0, SLI_ERR_SHAPE, "sli_rmsnorm: dim");
    hipLaunchKernelGGL(rmsnorm_kernel, dim3(1), dim3(1024), 0, as_stream(stream), x, w, y, dim, eps);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

int sli_rope_cache(int32_t head_dim, int32_t max_seq_len, float* sin_dev, float* cos_dev, float theta,
                   sli_stream_t stream) {
    SLI_CHECK(sin_dev && cos_dev, SLI_ERR_ARG, "sli_rope_cache: null pointer");
    SLI_CHECK(head_dim > 0 && head_dim % 2 == 0 && max_seq_len > 0, SLI_ERR_SHAPE, "sli_rope_cache: shape");
    std::vector<float> s, c;
    rope_table_host(head_dim, max_seq_len, theta, s, c);
    hipStream_t st = as_stream(stream);
    SLI_HIP(hipMemcpyAsync(sin_dev, s.data(), s.size() * 4, hipMemcpyHostToDevice, st));
    SLI_HIP(hipMemcpyAsync(cos_dev, c.data(), c.size() * 4, hipMemcpyHostToDevice, st));
    SLI_HIP(hipStreamSynchronize(st));
    return SLI_OK;
}

int sli_rope(float* q, float* k, int32_t pos, const int32_t* pos_dev, const float* sin_dev, const float* cos_dev,
             int32_t q_dim, int32_t k_dim, int32_t head_dim, sli_stream_t stream) {
    SLI_CHECK(q && k && sin_dev && cos_dev, SLI_ERR_ARG, "sli_rope: null pointer");
    SLI_CHECK(head_dim > 0 && head_dim % 2 == 0 && q_dim % head_dim == 0 && k_dim % head_dim == 0, SLI_ERR_SHAPE,
              "sli_rope: dims must be multiples of head_dim");
    SLI_CHECK(pos_dev || pos >= 0, SLI_ERR_RANGE, "sli_rope: negative position");
    const int n = (q_dim + k_dim) / 2;
    const int blocks = std::max(1, std::min(256, (n + 255) / 256));
    hipLaunchKernelGGL(rope_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), q, k, pos, pos_dev, sin_dev,
                       cos_dev, q_dim, k_dim, head_dim);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

size_t sli_mha_workspace_bytes(int32_t max_seq_len, int32_t n_heads, int32_t head_dim) {
    if (max_seq_len <= 0 || n_heads <= 0 || head_dim <= 0) return 0;
    return mha_workspace_bytes(max_seq_len, n_heads, head_dim);
}

int sli_mha(const float* q, const void* kcache, const void* vcache, int kv_dtype, float* out, int32_t layer,
            int32_t pos, int32_t max_seq_len, int32_t head_dim, int32_t n_heads, int32_t n_kv_heads, void* workspace,
            size_t workspace_bytes, sli_stream_t stream) {
    SLI_CHECK(q && kcache && vcache && out && workspace, SLI_ERR_ARG, "sli_mha: null pointer");
    SLI_CHECK(n_heads > 0 && n_kv_heads > 0 && n_heads % n_kv_heads == 0, SLI_ERR_SHAPE, "sli_mha: heads");
    SLI_CHECK(pos >= 0 && pos < max_seq_len && layer >= 0, SLI_ERR_RANGE, "sli_mha: position out of range");
    SLI_CHECK(workspace_bytes >= mha_workspace_bytes(max_seq_len, n_heads, head_dim), SLI_ERR_ARG,
              "sli_mha: workspace too small");
    const long long kv = (long long)n_kv_heads * head_dim;
    hipStream_t s = as_stream(stream);
    unsigned* counters = (unsigned*)((char*)workspace + mha_part_bytes(max_seq_len, n_heads, head_dim));
    SLI_HIP(hipMemsetAsync(counters, 0, sizeof(unsigned) * n_kv_heads, s));
    if (kv_dtype == SLI_DT_F32)
        return mha_launch<float>(q, (const float*)kcache, (const float*)vcache, out, layer, pos, nullptr, max_seq_len,
                                 head_dim, n_heads, n_kv_heads, kv, head_dim, kv * max_seq_len, (float*)workspace,
                                 counters, s);
    if (kv_dtype == SLI_DT_F16)
        return mha_launch<__half>(q, (const __half*)kcache, (const __half*)vcache, out, layer, pos, nullptr,
                                  max_seq_len, head_dim, n_heads, n_kv_heads, kv, head_dim, kv * max_seq_len,
                                  (float*)workspace, counters, s);
    return fail(SLI_ERR_ARG, "sli_mha: bad kv dtype");
}

int sli_softmax(float* x, int32_t n, sli_stream_t stream) {
    SLI_CHECK(x, SLI_ERR_ARG, "sli_softmax: null pointer");
    SLI_CHECK(n > 0, SLI_ERR_SHAPE, "sli_softmax: n");
    hipLaunchKernelGGL(softmax_kernel, dim3(1), dim3(1024), 0, as_stream(stream), x, n);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

int sli_swiglu(const float* up, const float* gate, float* out, int32_t n, sli_stream_t stream) {
    SLI_CHECK(up && gate && out, SLI_ERR_ARG, "sli_swiglu: null pointer");
    SLI_CHECK(n > 0, SLI_ERR_SHAPE, "sli_swiglu: n");
    const int blocks = std::min(1024, (n + 255) / 256);
    hipLaunchKernelGGL(swiglu_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), up, gate, out, n);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

int sli_add(const float* a, const float* b, float* out, int32_t n, sli_stream_t stream) {
    SLI_CHECK(a && b && out, SLI_ERR_ARG, "sli_add: null pointer");
    SLI_CHECK(n > 0, SLI_ERR_SHAPE, "sli_add: n");
    const int blocks = std::min(1024, (n + 255) / 256);
    hipLaunchKernelGGL(add_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), a, b, out, n);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

int sli_embedding(int32_t token, const int32_t* token_dev, const void* table, int dtype, const float* row_scale,
                  float* out, int32_t vocab, int32_t dim, sli_stream_t stream) {
    SLI_CHECK(table && out, SLI_ERR_ARG, "sli_embedding: null pointer");
    SLI_CHECK(vocab > 0 && dim > 0, SLI_ERR_SHAPE, "sli_embedding: shape");
    SLI_CHECK(token_dev || (token >= 0 && token < vocab), SLI_ERR_RANGE, "Token index is greater than vocab size.");
    SLI_CHECK(dtype != SLI_DT_I8 || row_scale, SLI_ERR_ARG, "sli_embedding: int8 table needs row scales");
    return embedding_launch(token, token_dev, table, dtype, row_scale, out, vocab, dim, as_stream(stream));
}

int sli_argmax(const float* logits, int32_t n, int32_t* out_dev, sli_stream_t stream) {
    SLI_CHECK(logits && out_dev, SLI_ERR_ARG, "sli_argmax: null pointer");
    SLI_CHECK(n > 0, SLI_ERR_SHAPE, "sli_argmax: n");
    hipLaunchKernelGGL(argmax_kernel, dim3(1), dim3(1024), 0, as_stream(stream), logits, n, out_dev);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

}  // extern "C"
