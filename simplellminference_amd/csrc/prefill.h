// prefill.h — prompt prefill as real GEMMs over the prompt (the reference teacher-forces the
// prompt one token per forward, source/model/model.cpp:157-165, so every weight is streamed once per prompt
// token). Here a chunk of up to kPfMaxChunk prompt positions runs through each layer together:
//
//   1. pf_norm_split_kernel: per position RMSNorm (rms_kernel.cpp:5-23, fp32) and the split of the fp32
//      result into fp16 hi + lo (hi = fp16(h), lo = fp16(h - hi): h to ~2^-22 relative);
//   2. pgemm_kernel: Y[pos][row] = sum_k W[row][k] * H[pos][k] on MFMA (v_mfma_f32_16x16x32_f16), A = a 16-row
//      weight tile, B = 16 positions' hi columns, then the same tile with the lo columns into the same fp32
//      accumulator (W * (hi + lo)); a workgroup owns 64 weight rows x BM positions, so a weight row is read
//      from HBM once per BM positions (the decode step reads it once per position). Operands are staged
//      through a 3-deep LDS ring by LDS-DMA (global_load_lds_dwordx4: one 1-KiB fragment image per
//      wave-instruction, read back conflict-free by ds_read_b128), two k-blocks in flight behind a counted
//      vmcnt and a raw s_barrier (cdna_hip_programming.md §5 "Pipelining across barriers"). Fused epilogues:
//      RoPE + K/V cache rows + q (model.cpp:52-67), residual add (:86-90, :124-128), SwiGLU (:111-115,
//      written straight as the down projection's hi/lo operand);
//   3. pf_attn_kernel: block-causal attention of a 64-position query block of one head against the cache
//      rows 0 .. position (mha_kernel.cpp:36-77 per query: s_t = q.k_t * scale, softmax, sum p_t v_t), fp32,
//      K/V tiles of 64 positions in LDS, online softmax.
// The chunk's start position and valid count live in device memory (PfState), so one captured graph per
// chunk size serves every chunk of every prompt.
#pragma once
#include "common.h"

namespace sli {

constexpr int kPfMaxChunk = 256;   // prompt positions per weight pass
constexpr int kPgThreads = 256;    // 4 waves: 2 (row halves) x 2 (position halves)
constexpr int kPgBN = 64;          // weight rows per workgroup
constexpr int kPgStages = 3;       // LDS ring depth (k-blocks of 32)

struct PfState {
    int32_t p0;  // position of chunk row 0
    int32_t nv;  // valid chunk rows (the rest is padding: computed, never written to the cache)
};

typedef _Float16 pf_half8 __attribute__((ext_vector_type(8)));
typedef float pf_float4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ pf_float4 pf_mfma(const u32x4& a, const u32x4& b, pf_float4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(pf_half8, a), __builtin_bit_cast(pf_half8, b), c,
                                                  0, 0, 0);
}

// fp32 -> fp16 hi + fp16 lo
__device__ __forceinline__ void pf_split(float v, __half& hi, __half& lo) {
    hi = __float2half_rn(v);
    lo = __float2half_rn(v - __half2float(hi));
}

// ---------------------------------------------------------------- 1. embedding + RMSNorm / split
// x[m] = emb[prompt[p0 + m]] (emb_kernel.cpp:4-21; padding rows repeat the last valid token)
template <typename WT>
__global__ void __launch_bounds__(256) pf_embed_kernel(const PfState* __restrict__ ps, const int32_t* __restrict__ prompt,
                                                      const WT* __restrict__ emb, const float* __restrict__ emb_s,
                                                      float* __restrict__ x, int D) {
    const int m = blockIdx.x;
    const int nv = ps->nv;
    const int tok = prompt[ps->p0 + min(m, nv - 1)];
    const float s = emb_s ? emb_s[tok] : 1.0f;
    for (int i = threadIdx.x; i < D; i += 256) x[(size_t)m * D + i] = to_f32(emb[(size_t)tok * D + i]) * s;
}

// one workgroup per chunk row: h = (x * 1/rms) * w (rms_kernel.cpp:12-22) or plain x (w == nullptr), as hi/lo
__global__ void __launch_bounds__(256) pf_norm_split_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           __half* __restrict__ hi, __half* __restrict__ lo, int D,
                                                           float eps) {
    const int m = blockIdx.x;
    const float* xr = x + (size_t)m * D;
    float inv = 1.0f;
    if (w) {
        float ss = 0.0f;
        for (int i = threadIdx.x; i < D; i += 256) ss += xr[i] * xr[i];
        ss = wave_sum(ss);
        __shared__ float red[4];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
        __syncthreads();
        const float t = red[0] + red[1] + red[2] + red[3];
        const float tep = t / (float)D;      // rms_kernel.cpp:17
        const float rms = sqrtf(tep + eps);  // :18
        inv = 1.0f / rms;                    // :19
    }
    for (int i = threadIdx.x; i < D; i += 256) {
        const float v = w ? (xr[i] * inv) * w[i] : xr[i];  // :20-22
        pf_split(v, hi[(size_t)m * D + i], lo[(size_t)m * D + i]);
    }
}

// ---------------------------------------------------------------- 2. the GEMM
// LDS-DMA of one 1-KiB fragment image: lane i's 16 bytes at gsrc land at LDS byte lds + 16 i (inline asm: the
// compiler neither counts nor drains it; the kernel counts its own vmcnt).
__device__ __forceinline__ void pf_dma(const void* gsrc, unsigned lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds)
        : "memory");
}
template <int N>
__device__ __forceinline__ void pf_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename WT>
struct PgIn {
    const WT* W;        // [N][K] fp16 or int8 (row-major, PyTorch [out][in]; int8 row scales in the epilogue)
    const __half* Bhi;  // [M][K] activations, fp16 hi
    const __half* Blo;  // [M][K] fp16 lo
    int N, K, M;        // rows, depth, chunk rows (a multiple of BM)
};

// Stage geometry. A stage covers KBS k-blocks of 32: fp16 weights one (a weight image = 16 rows x 32 k),
// int8 two (a weight image = 16 rows x 64 k int8 — the same 1 KiB). Images per stage: 4 weight row tiles,
// then for each position tile and k-block the hi and the lo image.
// Epilogue contract: row(t, i) = weight row of 16-row tile t's row i (i < 16, always valid); store(t, i0, m, v)
// gets the fp32 sums of tile rows i0 .. i0+3 (i0 % 4 == 0) for chunk row m.
template <int BM, typename WT>
struct PgGeo {
    static constexpr int KBS = sizeof(WT) == 1 ? 2 : 1;
    static constexpr int PT = BM / 16;             // position tiles per workgroup
    static constexpr int WPT = PT / 2;             // per wave
    static constexpr int NDMA = 4 + 2 * PT * KBS;  // 1-KiB images per stage
    static constexpr int DPW = NDMA / 4;           // per wave
    static constexpr int STAGE = NDMA * 1024;
    static_assert(WPT >= 1 && NDMA % 4 == 0, "BM");
};

// 8 int8 weights -> 8 fp16 (exact): fp16 bits 0x6400 | (b ^ 0x80) = 1024 + b + 128, minus 1152
__device__ __forceinline__ u32x4 pg_i8_to_f16(uint2 w) {
    u32x4 r;
    const unsigned x[2] = {w.x ^ 0x80808080u, w.y ^ 0x80808080u};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        // bytes b0 b1 -> halves (0x64 b0), (0x64 b1) via byte permutes
        const unsigned lo = __builtin_amdgcn_perm(0x64646464u, x[h], 0x05010400u);  // {b0, 0x64, b1, 0x64}
        const unsigned hi = __builtin_amdgcn_perm(0x64646464u, x[h], 0x07030602u);  // {b2, 0x64, b3, 0x64}
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        const h2 k = {(_Float16)1152.0f, (_Float16)1152.0f};
        r[2 * h] = __builtin_bit_cast(unsigned, __builtin_bit_cast(h2, lo) - k);
        r[2 * h + 1] = __builtin_bit_cast(unsigned, __builtin_bit_cast(h2, hi) - k);
    }
    return r;
}

template <class Epi, int BM, typename WT>
__global__ void __launch_bounds__(kPgThreads) pgemm_kernel(PgIn<WT> in, Epi epi, const PfState* __restrict__ ps) {
    using Geo = PgGeo<BM, WT>;
    constexpr int KBS = Geo::KBS;
    extern __shared__ __attribute__((aligned(1024))) char pg_smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int wr = wave & 1, wp = wave >> 1;  // row half, position half
    const int PB = in.M / BM;
    // workgroups that share a row block run on one XCD (blocks b and b + 8 share one under round-robin
    // placement; speed only): the second read of the weight rows hits that XCD's L2
    const int bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const int rb = (slot / PB) * 8 + xcd, pb = slot - (slot / PB) * PB;
    const int nrb = (in.N + kPgBN - 1) / kPgBN;
    if (rb >= nrb) return;  // (uniform) padding of the grid to a multiple of 8 row blocks
    const int ns = in.K / (32 * KBS);  // stages
    const unsigned ring = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)pg_smem;

    // this wave's DMA images: image d in [wave*DPW, (wave+1)*DPW). Lane l of an image: fragment row / column
    // l & 15, k group l >> 4 (8 fp16 or 16 int8 elements).
    const int kg = lane >> 4, c16 = lane & 15;
    const char* src[Geo::DPW];
    int adv[Geo::DPW];  // bytes per stage
#pragma unroll
    for (int j = 0; j < Geo::DPW; ++j) {
        const int d = wave * Geo::DPW + j;
        if (d < 4) {
            const int t = rb * 4 + d;
            const int row = epi.row(min(t, (in.N >> 4) - 1), c16);
            src[j] = reinterpret_cast<const char*>(in.W) + (size_t)row * in.K * sizeof(WT) + kg * 16;
            adv[j] = 64;
        } else {
            const int e = d - 4, r = e >> 1;
            const int pt = r / KBS, kb = r - pt * KBS;
            const __half* B = (e & 1) ? in.Blo : in.Bhi;
            const int m = pb * BM + pt * 16 + c16;
            src[j] = reinterpret_cast<const char*>(B) + ((size_t)m * in.K + kb * 32 + kg * 8) * 2;
            adv[j] = 64 * KBS;
        }
    }
    auto issue = [&](int s) {
        const unsigned dst = ring + (unsigned)((s % kPgStages) * Geo::STAGE);
#pragma unroll
        for (int j = 0; j < Geo::DPW; ++j)
            pf_dma(src[j] + (size_t)s * adv[j], dst + (unsigned)((wave * Geo::DPW + j) * 1024));
    };

    pf_float4 acc[2][Geo::WPT];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < Geo::WPT; ++b) acc[a][b] = pf_float4{0.0f, 0.0f, 0.0f, 0.0f};

    issue(0);
    if (ns > 1) issue(1);
    for (int s = 0; s < ns; ++s) {
        if (s + 1 < ns)
            pf_wait_vm<Geo::DPW>();  // this wave's images of stage s landed (s + 1 may stay in flight)
        else
            pf_wait_vm<0>();
        __builtin_amdgcn_s_barrier();  // every wave's images of s landed; every wave is done with s - 1
        if (s + 2 < ns) issue(s + 2);  // into the buffer of s - 1
        const char* st = pg_smem + (size_t)(s % kPgStages) * Geo::STAGE;
#pragma unroll
        for (int kb = 0; kb < KBS; ++kb) {
            u32x4 af[2], bh[Geo::WPT], bl[Geo::WPT];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const char* img = st + (wr * 2 + a) * 1024;
                if constexpr (KBS == 1) {
                    af[a] = reinterpret_cast<const u32x4*>(img)[lane];
                } else {  // k 32 kb + 8 (l >> 4) .. +8 of row l & 15: 16-k group 2 kb + (l >> 5), half (l >> 4) & 1
                    const int off = ((2 * kb + (lane >> 5)) * 16 + c16) * 16 + 8 * ((lane >> 4) & 1);
                    af[a] = pg_i8_to_f16(*reinterpret_cast<const uint2*>(img + off));
                }
            }
#pragma unroll
            for (int b = 0; b < Geo::WPT; ++b) {
                const int pt = wp * Geo::WPT + b;
                const u32x4* bi = reinterpret_cast<const u32x4*>(st + (4 + 2 * (pt * KBS + kb)) * 1024) + lane;
                bh[b] = bi[0];
                bl[b] = bi[64];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < Geo::WPT; ++b) {
                    acc[a][b] = pf_mfma(af[a], bh[b], acc[a][b]);
                    acc[a][b] = pf_mfma(af[a], bl[b], acc[a][b]);
                }
        }
    }
    // C[i][n] of a 16x16 tile: lane l holds rows 4 (l >> 4) + r, column l & 15
    const int i0 = 4 * (lane >> 4);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const int t = rb * 4 + wr * 2 + a;
        if (t >= (in.N >> 4)) continue;
#pragma unroll
        for (int b = 0; b < Geo::WPT; ++b) {
            const int m = pb * BM + (wp * Geo::WPT + b) * 16 + c16;
            const float v[4] = {acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]};
            epi.store(t, i0, m, v, ps);
        }
    }
}

// ---- epilogues. Tiles hold 4-row groups {first(u), first(u + 1), second(u), second(u + 1)} where a pair is a
// RoPE pair {d, d + hd/2} (q/k/v) or {gate u, up u}, so each lane's 4 rows are 2 complete pairs.
template <typename KT>
struct PgEpiQKV {  // model.cpp:52-67: q (fp32 [M][hq*hd]), rotated k / v rows of the cache at p0 + m
    float* q;
    KT* kc;  // this layer's cache base [hkv][T][hd]
    KT* vc;
    const float* rscale;  // int8 row scales (nullable)
    const float* sin_t;
    const float* cos_t;
    int hq, hkv, hd, T;
    __device__ int row(int t, int i) const {
        const int half = hd >> 1;
        const int u = t * 8 + (i >> 2) * 2 + (i & 1);
        const int uh = u / half, d = u - uh * half;
        return uh * hd + d + ((i & 2) ? half : 0);
    }
    __device__ void store(int t, int i0, int m, const float* v, const PfState* ps) const {
        const int nv = ps->nv, pos = ps->p0 + m;
        const int half = hd >> 1;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int u = t * 8 + (i0 >> 2) * 2 + e;
            const int uh = u / half, d = u - uh * half;
            float a0 = v[e], a1 = v[2 + e];
            if (rscale) {
                a0 *= rscale[uh * hd + d];
                a1 *= rscale[uh * hd + d + half];
            }
            if (uh < hq + hkv) {  // rope_kernel.cpp:30-38
                const int pp = min(pos, T - 1);
                const float fci = sin_t[pp * half + d], fcr = cos_t[pp * half + d];
                const float r0 = a0 * fcr - a1 * fci;
                const float r1 = a1 * fcr + a0 * fci;
                if (uh < hq) {
                    float* qr = q + (size_t)m * hq * hd + (size_t)uh * hd;
                    qr[d] = r0;
                    qr[d + half] = r1;
                } else if (m < nv && pos < T) {
                    KT* kr = kc + ((size_t)(uh - hq) * T + pos) * hd;
                    kr[d] = from_f32<KT>(r0);
                    kr[d + half] = from_f32<KT>(r1);
                }
            } else if (m < nv && pos < T) {
                KT* vr = vc + ((size_t)(uh - hq - hkv) * T + pos) * hd;
                vr[d] = from_f32<KT>(a0);
                vr[d + half] = from_f32<KT>(a1);
            }
        }
    }
};

struct PgEpiSwiGLU {  // model.cpp:99-115: act = sigmoid(g) * u (or SiLU), stored as the down GEMM's hi / lo
    __half* ahi;
    __half* alo;
    const float* rscale;
    int inter, silu;
    __device__ int row(int t, int i) const { return t * 8 + (i >> 2) * 2 + (i & 1) + ((i & 2) ? inter : 0); }
    __device__ void store(int t, int i0, int m, const float* v, const PfState*) const {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int u = t * 8 + (i0 >> 2) * 2 + e;
            float g = v[e], up = v[2 + e];
            if (rscale) {
                g *= rscale[u];
                up *= rscale[inter + u];
            }
            float sg = 1.0f / (1.0f + expf(-g));  // swiglu_kernel.cpp:12
            if (silu) sg = g * sg;
            pf_split(sg * up, ahi[(size_t)m * inter + u], alo[(size_t)m * inter + u]);  // :13
        }
    }
};

struct PgEpiResid {  // y[m][row] = resid[m][row] + sum * row scale (matmul_kernel.cpp:26 + add_kernel.cpp:5-14)
    float* y;        // [M][ld]: the residual stream (in place), or this rank's partial under TP
    const float* resid;  // the residual stream (tensor-parallel ranks > 0: null, their partial has none)
    const float* rscale;
    int nrows, ld;
    __device__ int row(int t, int i) const { return min(t * 16 + i, nrows - 1); }
    __device__ void store(int t, int i0, int m, const float* v, const PfState*) const {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = t * 16 + i0 + r;
            if (row >= nrows) continue;
            const size_t i = (size_t)m * ld + row;
            const float p = rscale ? v[r] * rscale[row] : v[r];
            y[i] = resid ? resid[i] + p : p;
        }
    }
};

template <int BM, typename WT>
constexpr size_t pgemm_lds_bytes() {
    return (size_t)kPgStages * PgGeo<BM, WT>::STAGE;
}

template <class Epi, int BM, typename WT>
hipError_t launch_pgemm(const PgIn<WT>& in, const Epi& epi, const PfState* ps, hipStream_t s) {
    const int nrb = (in.N + kPgBN - 1) / kPgBN;
    const int nrb8 = (nrb + 7) / 8 * 8;
    const dim3 grid(nrb8 * (in.M / BM));
    constexpr size_t lds = pgemm_lds_bytes<BM, WT>();
    hipLaunchKernelGGL((pgemm_kernel<Epi, BM, WT>), grid, dim3(kPgThreads), lds, s, in, epi, ps);
    return hipGetLastError();
}

template <class Epi, int BM, typename WT>
hipError_t pgemm_allow_lds() {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&pgemm_kernel<Epi, BM, WT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)pgemm_lds_bytes<BM, WT>());
}

// ---------------------------------------------------------------- 3. block-causal attention
// grid (M / 64, hq); 4 waves x 16 queries; lane l: query l & 15 of the wave, dims [c * HD/4, (c+1) * HD/4) with
// c = l >> 4. Scores: the 4 lanes of a query add their quarter dot products (xor 16 / 32 exchanges); every lane
// of a query keeps the same online-softmax state (m, l) and its quarter of o. Output attn / l as hi / lo.
constexpr int kPaQB = 64;  // queries per workgroup
constexpr int kPaKT = 64;  // keys per LDS tile

template <typename KT>
struct PfAttnArgs {
    const float* q;    // [M][hq*hd]
    const KT* kc;      // layer base [hkv][T][hd]
    const KT* vc;
    __half* ohi;       // [M][hq*hd]
    __half* olo;
    int hq, hkv, T;
    float scale;       // 1/sqrt(hd) (mha_kernel.cpp:41)
};

template <typename KT, int HD>
__global__ void __launch_bounds__(256) pf_attn_kernel(PfAttnArgs<KT> a, const PfState* __restrict__ ps) {
    constexpr int QD = HD / 4;  // dims per lane
    __shared__ __attribute__((aligned(16))) KT ks[kPaKT][HD];
    __shared__ __attribute__((aligned(16))) KT vs[kPaKT][HD];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = blockIdx.y, G = a.hq / a.hkv, kvh = h / G;
    const int p0 = ps->p0;
    const int mi = blockIdx.x * kPaQB + wave * 16 + (lane & 15);  // this lane's query (chunk row)
    const int c = lane >> 4;
    const int pos = p0 + mi;                                      // its position
    const int pos_max = p0 + blockIdx.x * kPaQB + kPaQB - 1;      // the block's last query position
    const int nt = min(pos_max, a.T - 1) / kPaKT + 1;             // key tiles
    float qv[QD], o[QD];
#pragma unroll
    for (int e = 0; e < QD; ++e) {
        qv[e] = a.q[(size_t)mi * a.hq * HD + (size_t)h * HD + c * QD + e];
        o[e] = 0.0f;
    }
    float mx = -INFINITY, l = 0.0f;
    const KT* kb = a.kc + (size_t)kvh * a.T * HD;
    const KT* vb = a.vc + (size_t)kvh * a.T * HD;
    constexpr int V16 = 16 / (int)sizeof(KT);  // elements per 16-byte vector
    for (int tt = 0; tt < nt; ++tt) {
        const int t0 = tt * kPaKT;
        __syncthreads();
        for (int i = threadIdx.x; i < kPaKT * HD / V16; i += 256) {  // the tile's K and V rows
            const int r = i / (HD / V16), cc = i - r * (HD / V16);
            const int t = min(t0 + r, a.T - 1);
            reinterpret_cast<u32x4*>(&ks[r][0])[cc] = reinterpret_cast<const u32x4*>(kb + (size_t)t * HD)[cc];
            reinterpret_cast<u32x4*>(&vs[r][0])[cc] = reinterpret_cast<const u32x4*>(vb + (size_t)t * HD)[cc];
        }
        __syncthreads();
        float s[kPaKT];
        float tmax = -INFINITY;
#pragma unroll
        for (int j = 0; j < kPaKT; ++j) {
            float d = 0.0f;
#pragma unroll
            for (int e = 0; e < QD; ++e) d = fmaf(qv[e], to_f32(ks[j][c * QD + e]), d);
            d = sum_xor16(d);
            d = sum_xor32(d);
            s[j] = (t0 + j <= pos) ? d * a.scale : -INFINITY;  // mha_kernel.cpp:51-60 (sum * scale), causal
            tmax = fmaxf(tmax, s[j]);
        }
        const float mn = fmaxf(mx, tmax);
        const float corr = mn == -INFINITY ? 1.0f : expf(mx - mn);
        l *= corr;
#pragma unroll
        for (int e = 0; e < QD; ++e) o[e] *= corr;
        mx = mn;
#pragma unroll
        for (int j = 0; j < kPaKT; ++j) {
            const float p = (t0 + j <= pos) ? expf(s[j] - mx) : 0.0f;
            l += p;
#pragma unroll
            for (int e = 0; e < QD; ++e) o[e] = fmaf(p, to_f32(vs[j][c * QD + e]), o[e]);
        }
    }
#pragma unroll
    for (int e = 0; e < QD; ++e) {
        const size_t idx = (size_t)mi * a.hq * HD + (size_t)h * HD + c * QD + e;
        pf_split(o[e] / l, a.ohi[idx], a.olo[idx]);
    }
}

}  // namespace sli
