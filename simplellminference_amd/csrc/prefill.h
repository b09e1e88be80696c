// prefill.h — prompt prefill as real GEMMs over the prompt (the reference teacher-forces the
// prompt one token per forward, source/model/model.cpp:157-165, so every weight is streamed once per prompt
// token). Here a chunk of up to kPfMaxChunk prompt positions runs through each layer together:
//
//   1. pf_norm_split_kernel: per position RMSNorm (rms_kernel.cpp:5-23, fp32) and the split of the fp32
//      result into fp16 hi + lo (hi = fp16(h), lo = fp16(h - hi): h to ~2^-22 relative);
//   2. pgemm_kernel: Y[pos][row] = sum_k W[row][k] * H[pos][k] on MFMA (v_mfma_f32_16x16x32_f16), A = a 16-row
//      weight tile, B = 16 positions' hi columns, then the same tile with the lo columns into the same fp32
//      accumulator (W * (hi + lo)); a workgroup owns 16 AT WR weight rows x BM positions (PgCfg), so a weight row
//      is read from HBM once per BM positions (the decode step reads it once per position). Operands are staged
//      through an S-deep LDS ring by LDS-DMA (global_load_lds_dwordx4: one 1-KiB fragment image per
//      wave-instruction, read back conflict-free by ds_read_b128), S - 1 stages in flight behind a counted
//      vmcnt and a raw s_barrier (cdna_hip_programming.md §5 "Pipelining across barriers"), or the weight images
//      in a deeper ring of their own (PgCfg::SA, round 6); the fragment reads of
//      the next k-block are issued ahead of the current k-block's MFMAs (two register sets, across the stage
//      barrier too: PgCfg::PIPE, round 6, 5-20 % faster per GEMM, bit-identical sums). Fused epilogues:
//      RoPE + K/V cache rows + q (model.cpp:52-67), residual add (:86-90, :124-128), SwiGLU (:111-115,
//      written straight as the down projection's hi/lo operand);
//   3. pf_attn_mfma_kernel (fp16 KV, the default): block-causal attention of 16 chunk rows x one head against
//      the cache rows 0 .. position (mha_kernel.cpp:36-77 per query: s_t = q.k_t * scale, softmax, sum p_t v_t):
//      S = K q^T on MFMA with q split hi/lo, online softmax in fp32, P V on MFMA with V read transposed
//      (ds_read_b64_tr_b16) from LDS-DMA'd K/V tiles; pf_attn_kernel, the VALU form (fp32, 64-position query
//      blocks, K/V tiles of 64 positions in LDS), serves fp32 KV caches.
// int8 weights: stages of 128 k; a depth that is 64 mod 128 (e.g. Llama-2-7B int8 down at TP 4, 2752) ends with
// a half stage (pgemm_kernel).
// The chunk's start position and valid count live in device memory (PfState), so one captured graph per
// chunk size serves every chunk of every prompt.
#pragma once
#include "common.h"

namespace sli {

constexpr int kPfMaxChunk = 256;   // prompt positions per weight pass

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

// one workgroup per chunk row: h = (x * 1/rms) * w (rms_kernel.cpp:12-22) or plain x (w == nullptr), as hi/lo.
// The row is held in registers (a float4 per thread and pass; D % 4 == 0, D <= 8192): one read of x, 8-byte
// hi / lo stores.
__global__ void __launch_bounds__(256) pf_norm_split_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           __half* __restrict__ hi, __half* __restrict__ lo, int D,
                                                           float eps) {
    constexpr int MAXV = 8;  // float4 per thread: D <= 8192
    const int m = blockIdx.x;
    const float* xr = x + (size_t)m * D;
    const int n4 = D / 4;
    float4 v[MAXV], wv[MAXV];
    float ss = 0.0f;
    // the norm weights are loaded with x (round 6: not after the reduction, one memory round trip fewer)
    const float4* w4 = reinterpret_cast<const float4*>(w ? w : xr);
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
        if (j * 256 + (int)threadIdx.x < n4) {
            v[j] = reinterpret_cast<const float4*>(xr)[j * 256 + threadIdx.x];
            wv[j] = w4[j * 256 + threadIdx.x];
            ss += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
        }
    float inv = 1.0f;
    if (w) {
        ss = wave_sum(ss);
        __shared__ float red[4];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
        __syncthreads();
        const float t = red[0] + red[1] + red[2] + red[3];
        const float tep = t / (float)D;      // rms_kernel.cpp:17
        const float rms = sqrtf(tep + eps);  // :18
        inv = 1.0f / rms;                    // :19
    }
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
        if (j * 256 + (int)threadIdx.x < n4) {
            const int i = (j * 256 + threadIdx.x) * 4;
            const float f[4] = {v[j].x, v[j].y, v[j].z, v[j].w}, g[4] = {wv[j].x, wv[j].y, wv[j].z, wv[j].w};
            __half hh[4], hl[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) pf_split(w ? (f[e] * inv) * g[e] : f[e], hh[e], hl[e]);  // :20-22
            *reinterpret_cast<uint2*>(hi + (size_t)m * D + i) = *reinterpret_cast<const uint2*>(hh);
            *reinterpret_cast<uint2*>(lo + (size_t)m * D + i) = *reinterpret_cast<const uint2*>(hl);
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

// Tiling: a workgroup of 2 WR waves owns BN = 32 WR weight rows x BM chunk rows; wave w holds the 2 x BM/32
// accumulator tiles of rows 32 (w % WR) .. +32 and position half w / WR. A stage covers KS depth: 64 for fp16
// weights, 128 for int8, so a weight row's slice is one whole 128-byte line (a chunk row's fp16 hi / lo slice
// one or two lines). Each LDS-DMA wave-instruction moves 1 KiB of whole lines (8 rows x 128 B or 4 x 256 B;
// fragment-shaped pieces of 16 rows x 64 B fetched every line twice and capped the ingest at ~29 GB/s per
// CU, tools/pgemm_lab); the 16-byte chunks of a row are XOR-swizzled by the row so the fragment reads
// (16 rows x 16 B per lane group) stay conflict-free. S stages in the LDS ring, S - 1 of them in flight.
// Epilogue contract: row(t, i) = weight row of 16-row tile t's row i (i < 16, always valid); store(t, i0, m, v)
// gets the fp32 sums of tile rows i0 .. i0+3 (i0 % 4 == 0) for chunk row m.
// AT_: 16-row weight tiles per wave (2: a wave's 32 rows; 4: 64 rows, so every B fragment read from LDS feeds twice
// the MFMAs). PIPE_: the fragment reads of k-block j + 1 issued before the MFMAs of k-block j (two register sets),
// across the stage barrier too, and every hi MFMA of a k-block ahead of its lo MFMAs (no back-to-back MFMAs on one
// accumulator); each tile's sums are added in the same order either way (bit-identical).
// SA_ > 0 (PIPE only): the weight (A) images get a ring of their own, SA_ stages deep (SA_ - 1 issued ahead), and
// the activation (B) images a 2-stage ring (one ahead): the A bytes come from HBM (read once per chunk), the B bytes
// from L2, so only A needs the deep prefetch, and B, the larger image, does not pay for it in LDS.
template <int BM_, int WR_, int S_, int AT_ = 2, bool PIPE_ = false, int SA_ = 0>
struct PgCfg {
    static constexpr int BM = BM_, WR = WR_, S = S_, AT = AT_, SA = SA_;
    static constexpr bool PIPE = PIPE_;
};

template <class Cfg, typename WT>
struct PgGeo {
    static constexpr int BM = Cfg::BM, WR = Cfg::WR, S = Cfg::S, AT = Cfg::AT;
    static constexpr int WAVES = 2 * WR, THREADS = 64 * WAVES, BN = 16 * AT * WR;
    static constexpr int KS = sizeof(WT) == 1 ? 128 : 64;  // depth per stage
    static constexpr int KBS = KS / 32;                    // MFMA k-blocks per stage
    static constexpr int A_ROW = KS * (int)sizeof(WT);     // 128 B
    static constexpr int B_ROW = KS * 2;                   // 128 or 256 B
    static constexpr int A_IMG = 16 * A_ROW, B_IMG = 16 * B_ROW;
    static constexpr int PT = BM / 16;  // position tiles per workgroup
    static constexpr int WPT = PT / 2;  // per wave
    static constexpr int NA = AT * WR;  // weight row tiles
    static constexpr int A_BYTES = NA * A_IMG;
    static constexpr int STAGE = A_BYTES + 2 * PT * B_IMG;
    static constexpr int NDMA = STAGE / 1024;  // wave-instructions per stage
    static constexpr int DPW = NDMA / WAVES;   // per wave
    static constexpr int SA = Cfg::SA;         // split rings (PgCfg): A pieces per wave DPA, B pieces DPB
    static constexpr int B_BYTES = STAGE - A_BYTES;
    static constexpr int DPA = SA ? A_BYTES / 1024 / WAVES : 0, DPB = SA ? B_BYTES / 1024 / WAVES : 0;
    static constexpr size_t LDS = SA ? (size_t)SA * A_BYTES + (size_t)S * B_BYTES : (size_t)S * STAGE;
    static_assert(A_ROW == 128 && WPT >= 1 && NDMA % WAVES == 0, "tiling");
    static_assert(S >= 2 && (S - 1) * DPW <= 63, "ring depth (vmcnt counts 63 loads)");
    // (SA > S: A(s) must be issued in an earlier iteration than B(s), the wait below counts on it; SA == S computed
    // wrong sums in tools/pgemm_lab)
    static_assert(SA == 0 || (Cfg::PIPE && S == 2 && SA > S && (A_BYTES / 1024) % WAVES == 0 &&
                              (B_BYTES / 1024) % WAVES == 0 && (SA - 1) * DPA + DPB <= 63), "split rings");
    static_assert(LDS <= 160 * 1024, "LDS");
};

// 16-byte chunk swizzle of an image row (conflict-free fragment reads): rows of 128 B pair up in one 256-B
// bank span, so the chunk index is XORed with row / 2; rows of 256 B with the row
__device__ __forceinline__ int pg_swz(int row, int row_bytes) { return row_bytes == 128 ? (row >> 1) & 7 : row & 15; }

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

// wait until at most `later` stages of DPW images each are still in flight (later: 0 .. 6)
template <int DPW>
__device__ __forceinline__ void pg_wait_stages(int later) {
    switch (later) {
        case 0: pf_wait_vm<0>(); break;
        case 1: pf_wait_vm<1 * DPW>(); break;
        case 2: pf_wait_vm<(2 * DPW > 63 ? 63 : 2 * DPW)>(); break;
        case 3: pf_wait_vm<(3 * DPW > 63 ? 63 : 3 * DPW)>(); break;
        case 4: pf_wait_vm<(4 * DPW > 63 ? 63 : 4 * DPW)>(); break;
        case 5: pf_wait_vm<(5 * DPW > 63 ? 63 : 5 * DPW)>(); break;
        default: pf_wait_vm<(6 * DPW > 63 ? 63 : 6 * DPW)>(); break;
    }
}

template <class Epi, class Cfg, typename WT>
__global__ void __launch_bounds__(128 * Cfg::WR) pgemm_kernel(PgIn<WT> in, Epi epi, const PfState* __restrict__ ps) {
    using Geo = PgGeo<Cfg, WT>;
    constexpr int KBS = Geo::KBS, BM = Geo::BM, WR = Geo::WR, S = Geo::S;
    extern __shared__ __attribute__((aligned(1024))) char pg_smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int wr = wave % WR, wp = wave / WR;  // row pair, position half
    const int PB = in.M / BM;
    // workgroups that share a row block run on one XCD (blocks b and b + 8 share one under round-robin
    // placement; speed only): the second read of the weight rows hits that XCD's L2
    const int bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
    const int rb = (slot / PB) * 8 + xcd, pb = slot - (slot / PB) * PB;
    const int nrb = (in.N + Geo::BN - 1) / Geo::BN;
    if (rb >= nrb) return;  // (uniform) padding of the grid to a multiple of 8 row blocks
    // stages: K is a multiple of 64, so with int8 weights (KS 128) the last stage may be a half stage. Its DMA
    // pieces past the row's end reload the stage's first half instead (in bounds; never read), and only its
    // first KBS / 2 k-blocks are multiplied.
    const int ns = (in.K + Geo::KS - 1) / Geo::KS;
    const bool half_tail = (in.K % Geo::KS) != 0;
    const int nt = in.N >> 4;       // row tiles
    const unsigned ring = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)pg_smem;

    // this wave's DMA instructions d in [wave*DPW, (wave+1)*DPW): stage bytes [1024 d, 1024 (d + 1)). Lane i
    // lands at byte 16 i of it: image row i / cpr, physical chunk i % cpr (cpr = 16-B chunks per image row),
    // so it loads the row's logical chunk (i % cpr) ^ swizzle(row).
    const char* src[Geo::DPW];
    int adv[Geo::DPW];   // bytes per stage
    int back[Geo::DPW];  // bytes to step back in a half last stage (logical chunk in the stage's second half)
#pragma unroll
    for (int j = 0; j < Geo::DPW; ++j) {
        // split rings: the wave's DPA pieces of the A images, then its DPB pieces of the B images
        const int off = Geo::SA ? (j < Geo::DPA ? (wave * Geo::DPA + j) * 1024
                                                : Geo::A_BYTES + (wave * Geo::DPB + j - Geo::DPA) * 1024)
                                : (wave * Geo::DPW + j) * 1024;
        if (off < Geo::A_BYTES) {
            const int t = rb * Geo::NA + off / Geo::A_IMG;
            const int r = (off % Geo::A_IMG) / Geo::A_ROW + lane / 8;
            const int c = (lane % 8) ^ pg_swz(r, Geo::A_ROW);
            const int row = epi.row(min(t, nt - 1), r);
            src[j] = reinterpret_cast<const char*>(in.W) + (size_t)row * in.K * sizeof(WT) + c * 16;
            adv[j] = Geo::A_ROW;
            back[j] = c >= 4 ? Geo::A_ROW / 2 : 0;
        } else {
            constexpr int cpr = Geo::B_ROW / 16;
            const int o2 = off - Geo::A_BYTES;
            const int u = o2 / Geo::B_IMG, pt = u >> 1;
            const int r = (o2 % Geo::B_IMG) / Geo::B_ROW + lane / cpr;
            const int c = (lane % cpr) ^ pg_swz(r, Geo::B_ROW);
            const __half* B = (u & 1) ? in.Blo : in.Bhi;
            const int m = pb * BM + pt * 16 + r;
            src[j] = reinterpret_cast<const char*>(B) + (size_t)m * in.K * 2 + c * 16;
            adv[j] = Geo::B_ROW;
            back[j] = c >= cpr / 2 ? Geo::B_ROW / 2 : 0;
        }
    }
    auto issue = [&](int s) {
        const unsigned dst = ring + (unsigned)((s % S) * Geo::STAGE);
        const bool tail = half_tail && s == ns - 1;
#pragma unroll
        for (int j = 0; j < Geo::DPW; ++j) {
#ifdef PG_LAB_SKIP  // tools/pgemm_lab only (bit 0: no A pieces, bit 1: no B pieces): timing bounds, wrong sums
            const bool isa = (wave * Geo::DPW + j) * 1024 < Geo::A_BYTES;
            if (((PG_LAB_SKIP & 1) && isa) || ((PG_LAB_SKIP & 2) && !isa)) continue;
#endif
            pf_dma(src[j] + (size_t)s * adv[j] - (tail ? back[j] : 0), dst + (unsigned)((wave * Geo::DPW + j) * 1024));
        }
    };

    // split rings: A stage s in slot s % SA at ring, B stage s in slot s % 2 behind the A ring
    const unsigned ring_b = ring + (unsigned)(Geo::SA * Geo::A_BYTES);
    auto issue_a = [&](int s) {
        const unsigned dst = ring + (unsigned)((s % Geo::SA) * Geo::A_BYTES);
        const bool tail = half_tail && s == ns - 1;
#pragma unroll
        for (int j = 0; j < Geo::DPA; ++j)
            pf_dma(src[j] + (size_t)s * adv[j] - (tail ? back[j] : 0), dst + (unsigned)((wave * Geo::DPA + j) * 1024));
    };
    auto issue_b = [&](int s) {
        const unsigned dst = ring_b + (unsigned)((s & 1) * Geo::B_BYTES);
        const bool tail = half_tail && s == ns - 1;
#pragma unroll
        for (int j = 0; j < Geo::DPB; ++j)
            pf_dma(src[Geo::DPA + j] + (size_t)s * adv[Geo::DPA + j] - (tail ? back[Geo::DPA + j] : 0),
                   dst + (unsigned)((wave * Geo::DPB + j) * 1024));
    };
    constexpr int AT = Geo::AT;
    pf_float4 acc[AT][Geo::WPT];
#pragma unroll
    for (int a = 0; a < AT; ++a)
#pragma unroll
        for (int b = 0; b < Geo::WPT; ++b) acc[a][b] = pf_float4{0.0f, 0.0f, 0.0f, 0.0f};

    // fragment read offsets: lane l reads row / column r = l & 15, k group kg = l >> 4 of each 32-k block
    const int kg = lane >> 4, r16 = lane & 15;
    const int sa = pg_swz(r16, Geo::A_ROW), sb = pg_swz(r16, Geo::B_ROW);
    if constexpr (Geo::SA == 0) {
        for (int s = 0; s < S - 1 && s < ns; ++s) issue(s);
    } else {  // the schedule of iterations -(SA - 1) .. -1: B(i + 1), then A(i + SA - 1)
        for (int i = 1 - Geo::SA; i < 0; ++i) {
            if (i + 1 >= 0 && i + 1 < ns) issue_b(i + 1);
            if (i + Geo::SA - 1 >= 0 && i + Geo::SA - 1 < ns) issue_a(i + Geo::SA - 1);
        }
    }
    // fragments of k-block kb of stage buffer st (A images at st, B images at stb) into (af, bh, bl)
    auto read_frags = [&](const char* st, const char* stb, int kb, u32x4(&af)[AT], u32x4(&bh)[Geo::WPT],
                          u32x4(&bl)[Geo::WPT]) {
#pragma unroll
        for (int a = 0; a < AT; ++a) {
            const char* img = st + (wr * AT + a) * Geo::A_IMG + r16 * Geo::A_ROW;
            if constexpr (sizeof(WT) == 2) {
                af[a] = *reinterpret_cast<const u32x4*>(img + ((4 * kb + kg) ^ sa) * 16);
            } else {
                const int off = ((2 * kb + (kg >> 1)) ^ sa) * 16 + 8 * (kg & 1);
                af[a] = pg_i8_to_f16(*reinterpret_cast<const uint2*>(img + off));
            }
        }
#pragma unroll
        for (int b = 0; b < Geo::WPT; ++b) {
            const int pt = wp * Geo::WPT + b;
            const char* img = stb + (2 * pt) * Geo::B_IMG + r16 * Geo::B_ROW + ((4 * kb + kg) ^ sb) * 16;
            bh[b] = *reinterpret_cast<const u32x4*>(img);
            bl[b] = *reinterpret_cast<const u32x4*>(img + Geo::B_IMG);
        }
    };
    auto mfmas = [&](const u32x4(&af)[AT], const u32x4(&bh)[Geo::WPT], const u32x4(&bl)[Geo::WPT]) {
#pragma unroll
        for (int b = 0; b < Geo::WPT; ++b)
#pragma unroll
            for (int a = 0; a < AT; ++a) acc[a][b] = pf_mfma(af[a], bh[b], acc[a][b]);
#pragma unroll
        for (int b = 0; b < Geo::WPT; ++b)
#pragma unroll
            for (int a = 0; a < AT; ++a) acc[a][b] = pf_mfma(af[a], bl[b], acc[a][b]);
    };
    if constexpr (Cfg::PIPE) {
        // set X holds even k-blocks, set Y odd ones (KBS is even; an int8 half stage has KBS / 2 = 2): per stage
        // read(0) -> X, MFMA(Y: the previous stage's last k-block), read(1) -> Y, MFMA(X), ... The stage barrier
        // follows this wave's lgkmcnt(0), so the previous stage's buffer is free for the DMA issued after it while
        // its last fragments wait in registers.
        static_assert(KBS % 2 == 0, "k-blocks per stage");
        u32x4 xa[AT], xh[Geo::WPT], xl[Geo::WPT], ya[AT], yh[Geo::WPT], yl[Geo::WPT];
        for (int s = 0; s < ns; ++s) {
            const char *st, *stb;
            if constexpr (Geo::SA == 0) {
                pg_wait_stages<Geo::DPW>(min(S - 2, ns - 1 - s));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (s + S - 1 < ns) issue(s + S - 1);
                st = pg_smem + (size_t)(s % S) * Geo::STAGE;
                stb = st + Geo::A_BYTES;
            } else {
                // B(s) was the first load of iteration s - 1; only that iteration's A pieces (if it issued any) were
                // issued after it, and A(s) before it
                if (s + Geo::SA - 2 < ns)
                    pf_wait_vm<Geo::DPA>();
                else
                    pf_wait_vm<0>();
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (s + 1 < ns) issue_b(s + 1);
                if (s + Geo::SA - 1 < ns) issue_a(s + Geo::SA - 1);
                st = pg_smem + (size_t)(s % Geo::SA) * Geo::A_BYTES;
                stb = pg_smem + (size_t)Geo::SA * Geo::A_BYTES + (size_t)(s & 1) * Geo::B_BYTES;
            }
            const int kbs = (half_tail && s == ns - 1) ? KBS / 2 : KBS;  // wave-uniform, even
#pragma unroll
            for (int kb = 0; kb < KBS; kb += 2) {
                if (kb >= kbs) break;
                read_frags(st, stb, kb, xa, xh, xl);
                if (s > 0 || kb > 0) mfmas(ya, yh, yl);
                read_frags(st, stb, kb + 1, ya, yh, yl);
                mfmas(xa, xh, xl);
            }
        }
        mfmas(ya, yh, yl);
    } else {
    for (int s = 0; s < ns; ++s) {
        // this wave's pieces of stage s landed (stages s + 1 .. s + S - 2 may stay in flight)
        pg_wait_stages<Geo::DPW>(min(S - 2, ns - 1 - s));
        __builtin_amdgcn_s_barrier();  // every wave's pieces of s landed; every wave is done with s - 1
        if (s + S - 1 < ns) issue(s + S - 1);  // into the buffer of s - 1
        const char* st = pg_smem + (size_t)(s % S) * Geo::STAGE;
        const int kbs = (half_tail && s == ns - 1) ? KBS / 2 : KBS;  // wave-uniform
#pragma unroll
        for (int kb = 0; kb < KBS; ++kb) {
            if (kb >= kbs) break;
            u32x4 af[AT], bh[Geo::WPT], bl[Geo::WPT];
#pragma unroll
            for (int a = 0; a < AT; ++a) {
                const char* img = st + (wr * AT + a) * Geo::A_IMG + r16 * Geo::A_ROW;
                if constexpr (sizeof(WT) == 2) {
                    af[a] = *reinterpret_cast<const u32x4*>(img + ((4 * kb + kg) ^ sa) * 16);
                } else {  // k 32 kb + 8 kg .. +8: chunk 2 kb + kg / 2, half kg % 2
                    const int off = ((2 * kb + (kg >> 1)) ^ sa) * 16 + 8 * (kg & 1);
                    af[a] = pg_i8_to_f16(*reinterpret_cast<const uint2*>(img + off));
                }
            }
#pragma unroll
            for (int b = 0; b < Geo::WPT; ++b) {
                const int pt = wp * Geo::WPT + b;
                const char* img = st + Geo::A_BYTES + (2 * pt) * Geo::B_IMG + r16 * Geo::B_ROW + ((4 * kb + kg) ^ sb) * 16;
                bh[b] = *reinterpret_cast<const u32x4*>(img);
                bl[b] = *reinterpret_cast<const u32x4*>(img + Geo::B_IMG);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int a = 0; a < AT; ++a)
#pragma unroll
                for (int b = 0; b < Geo::WPT; ++b) {
#if defined(PG_LAB_MFMA) && PG_LAB_MFMA == 0  // tools/pgemm_lab only: no MFMA (data movement alone)
                    acc[a][b][0] += __uint_as_float(af[a][0] ^ bh[b][0] ^ bl[b][0]);
#else
                    acc[a][b] = pf_mfma(af[a], bh[b], acc[a][b]);
#if !(defined(PG_LAB_MFMA) && PG_LAB_MFMA == 1)  // PG_LAB_MFMA 1: the hi MFMA only
                    acc[a][b] = pf_mfma(af[a], bl[b], acc[a][b]);
#endif
#endif
                }
        }
    }
    }
    // C[i][n] of a 16x16 tile: lane l holds rows 4 (l >> 4) + r, column l & 15
    const int i0 = 4 * (lane >> 4);
#pragma unroll
    for (int a = 0; a < AT; ++a) {
        const int t = rb * Geo::NA + wr * AT + a;
        if (t >= nt) continue;
#pragma unroll
        for (int b = 0; b < Geo::WPT; ++b) {
            const int m = pb * BM + (wp * Geo::WPT + b) * 16 + r16;
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
        // units u, u + 1 (u even): d, d + 1 of one head (hd / 2 is even), so every store is a pair
        const int nv = ps->nv, pos = ps->p0 + m;
        const int half = hd >> 1;
        const int u = t * 8 + (i0 >> 2) * 2;
        const int uh = u / half, d = u - uh * half;
        float a0[2] = {v[0], v[1]}, a1[2] = {v[2], v[3]};  // first / second element of the pairs of u, u + 1
        if (rscale) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                a0[e] *= rscale[uh * hd + d + e];
                a1[e] *= rscale[uh * hd + d + e + half];
            }
        }
        if (uh < hq + hkv) {  // rope_kernel.cpp:30-38
            const int pp = min(pos, T - 1);
            float r0[2], r1[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const float fci = sin_t[pp * half + d + e], fcr = cos_t[pp * half + d + e];
                r0[e] = a0[e] * fcr - a1[e] * fci;
                r1[e] = a1[e] * fcr + a0[e] * fci;
            }
            if (uh < hq) {
                float* qr = q + (size_t)m * hq * hd + (size_t)uh * hd;
                *reinterpret_cast<float2*>(qr + d) = make_float2(r0[0], r0[1]);
                *reinterpret_cast<float2*>(qr + d + half) = make_float2(r1[0], r1[1]);
            } else if (m < nv && pos < T) {
                KT* kr = kc + ((size_t)(uh - hq) * T + pos) * hd;
                store2(kr + d, r0);
                store2(kr + d + half, r1);
            }
        } else if (m < nv && pos < T) {
            KT* vr = vc + ((size_t)(uh - hq - hkv) * T + pos) * hd;
            store2(vr + d, a0);
            store2(vr + d + half, a1);
        }
    }
    __device__ static void store2(KT* p, const float* f) {
        if constexpr (sizeof(KT) == 2) {
            __half h[2] = {__float2half_rn(f[0]), __float2half_rn(f[1])};
            *reinterpret_cast<unsigned*>(p) = *reinterpret_cast<const unsigned*>(h);
        } else {
            *reinterpret_cast<float2*>(p) = make_float2(f[0], f[1]);
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
        const int u = t * 8 + (i0 >> 2) * 2;  // units u, u + 1: one 4-byte hi and lo store each
        __half hh[2], hl[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            float g = v[e], up = v[2 + e];
            if (rscale) {
                g *= rscale[u + e];
                up *= rscale[inter + u + e];
            }
            float sg = 1.0f / (1.0f + expf(-g));  // swiglu_kernel.cpp:12
            if (silu) sg = g * sg;
            pf_split(sg * up, hh[e], hl[e]);  // :13
        }
        *reinterpret_cast<unsigned*>(ahi + (size_t)m * inter + u) = *reinterpret_cast<const unsigned*>(hh);
        *reinterpret_cast<unsigned*>(alo + (size_t)m * inter + u) = *reinterpret_cast<const unsigned*>(hl);
    }
};

struct PgEpiResid {  // y[m][row] = resid[m][row] + sum * row scale (matmul_kernel.cpp:26 + add_kernel.cpp:5-14)
    float* y;        // [M][ld]: the residual stream (in place), or this rank's partial under TP
    const float* resid;  // the residual stream (tensor-parallel ranks > 0: null, their partial has none)
    const float* rscale;
    int nrows, ld;
    __device__ int row(int t, int i) const { return min(t * 16 + i, nrows - 1); }
    __device__ void store(int t, int i0, int m, const float* v, const PfState*) const {
        const int row = t * 16 + i0;  // rows row .. row + 3 (nrows % 16 == 0: the host's check)
        const size_t i = (size_t)m * ld + row;
        float4 p = make_float4(v[0], v[1], v[2], v[3]);
        if (rscale) {
            const float4 sc = *reinterpret_cast<const float4*>(rscale + row);
            p = make_float4(p.x * sc.x, p.y * sc.y, p.z * sc.z, p.w * sc.w);
        }
        if (resid) {
            const float4 r = *reinterpret_cast<const float4*>(resid + i);
            p = make_float4(r.x + p.x, r.y + p.y, r.z + p.z, r.w + p.w);
        }
        *reinterpret_cast<float4*>(y + i) = p;
    }
};

template <class Epi, class Cfg, typename WT>
hipError_t launch_pgemm(const PgIn<WT>& in, const Epi& epi, const PfState* ps, hipStream_t s) {
    using Geo = PgGeo<Cfg, WT>;
    const int nrb = (in.N + Geo::BN - 1) / Geo::BN;
    const int nrb8 = (nrb + 7) / 8 * 8;
    const dim3 grid(nrb8 * (in.M / Geo::BM));
    hipLaunchKernelGGL((pgemm_kernel<Epi, Cfg, WT>), grid, dim3(Geo::THREADS), Geo::LDS, s, in, epi, ps);
    return hipGetLastError();
}

template <class Epi, class Cfg, typename WT>
hipError_t pgemm_allow_lds() {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&pgemm_kernel<Epi, Cfg, WT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)PgGeo<Cfg, WT>::LDS);
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

// ---- 3b. block-causal attention on MFMA (fp16 cache). A workgroup = 16 chunk rows (queries) of one head;
// its 4 waves split the key range into 32-key tiles (wave w takes tiles w, w + 4, ...) and merge their
// (max, sum, o) through LDS at the end. Per tile a wave:
//   - LDS-DMAs K and V rows t0 .. t0+31 (16 x 1 KiB pieces) into its own images, 16-B chunks XOR-swizzled;
//   - Sᵀ = K Qᵀ: C[key][query] on v_mfma_f32_16x16x32_f16, A = K rows (exact fp16), B = Qᵀ as hi + lo fp16
//     (two MFMAs into one accumulator);
//   - online softmax per query (a lane's 8 keys, then the 4 lane groups of a query by xor 16 / 32);
//   - Oᵀ += Vᵀ Pᵀ: B = Pᵀ straight from the Sᵀ accumulators (lane l holds query l & 15, keys
//     {4g .. 4g+3, 16+4g .. 16+4g+3}, g = l >> 4 — the k order of the B operand), P as hi + lo; A = Vᵀ by
//     two ds_read_b64_tr_b16 per 16-d tile, whose 4-row blocks are exactly those keys.
// mha_kernel.cpp:36-77 per query: s_t = (q . k_t) * scale, softmax over t <= position, o = sum p_t v_t.
template <int HD>
struct PaGeo {
    static constexpr int ROWB = HD * 2;          // bytes per image row
    static constexpr int IMG = 32 * ROWB;        // one 32-key image
    static constexpr int WAVE = 2 * IMG;         // K + V
    static constexpr int PIECES = WAVE / 1024;   // DMA instructions per tile
    static constexpr int CPR = ROWB / 16;        // 16-B chunks per row
};
__device__ __forceinline__ int pa_swz_k(int r, int rowb) { return rowb == 256 ? r & 15 : (r >> 1) & 7; }
__device__ __forceinline__ int pa_swz_v(int r, int rowb) { return rowb == 256 ? (r & 7) << 1 : ((r >> 1) & 3) << 1; }

__device__ __forceinline__ uint2 pa_tr_read(unsigned lds_addr) {
    uint2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr) : "memory");
    return v;
}

template <int HD>
__global__ void __launch_bounds__(256) pf_attn_mfma_kernel(PfAttnArgs<__half> a, const PfState* __restrict__ ps) {
    using G = PaGeo<HD>;
    constexpr int ND = HD / 32, NT = HD / 16;  // 32-d blocks (S), 16-d tiles (O)
    __shared__ __attribute__((aligned(1024))) char sm[4 * G::WAVE];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int g = lane >> 4, i16 = lane & 15;
    const int h = blockIdx.y, kvh = h / (a.hq / a.hkv);
    const int p0 = ps->p0;
    const int mq = blockIdx.x * 16 + i16;  // this lane's query (chunk row)
    const int pos = p0 + mq;
    const int last = min(p0 + blockIdx.x * 16 + 15, a.T - 1);  // the group's last query position
    const int ntiles = last / 32 + 1;
    const size_t qs = (size_t)a.hq * HD;
    // Qᵀ as the B operand: lane l = query l & 15, d = 32 db + 8 g .. +8, fp32 -> hi + lo
    u32x4 qh[ND], ql[ND];
#pragma unroll
    for (int db = 0; db < ND; ++db) {
        const float4* qp = reinterpret_cast<const float4*>(a.q + (size_t)mq * qs + (size_t)h * HD + db * 32 + g * 8);
        const float4 v0 = qp[0], v1 = qp[1];
        const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        __half hh[8], hl[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) pf_split(f[e], hh[e], hl[e]);
        qh[db] = *reinterpret_cast<const u32x4*>(hh);
        ql[db] = *reinterpret_cast<const u32x4*>(hl);
    }
    pf_float4 o[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) o[t] = pf_float4{0.0f, 0.0f, 0.0f, 0.0f};
    float mx = -INFINITY, l = 0.0f;
    char* kimg = sm + wave * G::WAVE;
    const unsigned kbase = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)kimg;
    const unsigned vbase = kbase + G::IMG;
    const __half* kc = a.kc + (size_t)kvh * a.T * HD;
    const __half* vc = a.vc + (size_t)kvh * a.T * HD;
    for (int tt = wave; tt < ntiles; tt += 4) {
        const int t0 = tt * 32;
        // K pieces 0 .. P/2-1, V pieces P/2 .. P-1; lane i of a piece: row (piece rows) + i / CPR, physical
        // chunk i % CPR <- logical chunk (i % CPR) ^ swizzle(row)
#pragma unroll
        for (int j = 0; j < G::PIECES; ++j) {
            const bool isv = j >= G::PIECES / 2;
            const int jj = isv ? j - G::PIECES / 2 : j;
            const int r = jj * (1024 / G::ROWB) + lane / G::CPR;
            const int c = (lane % G::CPR) ^ (isv ? pa_swz_v(r, G::ROWB) : pa_swz_k(r, G::ROWB));
            const __half* src = (isv ? vc : kc) + (size_t)min(t0 + r, a.T - 1) * HD + c * 8;
            pf_dma(src, (isv ? vbase : kbase) + (unsigned)(jj * 1024));
        }
        pf_wait_vm<0>();
        // Sᵀ[key][query] for keys t0 + 16 kt + (0..15)
        pf_float4 sacc[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
            sacc[kt] = pf_float4{0.0f, 0.0f, 0.0f, 0.0f};
            const int r = kt * 16 + i16;
            const char* krow = kimg + r * G::ROWB;
#pragma unroll
            for (int db = 0; db < ND; ++db) {
                const u32x4 kf = *reinterpret_cast<const u32x4*>(krow + ((4 * db + g) ^ pa_swz_k(r, G::ROWB)) * 16);
                sacc[kt] = pf_mfma(kf, qh[db], sacc[kt]);
                sacc[kt] = pf_mfma(kf, ql[db], sacc[kt]);
            }
        }
        // lane holds keys t0 + 16 kt + 4 g + r of query mq
        float sv[8];
        float cmax = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = t0 + kt * 16 + 4 * g + r;
                const float v = key <= pos ? sacc[kt][r] * a.scale : -INFINITY;
                sv[kt * 4 + r] = v;
                cmax = fmaxf(cmax, v);
            }
        cmax = fmaxf(cmax, __shfl_xor(cmax, 16));
        cmax = fmaxf(cmax, __shfl_xor(cmax, 32));
        const float mn = fmaxf(mx, cmax);
        const float corr = mn == -INFINITY ? 1.0f : expf(mx - mn);
        float pv[8], psum = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            pv[e] = sv[e] == -INFINITY ? 0.0f : expf(sv[e] - mn);
            psum += pv[e];
        }
        psum += __shfl_xor(psum, 16);
        psum += __shfl_xor(psum, 32);
        l = l * corr + psum;
        mx = mn;
        __half ph[8], pl[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) pf_split(pv[e], ph[e], pl[e]);
        const u32x4 pfh = *reinterpret_cast<const u32x4*>(ph);
        const u32x4 pfl = *reinterpret_cast<const u32x4*>(pl);
        // Vᵀ 16-d tile dt: lane 16 g + 4 q + p addresses row (4 g + q) [+16], d 16 dt + 4 p .. +3
        const int q4 = (lane & 15) >> 2, p4 = lane & 3;
        const int r1 = 4 * g + q4, r2 = 16 + 4 * g + q4;
        const unsigned a1 = vbase + r1 * G::ROWB + 8 * (p4 & 1), a2 = vbase + r2 * G::ROWB + 8 * (p4 & 1);
        const int s1 = pa_swz_v(r1, G::ROWB), s2 = pa_swz_v(r2, G::ROWB);
        uint2 x1[NT], x2[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int c = 2 * t + (p4 >> 1);
            x1[t] = pa_tr_read(a1 + ((c ^ s1) * 16));
            x2[t] = pa_tr_read(a2 + ((c ^ s2) * 16));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            o[t] *= corr;
            const u32x4 vf = u32x4{x1[t].x, x1[t].y, x2[t].x, x2[t].y};
            o[t] = pf_mfma(vf, pfh, o[t]);
            o[t] = pf_mfma(vf, pfl, o[t]);
        }
    }
    // merge the 4 key splits: wave w publishes (mx, l, o) and merges 16-d tiles t = w, w + 4, ...
    __syncthreads();
    float* fo = reinterpret_cast<float*>(sm);                         // [wave][NT][64 lanes][4]
    float* fm = fo + 4 * NT * 64 * 4;                                 // [wave][64]
    float* fl = fm + 4 * 64;
#pragma unroll
    for (int t = 0; t < NT; ++t)
        *reinterpret_cast<pf_float4*>(fo + ((wave * NT + t) * 64 + lane) * 4) = o[t];
    fm[wave * 64 + lane] = mx;
    fl[wave * 64 + lane] = l;
    __syncthreads();
    float m4[4], w4[4], M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        m4[w] = fm[w * 64 + lane];
        M = fmaxf(M, m4[w]);
    }
    float L = 0.0f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        w4[w] = m4[w] == -INFINITY ? 0.0f : expf(m4[w] - M);
        L += fl[w * 64 + lane] * w4[w];
    }
    const float inv = 1.0f / L;
    for (int t = wave; t < NT; t += 4) {
        pf_float4 acc = pf_float4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int w = 0; w < 4; ++w) acc += *reinterpret_cast<const pf_float4*>(fo + ((w * NT + t) * 64 + lane) * 4) * w4[w];
        // lane holds d = 16 t + 4 g + r of query mq
        const size_t idx = (size_t)mq * qs + (size_t)h * HD + t * 16 + 4 * g;
        __half hh[4], hl[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) pf_split(acc[r] * inv, hh[r], hl[r]);
        *reinterpret_cast<uint2*>(a.ohi + idx) = *reinterpret_cast<const uint2*>(hh);
        *reinterpret_cast<uint2*>(a.olo + idx) = *reinterpret_cast<const uint2*>(hl);
    }
}

}  // namespace sli
