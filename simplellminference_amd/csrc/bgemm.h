// bgemm.h — batched decode projection on MFMA for gfx950: Y[b][row] = sum_k W[row][k] * X[b][k] for a
// batch of B <= 8 sequences decoding in lockstep ("the N=8 skinny GEMM is the only
// place MFMA pays"). It replaces the reference's one-row-per-block matmul_f32_kernel
// (source/kernel/cuda/matmul_kernel.cu:5-38) for B > 1, with the same fused epilogues as the batch-1
// GEMV (gemv.h): RMSNorm prologue (rms_kernel.cpp:5-23), RoPE + K/V cache write (rope_kernel.cpp:22-41),
// SwiGLU (swiglu_kernel.cpp:5-15), residual add (add_kernel.cpp:5-14), logits + argmax keys.
//
// Shape of the work (fp16 weights, fp32 activations, fp32 accumulate):
//   * the weight matrix is cut into 16-row tiles; the epilogue's tile row map lets a tile hold the RoPE
//     partner rows {d, d + hd/2} or the {gate u, up u} rows together (tile rows i and i + 8);
//   * v_mfma_f32_16x16x32_f16: A = 16 weight rows x 32 k straight from HBM (one 16-byte load per lane;
//     cdna_hip_programming.md §3 fragment layout: lane l holds row l&15, k 8(l>>4)..+7), B = 16
//     activation columns: column b < 8 is the fp16 high part of sequence b, column 8 + b its fp16 low
//     part (x - fp16(x)); the fp32 input is carried to ~2^-22 at no MFMA cost (the 8 spare columns of a
//     batch-8 tile) and hi + lo are summed in fp32 after the MFMA;
//   * a workgroup owns `tpw` consecutive tiles and one of `splits` contiguous k-ranges; its 16 waves split
//     the k-range of the current tile, stream it with the next two steps' loads in flight, and their 16
//     partials are reduced in LDS by one wave per tile (round-robin, off the other waves' path);
//   * the activations of the k-range are staged once per workgroup in LDS in the B-fragment layout
//     (lane-linear 16-byte slots: conflict-free ds_read_b128), RMS-normalised per sequence when fused;
//   * splits > 1: per-tile partials are published write-through (sc1) and the group's last-arriving
//     workgroup sums them in split order (deterministic) and runs the epilogue (the hand-off recipe of
//     attention.h, MI355X_MICROARCH.md).
#pragma once
#include "common.h"

namespace sli {

typedef _Float16 bg_half8 __attribute__((ext_vector_type(8)));
typedef float bg_float4 __attribute__((ext_vector_type(4)));

constexpr int kBgThreads = 1024;
constexpr int kBgWaves = kBgThreads / 64;
constexpr int kBgMaxBatch = 8;
constexpr int kBgNH = 4;               // staged half-slots (8 k of one sequence) per thread
constexpr int kBgMaxStageK = kBgNH * (kBgThreads / kBgMaxBatch) * 8;  // staged k per sequence <= 4096
constexpr int kBgScratch = 1024;       // bytes: ss partials [16][8] f32, inv [8] f32, keys [8] u64, flag
constexpr int kBgKeysOff = 640;
constexpr int kBgFlagOff = 704;
constexpr int kBgPBytes = 2 * kBgWaves * 16 * 8 * 4;  // double-buffered per-wave tile partials
constexpr int kBgLdsMax = 160 * 1024;
// 16-byte weight loads per lane per step (two steps in flight): 4, or 2 for one-tile plans (a finer
// pipeline over a workgroup's single tile; C4 wo 11.3 -> 10.7 us, TP-8 down 9.3 -> 7.4 us; the multi-tile
// plans lose with 2: down 31.6 -> 33.7 us) — bg_step_width
constexpr int bg_step_width(int tpw) { return tpw == 1 ? 2 : 4; }
// A plan whose waves own 6 or 7 k-blocks of every tile (C4 down: K 14336 over 4 splits, 7; the prefill's
// Llama-2 down: K 11008 over 4 splits, 6) streams each tile as ONE 7-vector step instead of 4 + 3 / 4 + 2
// (clamped duplicates in the second step): C4 down 31.6 -> 29.4 us, 512-token prefill +1.5 %.
#ifndef SLI_BG_U7_FROM
#define SLI_BG_U7_FROM 6
#endif
inline bool bg_seven_blocks(int splits, int K) {
    const int bpw = ((((K >> 5) + splits - 1) / splits) + kBgWaves - 1) / kBgWaves;
    return bpw >= SLI_BG_U7_FROM && bpw <= 7;
}

struct BgIn {
    const float* x;       // [B][K] fp32 activations
    const float* norm_w;  // fused RMSNorm weight [K], or nullptr
    float eps;
    int K;
    int B;
    int ntiles;           // 16-row output tiles
    int tpw;              // tiles per workgroup
    int splits;           // k-ranges (workgroups per tile group)
    float* ws;            // splits > 1: partials [ntiles][splits][16][8]
    unsigned* counters;   // splits > 1: [groups] arrival counters, zero between launches
    unsigned long long* stamps = nullptr;  // diagnostic (tools/bgemm_lab): per-workgroup s_memrealtime x4
    // W in the fragment layout (bg_tile_kernel): tile t's k-block kb is 1 KiB at ((t * K/32) + kb) * 1024, lane l's
    // 16-byte A operand at l * 16 — one wave load is one contiguous KiB (8 full 128-B lines) instead of 16 rows x
    // 64 B (16 half lines). 0: W row-major [rows][K] (the op-level entry, tools/bgemm_lab)
    int tiled = 0;
};

// ---------------------------------------------------------------- host-side plan
struct BgPlan {
    int ntiles = 0, tpw = 1, splits = 1, groups = 0;
    size_t lds = 0;
};

inline size_t bg_lds_bytes(int K, int splits, int tpw) {
    const int nkb = K / 32;
    const int kbs = (nkb + splits - 1) / splits;
    return (size_t)kBgScratch + (size_t)kbs * 1024 + kBgPBytes + (size_t)tpw * 512;
}

// (tiles per workgroup, k-splits) for a [16*ntiles x K] weight: about one workgroup per CU, the activation
// staging amortised over several tiles (B*K/splits*4 bytes from L2 per workgroup, plus B*K*4 for the
// fused RMS over the full row), the LDS image within 160 KiB. Cost in units of one 16x32 fp16 weight
// block (1 KiB of HBM); L2 bytes priced at a quarter of HBM bytes.
inline BgPlan bg_plan(int ntiles, int K, int B, bool norm, int cus = 256) {
    const int nkb = K / 32;
    BgPlan best;
    double best_cost = 1e30;
    for (int s = 1; s <= 16; ++s) {
        if (s > 1 && nkb / s < kBgWaves) break;  // every wave keeps at least one block per tile
        // the fused RMS needs the whole row in one workgroup (measured round 2: splitting k for the fused-
        // RMS plans, each split's sum of squares merged by the last arriver, was correct but slower — at
        // K 4096 a split leaves each wave one partly-filled step per tile and a barrier per step)
        if (norm && s > 1) break;
        const int kbs = (nkb + s - 1) / s;
        if (kbs * 32 > kBgMaxStageK) continue;  // staging registers
        for (int tpw = 1; tpw <= 64; ++tpw) {
            if (bg_lds_bytes(K, s, tpw) > (size_t)kBgLdsMax) break;
            const int groups = (ntiles + tpw - 1) / tpw;
            const int wgs = groups * s;
            const int rounds = (wgs + cus - 1) / cus;
            double per_wg = (double)tpw * kbs + 0.25 * kbs * B / 8.0 + 40.0;
            if (norm) per_wg += 0.25 * nkb * B / 8.0;
            if (s > 1) per_wg += 20.0 + 0.5 * s * tpw;
            const double cost = rounds * per_wg;
            if (cost < best_cost - 1e-9) {
                best_cost = cost;
                best.ntiles = ntiles;
                best.tpw = tpw;
                best.splits = s;
                best.groups = groups;
                best.lds = bg_lds_bytes(K, s, tpw);
            }
            if (groups == 1) break;
        }
    }
    return best;
}

// device workspace of a plan: split partials (256-B aligned), then one arrival counter per group
inline size_t bg_part_bytes(const BgPlan& p) {
    return p.splits > 1 ? (((size_t)p.ntiles * p.splits * 128 * sizeof(float) + 255) & ~(size_t)255) : 0;
}
inline size_t bg_ws_bytes(const BgPlan& p) { return bg_part_bytes(p) + sizeof(unsigned) * (size_t)p.groups + 256; }

// ---------------------------------------------------------------- device side
__device__ __forceinline__ bg_float4 bg_mfma(const u32x4& a, const u32x4& b, bg_float4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(bg_half8, a), __builtin_bit_cast(bg_half8, b), c,
                                                  0, 0, 0);
}

__device__ __forceinline__ float bg_load_sc1(const float* base, unsigned bytes, unsigned off) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, bytes, 0x00020000);
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 16 /* sc1 */));
}

// fp32 -> (fp16 hi, fp16 lo), hi + lo == v to ~2^-22 relative
__device__ __forceinline__ void bg_split8(const float* y, u32x4& hi, u32x4& lo) {
    unsigned h[4], l[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const _Float16 h0 = (_Float16)y[2 * p], h1 = (_Float16)y[2 * p + 1];
        const _Float16 l0 = (_Float16)(y[2 * p] - (float)h0), l1 = (_Float16)(y[2 * p + 1] - (float)h1);
        h[p] = (unsigned)__builtin_bit_cast(unsigned short, h0) | ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
        l[p] = (unsigned)__builtin_bit_cast(unsigned short, l0) | ((unsigned)__builtin_bit_cast(unsigned short, l1) << 16);
    }
    hi = u32x4{h[0], h[1], h[2], h[3]};
    lo = u32x4{l[0], l[1], l[2], l[3]};
}

// Epilogue contract (a mutable copy per thread):
//   row(t, i)                   weight row of tile t's row i (i < 16), always a valid row (clamped)
//   store(t, i, b, v0, v1, kl)  final sums of tile rows i (< 8) and i + 8 for sequence b; kl = the
//                               workgroup's per-sequence argmax keys in LDS
//   finish(kl, group, B)        once per workgroup that ran stores, after all of them
//   pre_a(t0, ntg, B), pre_b()  the epilogue's own inputs for this thread's first item (it = tid: tile t0 +
//                               (it >> 6), row pair (it >> 3) & 7, sequence it & 7), issued before the
//                               activation loads (pre_a) and right after the first weight steps (pre_b, for
//                               loads that depend on pre_a's), so they land during the stream instead of
//                               costing a round trip after it
template <class Epi, bool NORM, int kBgU = 4>
__global__ void __launch_bounds__(kBgThreads) bgemm_kernel(const __half* __restrict__ W, BgIn in, Epi epi_in) {
    Epi epi = epi_in;
    extern __shared__ __attribute__((aligned(16))) char bg_smem[];
    float* red = reinterpret_cast<float*>(bg_smem);  // [16][8]
    float* inv = red + kBgWaves * 8;                 // [8]
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(bg_smem + kBgKeysOff);
    int* flag = reinterpret_cast<int*>(bg_smem + kBgFlagOff);
    u32x4* img = reinterpret_cast<u32x4*>(bg_smem + kBgScratch);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int S = in.splits, K = in.K, B = in.B;
    const int g = blockIdx.x / S, s = blockIdx.x - g * S;
    const int nkb = K >> 5;
    const int kb0 = (s * nkb) / S, nkbs = ((s + 1) * nkb) / S - kb0;  // this split's 32-k blocks
    const int kbs_max = (nkb + S - 1) / S;
    float* P = reinterpret_cast<float*>(bg_smem + kBgScratch + (size_t)kbs_max * 1024);  // [2][16 waves][16][8]
    float* R = P + 2 * kBgWaves * 128;                                                 // [tpw][16][8]
    const int t0 = g * in.tpw;
    const int ntg = min(in.tpw, in.ntiles - t0);  // this workgroup's tiles (uniform)
    const int wb0 = kb0 + (wave * nkbs) / kBgWaves;  // this wave's blocks of every tile
    const int wnb = kb0 + ((wave + 1) * nkbs) / kBgWaves - wb0;
    const int per_wave_max = (nkbs + kBgWaves - 1) / kBgWaves;
    const int cpt = max((per_wave_max + kBgU - 1) / kBgU, 1);  // steps per tile (uniform)
    const int nsteps = ntg * cpt;

    if (tid < kBgMaxBatch) keys[tid] = 0ull;
    const unsigned long long t_entry = in.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    epi.pre_a(t0, ntg, B);

    // ---- 1. activation staging loads, issued first (s_waitcnt vmcnt counts in issue order). Thread t
    // stages sequence b = t & 7 at the 8-k groups (t >> 3) + 128 n: the 8 lanes of a group write 8
    // consecutive 16-byte image slots (conflict-free ds_write_b128), the loads stay 32 B per lane.
    // Without the fused RMS (wo, down) nothing needs the whole row, so every WAVE stages only its own
    // blocks [wb0, wb0 + wnb) (the blocks its MFMAs read, for every tile of the workgroup) and starts
    // streaming as soon as they land: no workgroup barrier behind the slowest wave's activations (the
    // B*K*4-byte image is pulled through L2 by 256 workgroups at once; profiles/r04_bgemm_lab_*).
    // Lane l: sequence l >> 3, block 2n + ((l >> 2) & 1), 8-k group l & 3: 8 lanes read 256
    // contiguous bytes of one sequence row.
    // With the fused RMS the norm is split the same way: the image holds x * w (rms_kernel.cpp:20-22
    // without the per-sequence 1/rms), every wave adds its blocks' sum of squares to LDS, and the
    // per-sequence 1/rms (:12-19) multiplies the finished row sums in the epilogue: a per-sequence scalar
    // commutes with the k-sum. NORM plans have one split (bg_plan), so the waves' blocks cover the row.
    const int sb = lane >> 3;
    const bool seq_live = sb < B;
    const int sbc = min(sb, B - 1);
    const int wq = lane & 3, wbo = (lane >> 2) & 1;  // per-wave staging: 8-k group, block offset
    float4 xa[kBgNH][2];
    float4 wn[NORM ? kBgNH : 1][2];
#ifdef BG_LAB_NOSTAGE  // tools/bgemm_lab only: no activation loads (an upper bound on what a ready image saves)
    constexpr bool kStage = false;
#else
    constexpr bool kStage = true;
#endif
#pragma unroll
    for (int n = 0; n < kBgNH; ++n) {
        const int blk = wb0 + max(min(2 * n + wbo, wnb - 1), 0);  // clamped into the row, never a branch
        const int k8 = min(blk, nkb - 1) * 4 + wq;
        const float4* xp = reinterpret_cast<const float4*>(in.x + (size_t)sbc * K + (size_t)k8 * 8);
        xa[n][0] = kStage ? xp[0] : make_float4(0.f, 0.f, 0.f, 0.f);
        xa[n][1] = kStage ? xp[1] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if constexpr (NORM && kStage) {
#pragma unroll
        for (int n = 0; n < kBgNH; ++n) {
            const int blk = wb0 + max(min(2 * n + wbo, wnb - 1), 0);
            const float4* wp = reinterpret_cast<const float4*>(in.norm_w + (size_t)(min(blk, nkb - 1) * 4 + wq) * 8);
            wn[n][0] = wp[0];
            wn[n][1] = wp[1];
        }
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- 2. the first two weight steps
    const size_t row_bytes = (size_t)K * 2;
    const int q8 = (lane >> 4) * 8;  // this lane's k offset inside a 32-k block
    const size_t bstride = in.tiled ? 1024 : 64;  // bytes between a lane's consecutive k-blocks
    auto load_step = [&](int k, u32x4(&w)[kBgU]) {
        const int kk = min(k, nsteps - 1);
        const int j = kk / cpt, c = kk - j * cpt;
        const char* base;
        if (in.tiled) {
            base = reinterpret_cast<const char*>(W) + (size_t)(t0 + j) * nkb * 1024 + (size_t)lane * 16;
        } else {
            const int row = epi.row(t0 + j, lane & 15);
            base = reinterpret_cast<const char*>(W) + (size_t)row * row_bytes + (size_t)q8 * 2;
        }
#pragma unroll
        for (int u = 0; u < kBgU; ++u) {
            const int bi = wb0 + min(c * kBgU + u, max(wnb - 1, 0));
            w[u] = load16<true>(base + (size_t)bi * bstride);
        }
    };
    u32x4 wa[kBgU], wb[kBgU];  // (a third step in flight measured slower: C4 1660 -> 1546 tok/s)
    load_step(0, wa);
    load_step(1, wb);
    __builtin_amdgcn_sched_barrier(0);
    epi.pre_b();

    // ---- 3./4. this wave's blocks into LDS as B fragments (hi: column b, lo: 8 + b), visible to the
    // wave's own later reads after lgkmcnt(0); NORM: x * w staged, this wave's sum of x^2 to red[wave][b]
    float ss = 0.0f;
#pragma unroll
    for (int n = 0; n < kBgNH; ++n) {
        const int bw = 2 * n + wbo;
        float y[8] = {xa[n][0].x, xa[n][0].y, xa[n][0].z, xa[n][0].w, xa[n][1].x, xa[n][1].y, xa[n][1].z, xa[n][1].w};
        if constexpr (NORM) {
            float v = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) v += y[e] * y[e];
            ss += bw < wnb ? v : 0.0f;
            const float wv[8] = {wn[n][0].x, wn[n][0].y, wn[n][0].z, wn[n][0].w,
                                 wn[n][1].x, wn[n][1].y, wn[n][1].z, wn[n][1].w};
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = y[e] * wv[e];
        }
        if (seq_live && bw < wnb) {
            u32x4 hi, lo;
            bg_split8(y, hi, lo);
            const int ib = wb0 - kb0 + bw;
            img[ib * 64 + wq * 16 + sb] = hi;
            img[ib * 64 + wq * 16 + 8 + sb] = lo;
        }
    }
    if constexpr (NORM) {
        ss = group_sum<8>(ss);  // the 8 lanes of one sequence
        if ((lane & 7) == 0) red[wave * 8 + sb] = ss;  // read after the stream's final barrier
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();

    const unsigned long long t_staged = in.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    // ---- 5. stream the tiles
    bg_float4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const u32x4* wimg = img + (size_t)(wb0 - kb0) * 64 + lane;
    auto mfma_step = [&](int k, const u32x4(&w)[kBgU]) {
        const int c = k - (k / cpt) * cpt;
#pragma unroll
        for (int u = 0; u < kBgU; ++u) {
            const int r = c * kBgU + u;
            if (r < wnb) acc = bg_mfma(w[u], wimg[(size_t)r * 64], acc);
        }
    };
    auto tile_end = [&](int k) {
        const int j = k / cpt, c = k - j * cpt;
        if (c == cpt - 1) {  // tile j complete in every wave (uniform branch)
            float* Pb = P + (j & 1) * (kBgWaves * 128);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] += dpp_f<kDppRor8>(acc[r]);  // hi + lo columns (lane + 8)
            if ((lane & 8) == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) Pb[wave * 128 + ((lane >> 4) * 4 + r) * 8 + (lane & 7)] = acc[r];
            }
            acc = bg_float4{0.0f, 0.0f, 0.0f, 0.0f};
            __syncthreads();
            if (wave == (j & (kBgWaves - 1))) {  // tile j's 16 wave partials, summed in wave order
                const int i = lane >> 3, b = lane & 7;
                float v0 = 0.0f, v1 = 0.0f;
#pragma unroll
                for (int w = 0; w < kBgWaves; ++w) {
                    v0 += Pb[w * 128 + i * 8 + b];
                    v1 += Pb[w * 128 + (i + 8) * 8 + b];
                }
                R[j * 128 + i * 8 + b] = v0;
                R[j * 128 + (i + 8) * 8 + b] = v1;
            }
        }
    };
    int k = 0;
    // The next step's loads go out as soon as the current step's MFMAs have read their registers, BEFORE
    // the tile-end workgroup barrier: two steps stay in flight through every tile boundary.
    for (; k + 2 < nsteps; k += 2) {
        mfma_step(k, wa);
        load_step(k + 2, wa);
        tile_end(k);
        mfma_step(k + 1, wb);
        load_step(k + 3, wb);
        tile_end(k + 1);
    }
    if (k < nsteps) {
        mfma_step(k, wa);
        tile_end(k);
    }
    if (k + 1 < nsteps) {
        mfma_step(k + 1, wb);
        tile_end(k + 1);
    }
    __syncthreads();
    if constexpr (NORM) {  // per-sequence 1/rms from the waves' sums of squares, in wave order
        if (tid < B) {
            float t = 0.0f;
            for (int w = 0; w < kBgWaves; ++w) t += red[w * 8 + tid];
            const float tep = t / (float)K;         // rms_kernel.cpp:17
            const float rms = sqrtf(tep + in.eps);  // :18
            inv[tid] = 1.0f / rms;                  // :19
        }
        __syncthreads();
    }
    if (in.stamps && tid == 0) {
        unsigned long long* p = in.stamps + (size_t)blockIdx.x * 4;
        p[0] = t_entry;
        p[1] = t_staged;
        p[2] = __builtin_amdgcn_s_memrealtime();
    }

    // ---- 6. epilogue (one split) or publish + the group's last arriver merges in split order
    const int items = ntg * 64;  // (tile, row pair i < 8, sequence slot b < 8)
    if (S == 1) {
        for (int it = tid; it < items; it += kBgThreads) {
            const int j = it >> 6, i = (it >> 3) & 7, b = it & 7;
            const float iv = NORM ? inv[b] : 1.0f;
            if (b < B) epi.store(t0 + j, i, b, R[j * 128 + i * 8 + b] * iv, R[j * 128 + (i + 8) * 8 + b] * iv, keys);
        }
    } else {
        for (int e = tid; e < ntg * 128; e += kBgThreads) {
            const int j = e >> 7, r = e & 127;
            __hip_atomic_store(in.ws + ((size_t)(t0 + j) * S + s) * 128 + r, R[e], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the arrival
        __syncthreads();
        if (tid == 0) {
            const unsigned prev = __hip_atomic_fetch_add(in.counters + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = prev == (unsigned)(S - 1);
            if (*flag) __hip_atomic_store(in.counters + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (*flag == 0) return;  // uniform
        const float* base = in.ws + (size_t)t0 * S * 128;
        const unsigned bytes = (unsigned)(sizeof(float) * (size_t)ntg * S * 128);
        for (int it = tid; it < items; it += kBgThreads) {
            const int j = it >> 6, i = (it >> 3) & 7, b = it & 7;
            if (b >= B) continue;
            float v0 = 0.0f, v1 = 0.0f;
            for (int sp = 0; sp < S; ++sp) {  // split order: deterministic
                const unsigned o = (unsigned)((j * S + sp) * 128);
                v0 += bg_load_sc1(base, bytes, 4u * (o + i * 8 + b));
                v1 += bg_load_sc1(base, bytes, 4u * (o + (i + 8) * 8 + b));
            }
            epi.store(t0 + j, i, b, v0, v1, keys);
        }
    }
    epi.finish(keys, g, B);
    if (in.stamps && tid == 0) in.stamps[(size_t)blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------- epilogues
// Plain rows: tile t holds rows 16t .. 16t+15. y[b][row] = resid[b][row] + (sum * rscale[row]) * scale
// (matmul_kernel.cpp:26 fused with add_kernel.cpp:5-14).
struct BgEpiStore {
    float* y;
    const float* resid;
    const float* rscale;
    float scale;
    int nrows;
    int ld;  // per-sequence stride of y / resid
    __device__ int row(int t, int i) const { return min(t * 16 + i, nrows - 1); }
    // (prefetching the residuals measured slower: C4 wo 8.89 -> 9.21 us, profiles/r4_bg_epi_prefetch_ab.txt)
    __device__ void pre_a(int, int, int) {}
    __device__ void pre_b() {}
    __device__ void one(int row, int b, float v) const {
        if (row >= nrows) return;
        float a = rscale ? v * rscale[row] : v;
        a = a * scale;
        const size_t o = (size_t)b * ld + row;
        y[o] = resid ? resid[o] + a : a;
    }
    __device__ void store(int t, int i, int b, float v0, float v1, unsigned long long*) const {
        one(t * 16 + i, b, v0);
        one(t * 16 + i + 8, b, v1);
    }
    __device__ void finish(unsigned long long*, int, int) const {}
};

// Fused q/k/v + RoPE + K/V cache write (model.cpp:54-67) per sequence: tile rows i and i + 8 are the
// RoPE pair {d, d + hd/2} of one head (8 pairs per tile). Cache [B][hkv][T][hd] per layer; sequence b's
// position is pos_dev[b * pos_stride].
template <typename KT>
struct BgEpiQKV {
    float* q_out;  // [B][hq*hd]
    KT* kc;        // layer base
    KT* vc;
    const int32_t* pos_dev;
    int pos_stride;
    const float* sin_t;
    const float* cos_t;
    int hq, hkv, hd, T;
    int kv_seq = 1;  // 1: sequence b owns cache heads [b*hkv, (b+1)*hkv); 0: one cache shared by every lane
                     // (prefill lanes of one sequence at consecutive positions)
    int p_t = -1, p_i = 0, p_b = 0, p_pos = 0;  // the prefetched item: its position, then its RoPE row
    float p_sin = 0.0f, p_cos = 0.0f;
    __device__ void pre_a(int t0, int ntg, int B) {
        const int it = threadIdx.x;
        if (it >= ntg * 64 || (it & 7) >= B) return;
        p_t = t0 + (it >> 6);
        p_i = (it >> 3) & 7;
        p_b = it & 7;
        p_pos = pos_dev[(size_t)p_b * pos_stride];
    }
    __device__ void pre_b() {
        if (p_t < 0) return;
        const int half = hd >> 1;
        const int u = p_t * 8 + p_i;
        const int uh = u / half, d = u - uh * half;
        if (uh < hq + hkv) {
            p_sin = sin_t[p_pos * half + d];
            p_cos = cos_t[p_pos * half + d];
        }
    }
    __device__ int row(int t, int i) const {
        const int half = hd >> 1;
        const int u = t * 8 + (i & 7);
        const int uh = u / half, d = u - uh * half;
        return uh * hd + d + (i >= 8 ? half : 0);
    }
    __device__ void store(int t, int i, int b, float a0, float a1, unsigned long long*) const {
        const int half = hd >> 1;
        const int u = t * 8 + i;
        const int uh = u / half, d = u - uh * half;
        const bool pre = t == p_t && i == p_i && b == p_b;
        const int pos = pre ? p_pos : pos_dev[(size_t)b * pos_stride];
        if (uh < hq + hkv) {  // rope_kernel.cpp:30-38
            const float fci = pre ? p_sin : sin_t[pos * half + d], fcr = pre ? p_cos : cos_t[pos * half + d];
            const float r0 = a0 * fcr - a1 * fci;
            const float r1 = a1 * fcr + a0 * fci;
            if (uh < hq) {
                float* q = q_out + ((size_t)b * hq + uh) * hd;
                q[d] = r0;
                q[d + half] = r1;
            } else {
                KT* kp = kc + (((size_t)b * kv_seq * hkv + (uh - hq)) * T + pos) * hd;
                kp[d] = from_f32<KT>(r0);
                kp[d + half] = from_f32<KT>(r1);
            }
        } else {
            KT* vp = vc + (((size_t)b * kv_seq * hkv + (uh - hq - hkv)) * T + pos) * hd;
            vp[d] = from_f32<KT>(a0);
            vp[d + half] = from_f32<KT>(a1);
        }
    }
    __device__ void finish(unsigned long long*, int, int) const {}
};

// Fused gate/up + activation (model.cpp:99-115): fused rows [gate(I); up(I)]; tile rows i / i + 8 are
// gate u / up u for u = 8t + i.
struct BgEpiSwiGLU {
    float* act;  // [B][inter]
    int inter;
    int silu;
    __device__ int row(int t, int i) const { return t * 8 + (i & 7) + (i >= 8 ? inter : 0); }
    __device__ void pre_a(int, int, int) {}
    __device__ void pre_b() {}
    __device__ void store(int t, int i, int b, float g, float up, unsigned long long*) const {
        float sg = 1.0f / (1.0f + expf(-g));  // swiglu_kernel.cpp:12
        if (silu) sg = g * sg;
        act[(size_t)b * inter + t * 8 + i] = sg * up;  // :13
    }
    __device__ void finish(unsigned long long*, int, int) const {}
};

// LM head (model.cpp:136-139) per sequence + the first stage of the device argmax: the workgroup that
// ran a group's stores writes each sequence's max orderable key to keys_out[b][group].
struct BgEpiLogits {
    float* logits;                 // [B][ld]
    unsigned long long* keys_out;  // [B][key_ld]
    int nrows, ld, vocab_off, key_ld;
    __device__ int row(int t, int i) const { return min(t * 16 + i, nrows - 1); }
    __device__ void pre_a(int, int, int) {}
    __device__ void pre_b() {}
    __device__ void one(int row, int b, float v, unsigned long long* kl) const {
        if (row >= nrows) return;
        logits[(size_t)b * ld + row] = v;
        atomicMax(kl + b, argmax_key(v, (unsigned)(row + vocab_off)));  // a max: order-independent
    }
    __device__ void store(int t, int i, int b, float v0, float v1, unsigned long long* kl) const {
        one(t * 16 + i, b, v0, kl);
        one(t * 16 + i + 8, b, v1, kl);
    }
    __device__ void finish(unsigned long long* kl, int g, int B) const {
        __syncthreads();
        if ((int)threadIdx.x < B) keys_out[(size_t)threadIdx.x * key_ld + g] = kl[threadIdx.x];
    }
};

// Row-major W [rows][K] -> the fragment layout of BgIn::tiled, rows in the epilogue's tile order (Epi::row:
// RoPE pairs, gate/up pairs, the last tile's clamped rows): out[(t * K/32 + kb) * 64 + l] (16-byte pieces) =
// W[row(t, l & 15)][32 kb + 8 (l >> 4) .. + 7]. Init-time only (weights placed or replaced).
template <class Epi>
__global__ void __launch_bounds__(256) bg_tile_kernel(const __half* __restrict__ W, int K, int ntiles, Epi epi,
                                                       uint4* __restrict__ out) {
    const int nkb = K / 32;
    const size_t n = (size_t)ntiles * nkb * 64;
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x) {
        const int l = (int)(p & 63);
        const size_t tb = p >> 6;
        const int t = (int)(tb / nkb), kb = (int)(tb - (size_t)t * nkb);
        const int row = epi.row(t, l & 15);
        out[p] = *reinterpret_cast<const uint4*>(W + (size_t)row * K + (size_t)kb * 32 + 8 * (l >> 4));
    }
}

template <class Epi>
hipError_t launch_bg_tile(const __half* W, int K, int ntiles, const Epi& epi, void* out, hipStream_t s) {
    if (K % 32) return hipErrorInvalidValue;
    const size_t n = (size_t)ntiles * (K / 32) * 64;
    const int blocks = (int)std::min<size_t>(8192, (n + 255) / 256);
    hipLaunchKernelGGL((bg_tile_kernel<Epi>), dim3(blocks), dim3(256), 0, s, W, K, ntiles, epi,
                       reinterpret_cast<uint4*>(out));
    return hipGetLastError();
}
// bytes of a tiled matrix
inline size_t bg_tiled_bytes(int ntiles, int K) { return (size_t)ntiles * (size_t)(K / 32) * 1024; }

// Allow the kernel its full dynamic LDS (once per instantiation; call outside stream capture).
template <class Epi, bool NORM>
hipError_t bg_allow_lds() {
    static const hipError_t e = [] {
        const hipError_t e4 = hipFuncSetAttribute(reinterpret_cast<const void*>(&bgemm_kernel<Epi, NORM, 4>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, kBgLdsMax);
        const hipError_t e2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&bgemm_kernel<Epi, NORM, 2>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, kBgLdsMax);
        if (!NORM) {
            const hipError_t e7 = hipFuncSetAttribute(reinterpret_cast<const void*>(&bgemm_kernel<Epi, NORM, 7>),
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, kBgLdsMax);
            if (e7 != hipSuccess) return e7;
        }
        return e4 != hipSuccess ? e4 : e2;
    }();
    return e;
}

template <class Epi>
hipError_t launch_bgemm(const __half* W, const BgIn& in_, const Epi& epi, const BgPlan& p, hipStream_t s) {
    BgIn in = in_;
    in.ntiles = p.ntiles;
    in.tpw = p.tpw;
    in.splits = p.splits;
    const dim3 grid(p.groups * p.splits);
    if (in.norm_w && p.splits != 1) return hipErrorInvalidValue;  // the fused RMS runs on one split only
    const bool u2 = bg_step_width(p.tpw) == 2;
    if (in.norm_w && u2)
        hipLaunchKernelGGL((bgemm_kernel<Epi, true, 2>), grid, dim3(kBgThreads), p.lds, s, W, in, epi);
    else if (in.norm_w)
        hipLaunchKernelGGL((bgemm_kernel<Epi, true, 4>), grid, dim3(kBgThreads), p.lds, s, W, in, epi);
    else if (u2)
        hipLaunchKernelGGL((bgemm_kernel<Epi, false, 2>), grid, dim3(kBgThreads), p.lds, s, W, in, epi);
    else if (bg_seven_blocks(p.splits, in.K))
        hipLaunchKernelGGL((bgemm_kernel<Epi, false, 7>), grid, dim3(kBgThreads), p.lds, s, W, in, epi);
    else
        hipLaunchKernelGGL((bgemm_kernel<Epi, false, 4>), grid, dim3(kBgThreads), p.lds, s, W, in, epi);
    return hipGetLastError();
}

}  // namespace sli
