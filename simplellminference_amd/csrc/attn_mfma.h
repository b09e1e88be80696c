// attn_mfma.h — single-token decode attention for an fp16 K/V cache on the matrix cores (gfx950), the
// reference's score / softmax / value trio (source/kernel/cpu/mha_kernel.cpp:36-77; CUDA
// source/kernel/cuda/mha_kernel.cu:63-169) as split-context flash-decoding whose K/V bytes in flight cost no
// registers:
//
//   * workgroup = 4 waves = one (kv head, context split of 128 * tpw positions); wave w owns the split's
//     32-key tiles w, w + 4, w + 8, ...;
//   * a tile's K and V rows reach the wave's own LDS images by LDS-DMA (global_load_lds_dwordx4, nt: each
//     cache row is read once per step), 16-B chunks XOR-swizzled; a wave keeps two tiles in flight (a
//     2-deep ring of its own, no workgroup barrier) and computes one while the next lands;
//   * Sᵀ[key][query] = K Qᵀ on v_mfma_f32_16x16x32_f16: A = 16 K rows (exact fp16), B = the G query heads
//     of the kv head as columns 0..G-1, fp32 q split into fp16 hi + mid + lo (three MFMAs into one
//     accumulator), so the products carry q in full and sum in fp32;
//   * online softmax per query column (a lane's 8 keys, then the 4 lane groups by xor 16 / 32); every
//     lane of a column holds its running (max, sum), so no lane exchange besides those two;
//   * Oᵀ[d][query] += Vᵀ Pᵀ: B = Pᵀ straight from the Sᵀ accumulators (k order {4g..4g+3, 16+4g..16+4g+3},
//     g = lane >> 4), P as hi + mid + lo fp16; A = Vᵀ by ds_read_b64_tr_b16, whose 4-row blocks are those keys;
//   * the 4 waves' (max, sum, o) merge in LDS into one partial per (q head, split), stored in the layout of
//     attention.h (o[hd], m, l) so every split consumer works unchanged: the wo GEMV's input staging
//     (defer_merge 1), attn_merge_kernel (2), or the head's last-arriving workgroup (0, attention.h
//     attn_merge, in split order).
//
// Why (round-4 C4 analysis): the register-staged GQA-4 kernel holds K/V bytes in flight in
// VGPRs (128 per lane), so its 1024 workgroups run in two residency rounds of K burst -> scores -> V burst
// with HBM idle between the bursts; its VALU work (fp16 -> fp32 unpack, 4 heads x 256 FMAs per key, row
// reductions) is ~9 us per CU at C4. Here the matrix cores do that work in ~1 us per CU and the in-flight
// bytes live in LDS, so one resident round streams the whole context.
#pragma once
#include "attention.h"

namespace sli {

constexpr int kAmWaves = 4;   // waves per workgroup (one per SIMD)
constexpr int kAmKeys = 32;   // keys per tile
constexpr int kAmWgKeys = kAmWaves * kAmKeys;  // keys per workgroup per tile round: ppwg = kAmWgKeys * tpw

template <int HD, int G>
struct AmGeo {
    static constexpr int ROWB = HD * 2;              // bytes per cache row
    static constexpr int IMG = kAmKeys * ROWB;       // one 32-key K (or V) image
    static constexpr int TILE = 2 * IMG;             // K + V
    static constexpr int PIECES = TILE / 1024;       // 1-KiB DMA pieces per tile
    static constexpr int CPR = ROWB / 16;            // 16-B chunks per row
    static constexpr int QB = ((G * HD * 4 + 1023) / 1024) * 1024;  // the q image (fp32), whole pieces
    static constexpr int QP = QB / 1024;
    static constexpr int ND = HD / 32, NT = HD / 16;  // 32-d blocks (S), 16-d tiles (O)
    template <int NBUF>
    static constexpr int wave_bytes() { return QB + NBUF * TILE; }
    static_assert(HD == 64 || HD == 128, "head_dim");
    static_assert(G >= 1 && G <= 16, "query heads per kv head: one MFMA column each");
};
// chunk swizzles of the K and V images (as prefill.h pf_attn_mfma_kernel): conflict-free ds_read_b128 row
// reads of K and ds_read_b64_tr_b16 transposed reads of V
__device__ __forceinline__ int am_swz_k(int r, int rowb) { return rowb == 256 ? r & 15 : (r >> 1) & 7; }
__device__ __forceinline__ int am_swz_v(int r, int rowb) { return rowb == 256 ? (r & 7) << 1 : ((r >> 1) & 3) << 1; }

// LDS-DMA of one 1-KiB piece (NT: non-temporal, aux 2, for the once-read K/V rows: MI355X_MICROARCH.md
// nt-weights; q, read by every split of its head, keeps the default policy): lane i's 16 bytes at gsrc
// land at LDS byte lds + 16 i. Inline asm, so the compiler neither counts nor drains it: the kernel waits with
// counted vmcnt, and issues no other vector-memory load while a piece is in flight.
template <bool NT>
__device__ __forceinline__ void am_dma(const void* gsrc, unsigned lds) {
    unsigned keep;
    if constexpr (NT)
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off nt\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(gsrc), "s"(lds)
            : "memory");
    else
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
__device__ __forceinline__ void am_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ uint2 am_tr_read(unsigned lds_addr) {
    uint2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr) : "memory");
    return v;
}
typedef _Float16 am_half8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float am_float4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ am_float4 am_mfma(const u32x4& a, const u32x4& b, am_float4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(am_half8, a), __builtin_bit_cast(am_half8, b), c,
                                                  0, 0, 0);
}
// fp32 -> fp16 hi + mid + lo: v - hi - mid - lo is below 2^-33 |v| (or the fp16 subnormal step 2^-24 for |v| <
// 2^-9), so the three exact fp16 products of an MFMA carry the fp32 operand in full (a hi + lo pair carries 22
// bits: measured at C4 position 1, where 32 layers amplify every rounding of the new K/V rows, the pair put the
// logits 1.51e-3 from a float64 restatement against 1.04 - 1.34e-3 for fp32 summation orders)
__device__ __forceinline__ void am_split3(float v, __half& hi, __half& mid, __half& lo) {
    hi = __float2half_rn(v);
    const float r = v - __half2float(hi);  // exact
    mid = __float2half_rn(r);
    lo = __float2half_rn(r - __half2float(mid));
}

// The head's last-arriving workgroup merges its ns live split partials into out (attention.h attn_merge's
// arithmetic: M = max m_i, w_i = e^{m_i - M}, out = sum w_i o_i / sum w_i l_i). A thread pair owns 4 consecutive
// outputs (q head g, dims d .. d+3): each thread of the pair merges every other split (its own max, rescaled
// sums), loading all of them in ONE batch of 16-byte o and 8-byte (m, l) write-through copies (sc1; 16 splits
// per thread: ns <= 32 in one round trip), and the pair combines over DPP (lanes 2j, 2j+1). Deterministic: a
// fixed split-to-thread map and combine order.
template <int HD, int G, int NSH>
__device__ __forceinline__ void am_merge(const float* part, float* out, int kvh, int max_splits, int ns) {
    constexpr int PS = HD + kAttnPartPad, NOG = G * HD / 4, NTH = 64 * kAmWaves, NPASS = (2 * NOG + NTH - 1) / NTH;
    const unsigned bytes = (unsigned)(sizeof(float) * (size_t)G * max_splits * PS);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(part + (size_t)kvh * G * max_splits * PS), 0,
                                                      bytes, 0x00020000);
    const int half = threadIdx.x & 1;
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
        const int og = min((int)(threadIdx.x >> 1) + pass * (NTH / 2), NOG - 1);  // (clamped: every lane of the pair
        const int g = og / (HD / 4), d = (og % (HD / 4)) * 4;                  //  computes, only valid ones store)
        float M = -INFINITY, L = 0.0f;
        float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        for (int s0 = half; s0 < ns; s0 += 2 * NSH) {
            u32x4 ov[NSH];
            u32x2 ml[NSH];
#pragma unroll
            for (int j = 0; j < NSH; ++j) {  // splits s0, s0 + 2, ... (clamped to the last live split of this half)
                const int sj = min(s0 + 2 * j, ns - 1 - ((ns - 1 - half) & 1));
                const unsigned r = (unsigned)(g * max_splits + sj) * PS;
                ov[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, 4u * (r + d), 0, 16 /* sc1 */);
                ml[j] = __builtin_amdgcn_raw_buffer_load_b64(rs, 4u * (r + HD), 0, 16);
            }
            float mb = M;
#pragma unroll
            for (int j = 0; j < NSH; ++j) mb = fmaxf(mb, __uint_as_float(ml[j].x));  // duplicates leave the max
            const float c = expf(M - mb);  // 0 on the first batch
            o.x *= c, o.y *= c, o.z *= c, o.w *= c;
            L *= c;
#pragma unroll
            for (int j = 0; j < NSH; ++j) {
                if (s0 + 2 * j < ns) {
                    const float w = expf(__uint_as_float(ml[j].x) - mb);
                    o.x = fmaf(w, __uint_as_float(ov[j].x), o.x);
                    o.y = fmaf(w, __uint_as_float(ov[j].y), o.y);
                    o.z = fmaf(w, __uint_as_float(ov[j].z), o.z);
                    o.w = fmaf(w, __uint_as_float(ov[j].w), o.w);
                    L = fmaf(w, __uint_as_float(ml[j].y), L);
                }
            }
            M = mb;
        }
        // the pair: the even lane's splits first (a fixed order)
        const float Mp = dpp_f<kDppXor1>(M), Lp = dpp_f<kDppXor1>(L);
        const float4 op = make_float4(dpp_f<kDppXor1>(o.x), dpp_f<kDppXor1>(o.y), dpp_f<kDppXor1>(o.z),
                                      dpp_f<kDppXor1>(o.w));
        const float Mt = fmaxf(M, Mp);  // finite: split 0 is live, and it is the even lane's
        const float ce = expf((half ? Mp : M) - Mt), co = expf((half ? M : Mp) - Mt);  // even, odd lane's weights
        const float4 oe = half ? op : o, oo = half ? o : op;
        const float Le = half ? Lp : L, Lo = half ? L : Lp;
        const float Lt = fmaf(ce, Le, co * Lo);
        const int ogv = (int)(threadIdx.x >> 1) + pass * (NTH / 2);
        if (half == 0 && ogv < NOG)
            *reinterpret_cast<float4*>(out + (size_t)kvh * G * HD + (size_t)g * HD + d) =
                make_float4(fmaf(ce, oe.x, co * oo.x) / Lt, fmaf(ce, oe.y, co * oo.y) / Lt,
                            fmaf(ce, oe.z, co * oo.z) / Lt, fmaf(ce, oe.w, co * oo.w) / Lt);
    }
}

// grid: n_kv_heads (every sequence's) * max_splits workgroups of 256 threads; a.ppwg = kAmWgKeys * tpw (the
// split length), NBUF = min(tpw, 2) ring slots per wave. The K/V rows of a split are read once (clamped to pos:
// rows past the live context re-read row pos, an L2 hit, and are masked).
template <int HD, int G, int NBUF>
__global__ void __launch_bounds__(64 * kAmWaves) attn_mfma_kernel(AttnArgs<__half> a) {
    using Geo = AmGeo<HD, G>;
    constexpr int ND = Geo::ND, NT = Geo::NT, P = Geo::PIECES;
    constexpr int WB = Geo::template wave_bytes<NBUF>();
    __shared__ __attribute__((aligned(1024))) char sm[kAmWaves * WB];
    __shared__ int last;
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4] = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int g = lane >> 4, i16 = lane & 15;
    const int kvh = blockIdx.x / a.max_splits, wgs = blockIdx.x - kvh * a.max_splits;
    const int pos = attn_pos(a, kvh);
    const int ppwg = a.ppwg;
    const int s0 = wgs * ppwg;
    if (s0 > pos) return;  // the whole split past the live context (uniform)
    const int tpw = ppwg / kAmWgKeys;
    const int rel = pos - s0;
    // live tiles of this wave: j with s0 + (4 j + wave) * 32 <= pos
    const int nl = rel >= wave * kAmKeys ? min(tpw, (rel / kAmKeys - wave) / kAmWaves + 1) : 0;

    char* wimg = sm + wave * WB;
    const unsigned wbase = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)wimg;
    const unsigned qbase = wbase, tbase = wbase + Geo::QB;
    const int ch = a.cache_heads > 0 ? kvh % a.cache_heads : kvh / a.kv_group;
    const __half* kc = a.k + (long long)ch * a.head_stride;
    const __half* vc = a.v + (long long)ch * a.head_stride;

    // tile j of this wave into ring slot j % NBUF: K pieces 0 .. P/2-1, V pieces P/2 .. P-1; lane i of a piece:
    // row (piece rows) + i / CPR, physical chunk i % CPR <- logical chunk (i % CPR) ^ swizzle(row)
    auto issue = [&](int j) {
        const int t0 = s0 + (kAmWaves * j + wave) * kAmKeys;
        const unsigned base = tbase + (unsigned)((j % NBUF) * Geo::TILE);
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const bool isv = p >= P / 2;
            const int jj = isv ? p - P / 2 : p;
            const int r = jj * (1024 / Geo::ROWB) + lane / Geo::CPR;
            const int c = (lane % Geo::CPR) ^ (isv ? am_swz_v(r, Geo::ROWB) : am_swz_k(r, Geo::ROWB));
            const __half* src = (isv ? vc : kc) + (long long)min(t0 + r, pos) * a.pos_stride + c * 8;
            am_dma<true>(src, base + (isv ? Geo::IMG : 0) + (unsigned)(jj * 1024));
        }
    };
    // q of the kv head's G query heads (fp32, contiguous): QP pieces, clamped inside the vector
    {
        const float* qs = a.q + (size_t)kvh * G * HD;
#pragma unroll
        for (int p = 0; p < Geo::QP; ++p)
            am_dma<false>(qs + min(p * 256 + lane * 4, G * HD - 4), qbase + (unsigned)(p * 1024));
    }
    if (nl > 0) issue(0);
    if (NBUF > 1 && nl > 1) issue(1);
    if (NBUF > 1 && nl > 1)  // q landed (the tiles may still be in flight)
        am_wait_vm<2 * P>();
    else if (nl > 0)
        am_wait_vm<P>();
    else
        am_wait_vm<0>();
    // Qᵀ as the B operand: lane l = query column l & 15 (q head kvh * G + col for col < G, else zero), d = 32 db +
    // 8 g .. +7, fp32 -> hi + lo
    u32x4 qh[ND], qm[ND], ql[ND];
#pragma unroll
    for (int db = 0; db < ND; ++db) {
        float f[8];
        if (i16 < G) {
            const float4* qp = reinterpret_cast<const float4*>(wimg + 4 * (i16 * HD + db * 32 + g * 8));
            const float4 v0 = qp[0], v1 = qp[1];
            f[0] = v0.x, f[1] = v0.y, f[2] = v0.z, f[3] = v0.w, f[4] = v1.x, f[5] = v1.y, f[6] = v1.z, f[7] = v1.w;
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = 0.0f;
        }
        __half hh[8], hm[8], hl[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) am_split3(f[e], hh[e], hm[e], hl[e]);
        qh[db] = *reinterpret_cast<const u32x4*>(hh);
        qm[db] = *reinterpret_cast<const u32x4*>(hm);
        ql[db] = *reinterpret_cast<const u32x4*>(hl);
    }
    am_float4 o[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) o[t] = am_float4{0.0f, 0.0f, 0.0f, 0.0f};
    float mx = -INFINITY, l = 0.0f;
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();

    for (int j = 0; j < nl; ++j) {
        // tile j landed (tile j + 1 may still be in flight)
        if (NBUF > 1 && j + 1 < nl)
            am_wait_vm<P>();
        else
            am_wait_vm<0>();
        const int t0 = s0 + (kAmWaves * j + wave) * kAmKeys;
        const char* kimg = wimg + Geo::QB + (j % NBUF) * Geo::TILE;
        const unsigned vbase = tbase + (unsigned)((j % NBUF) * Geo::TILE) + Geo::IMG;
        // Sᵀ[key][query] for keys t0 + 16 kt + (0..15)
        am_float4 sacc[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
            sacc[kt] = am_float4{0.0f, 0.0f, 0.0f, 0.0f};
            const int r = kt * 16 + i16;
            const char* krow = kimg + r * Geo::ROWB;
#pragma unroll
            for (int db = 0; db < ND; ++db) {
                const u32x4 kf = *reinterpret_cast<const u32x4*>(krow + ((4 * db + g) ^ am_swz_k(r, Geo::ROWB)) * 16);
                sacc[kt] = am_mfma(kf, qh[db], sacc[kt]);
                sacc[kt] = am_mfma(kf, qm[db], sacc[kt]);
                sacc[kt] = am_mfma(kf, ql[db], sacc[kt]);
            }
        }
        // Vᵀ 16-d tile dt: lane 16 g + 4 q + p addresses row (4 g + q) [+16], d 16 dt + 4 p .. +3 (issued before the
        // softmax so the LDS reads overlap it)
        const int q4 = (lane & 15) >> 2, p4 = lane & 3;
        const int r1 = 4 * g + q4, r2 = 16 + 4 * g + q4;
        const unsigned a1 = vbase + r1 * Geo::ROWB + 8 * (p4 & 1), a2 = vbase + r2 * Geo::ROWB + 8 * (p4 & 1);
        const int sw1 = am_swz_v(r1, Geo::ROWB), sw2 = am_swz_v(r2, Geo::ROWB);
        uint2 x1[NT], x2[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int c = 2 * t + (p4 >> 1);
            x1[t] = am_tr_read(a1 + ((c ^ sw1) * 16));
            x2[t] = am_tr_read(a2 + ((c ^ sw2) * 16));
        }
        // lane holds keys t0 + 16 kt + 4 g + r of its query column (mha_kernel.cpp:51-60: s = (q . k) * scale)
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
        const float mn = fmaxf(mx, cmax);  // finite: a live tile holds key t0 <= pos
        const float corr = expf(mx - mn);  // 0 on the first tile (mx = -inf)
        float pv[8], psum = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            pv[e] = expf(sv[e] - mn);  // 0 for masked keys
            psum += pv[e];
        }
        psum += __shfl_xor(psum, 16);
        psum += __shfl_xor(psum, 32);
        l = l * corr + psum;
        mx = mn;
        __half ph[8], pm[8], pl[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) am_split3(pv[e], ph[e], pm[e], pl[e]);
        const u32x4 pfh = *reinterpret_cast<const u32x4*>(ph);
        const u32x4 pfm = *reinterpret_cast<const u32x4*>(pm);
        const u32x4 pfl = *reinterpret_cast<const u32x4*>(pl);
        // the transposed reads landed. Their registers are named in the wait, so the compiler neither reads nor copies
        // them above it (an asm load's outputs count as written at its end: cdna_hip_programming.md "What hipcc does
        // not do" 1(ii); without this, copies into the MFMA operand raced the LDS returns under DMA load)
        if constexpr (NT == 8)
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(x1[0]), "+v"(x1[1]), "+v"(x1[2]), "+v"(x1[3]), "+v"(x1[4]), "+v"(x1[5]), "+v"(x1[6]),
                           "+v"(x1[7]), "+v"(x2[0]), "+v"(x2[1]), "+v"(x2[2]), "+v"(x2[3]), "+v"(x2[4]), "+v"(x2[5]),
                           "+v"(x2[6]), "+v"(x2[7])
                         :
                         : "memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(x1[0]), "+v"(x1[1]), "+v"(x1[2]), "+v"(x1[3]), "+v"(x2[0]), "+v"(x2[1]), "+v"(x2[2]),
                           "+v"(x2[3])
                         :
                         : "memory");
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            o[t] *= corr;
            const u32x4 vf = u32x4{x1[t].x, x1[t].y, x2[t].x, x2[t].y};
            o[t] = am_mfma(vf, pfh, o[t]);
            o[t] = am_mfma(vf, pfm, o[t]);
            o[t] = am_mfma(vf, pfl, o[t]);
        }
        // the slot's LDS reads are done (lgkmcnt(0) above): refill it with tile j + NBUF
        if (j + NBUF < nl) issue(j + NBUF);
    }
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memrealtime();

    // merge the 4 waves: each publishes (mx, l, o) into its own (drained) image, then wave w merges 16-d tiles
    // t = w, w + 4, ... (dead waves: mx = -inf, l = 0, o = 0)
    float* fo = reinterpret_cast<float*>(wimg);  // [NT][64 lanes][4]
    float* fml = fo + NT * 64 * 4;               // [64] mx, then [64] l
#pragma unroll
    for (int t = 0; t < NT; ++t) *reinterpret_cast<am_float4*>(fo + (t * 64 + lane) * 4) = o[t];
    fml[lane] = mx;
    fml[64 + lane] = l;
    __syncthreads();
    float m4[kAmWaves], w4[kAmWaves], M = -INFINITY;
#pragma unroll
    for (int w = 0; w < kAmWaves; ++w) {
        m4[w] = reinterpret_cast<const float*>(sm + w * WB)[NT * 256 + lane];
        M = fmaxf(M, m4[w]);
    }
    float L = 0.0f;
#pragma unroll
    for (int w = 0; w < kAmWaves; ++w) {
        w4[w] = m4[w] == -INFINITY ? 0.0f : expf(m4[w] - M);
        L = fmaf(w4[w], reinterpret_cast<const float*>(sm + w * WB)[NT * 256 + 64 + lane], L);
    }
    const bool publish = a.defer_merge == 0;
    for (int t = wave; t < NT; t += kAmWaves) {
        am_float4 acc = am_float4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int w = 0; w < kAmWaves; ++w)
            acc += *reinterpret_cast<const am_float4*>(reinterpret_cast<const float*>(sm + w * WB) + (t * 64 + lane) * 4) *
                   w4[w];
        if (i16 < G) {  // lane holds d = 16 t + 4 g + r of q head kvh * G + i16
            const size_t row = ((size_t)(kvh * G + i16) * a.max_splits + wgs) * (HD + kAttnPartPad);
            if (publish) {  // write-through (sc1, 16- and 8-byte stores) for the head's last-arriving workgroup
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.part + row, 0, 4u * (HD + kAttnPartPad), 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(
                    u32x4{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])},
                    rs, 4u * (t * 16 + 4 * g), 0, 16 /* sc1 */);
                if (t == 0 && g == 0)
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(M), __float_as_uint(L)}, rs, 4u * HD, 0, 16);
            } else {
                float* dst = a.part + row;
                *reinterpret_cast<float4*>(dst + t * 16 + 4 * g) = float4{acc[0], acc[1], acc[2], acc[3]};
                if (t == 0 && g == 0) {
                    dst[HD] = M;
                    dst[HD + 1] = L;
                }
            }
        }
    }
    if (!publish) return;  // partials for the next launch (the kernel boundary publishes them)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the arrival
    __syncthreads();
    const int ns = min(pos / ppwg + 1, a.max_splits);  // live workgroups of this kv head
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.counters + kvh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (unsigned)(ns - 1);
        if (last) __hip_atomic_store(a.counters + kvh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (last) {
        if (ns <= 4)
            am_merge<HD, G, 2>(a.part, a.out, kvh, a.max_splits, ns);
        else if (ns <= 8)
            am_merge<HD, G, 4>(a.part, a.out, kvh, a.max_splits, ns);
        else if (ns <= 16)
            am_merge<HD, G, 8>(a.part, a.out, kvh, a.max_splits, ns);
        else
            am_merge<HD, G, 16>(a.part, a.out, kvh, a.max_splits, ns);
        if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
}

// Tiles per wave for a launch over n_kv kv heads (every sequence's) of a T-position cache: one workgroup per CU
// over the whole context where the cache is long enough, at least one tile per wave, and at most kAmMaxSplits
// splits per kv head: the last arriver's merge grows with the split count (its arrivals serialise on one counter),
// 6.6 us at 32 splits against 3.7 at 16 — C4's TP-8 shard (8 kv heads, ctx 4096) at 16 splits on 128 workgroups
// takes 11.9 us instead of 13.3 on 256 (tools/attn_mfma_lab, profiles/r5_attn_mfma_tpw.txt).
constexpr int kAmMaxSplits = 16;
inline int attn_mfma_tpw(int n_kv, int T, int cus) {
    const long long keys = (long long)n_kv * T;
    const long long per = (keys + cus - 1) / cus;  // keys per CU
    int tpw = (int)((per + kAmWgKeys / 2) / kAmWgKeys);
    tpw = std::max(tpw, (T + kAmWgKeys * kAmMaxSplits - 1) / (kAmWgKeys * kAmMaxSplits));
    return tpw < 1 ? 1 : tpw > 64 ? 64 : tpw;
}

}  // namespace sli
