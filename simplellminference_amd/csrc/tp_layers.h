// tp_layers.h — a tensor-parallel rank's whole layer stack as ONE persistent launch (batch 1, fp16 weights and K/V,
// head_dim 128): LlamaModel::forward's layer loop (source/model/model.cpp:50-129) for the shard a rank holds
// (DESIGN.md §6), with every dependency edge inside the launch.
//
// Why at TP 4 / 8 and not at TP 1: a TP-8 rank's layer streams only ~55 MB
// (q/k/v 12.6, K/V 4.2, wo 4.2, gate/up 22.5, down 11.3), i.e. 16-88 KB per CU and op, yet the launch graph spends
// ~40 us on it: five launches each paying the boundary, the weight-stream ramp and the input staging. Here a CU
// issues the next op's weight share into registers BEFORE that op's input edge, so when the input arrives the op is
// a few register FMAs; what is left per op is the edge itself. tools/edge_chain_lab measured the five edges of a
// layer at 14.9 us, 19.3 us with the weight shares in flight (profiles/r6_edge_chain_lab.txt).
//
// Structure: one 512-thread workgroup per CU (nwg of them, all resident), every workgroup runs every op on its
// share. Edges are 8-byte {value, tag} granules (one sc1 store each, no drain, no flag; consumers sweep them with
// sc1 loads and re-read the ones whose tag is not yet this edge's: MI355X_MICROARCH.md "handoff-1to1",
// "allgather"). Tags are unique per (launch epoch, layer, edge), so one granule array per edge serves every layer:
// each edge is all-to-all, so no value is overwritten before every reader of the previous one has moved on.
//   E1  x (D)                    -> every workgroup: RMSNorm + q/k/v (layer 0 reads the embedding's x directly)
//   E2  q, k, v rows              -> the attention items (kv head, split of kTlKS keys)
//   E3  split partials (o, m, l)  -> the kv head's merging workgroup;  merged output (hq hd) -> every workgroup: wo
//   X   wo rows (+ residual)      -> exchange over the ranks per workgroup (the rows of x this workgroup owns)
//   E4  x1 (D)                    -> every workgroup: RMSNorm + gate/up + SwiGLU
//   E5  act (Il)                  -> every workgroup: down
//   X   down rows (+ x1)          -> exchange; then E1 of the next layer (the last layer stores x plainly)
// The exchange (mode 2) pushes each row's value as a granule into slot [rank] of every rank's comm buffer (uncached,
// IPC-mapped: oneshot.h) and sums its own rows' slots in rank order — the per-workgroup exchange of oneshot.h with
// the flags replaced by tags. Every wait is bounded: a wait that gives up sets DevState::error kTlErrWait and the
// workgroup skips every later wait, so the grid drains.
#pragma once
#include "common.h"
#include "step_state.h"

namespace sli {

constexpr int kTlThreads = 512;                 // 8 waves; one workgroup per CU
constexpr int kTlWaves = kTlThreads / 64;
constexpr int kTlCHQ = 6, kTlCHO = 4, kTlCHG = 12, kTlCHD = 6;  // 16-byte weight vectors per thread in one register
                                                                 // chunk: q/k/v, wo, gate/up, down (a TP-8 shard's share)
constexpr int kTlHD = 128;                      // head_dim
constexpr int kTlKS = 128;                      // keys per attention split: K and V are 8 vectors per thread
constexpr int kTlMaxG = 4;                      // q heads per kv head
constexpr int kTlMaxX = 8192;                   // LDS input vector (D, hq hd, Il)
constexpr int kTlMaxD = 4096;                   // model width (the norm weights a thread needs sit in 8 registers)
constexpr int kTlPartMax = 12288;               // per-(row, 8-column group) partial sums of one op in LDS
constexpr int kTlMaxRows = 256;                 // rows of x a workgroup owns (D / nwg)
constexpr int kTlMaxSplits = 64;                // T <= 8192
constexpr int kTlPart = kTlHD + 2;              // granules per split partial: o[hd], m, l
constexpr int kTlErrWait = 32;                  // DevState::error bit (oneshot.h 4, attention.h 8)
constexpr unsigned kTlSpin = 1u << 20;          // sweep passes of one wait before it gives up

typedef unsigned tl_u2 __attribute__((ext_vector_type(2)));

// threadIdx.x behind an empty asm: every per-thread offset is the same in every layer, and hoisted out of the layer
// loop the compiler kept them all live for the whole launch (256 VGPRs and 500+ bytes of scratch per lane); computed
// from this, they are recomputed where used
__device__ __forceinline__ int tl_tid() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

struct TlArgs {
    int D, hq, hkv, Il, L, T, nwg, act_mode;
    float eps, scale;
    const __half* const* w;   // [L][4] device table: qkv [(hq + 2 hkv) hd][D], wo [D][hq hd], gu [2 Il][D], down [D][Il]
    const float* norms;       // [2L + 1][D] (model.cpp:360-364 order)
    __half *kc, *vc;          // [L][hkv][T][hd]
    const float *sin_t, *cos_t;  // [T][hd / 2]
    DevState* st;
    float* x;                 // the residual stream: layer 0's input (the embedding's) and the last layer's output
    tl_u2 *g_x, *g_qkv, *g_part, *g_att, *g_x1, *g_act;  // granule arrays (zeroed once at creation)
    unsigned* epoch;          // launch counter: tags of launch e are (e L + layer) 8 + edge
    // residual exchange after wo and down: 0 one rank (x += projection); 1 debug no-comm (x = this rank's partial,
    // the residual added on rank 0, as the launch path's device copy); 2 granule exchange over xg
    int mode, rank, nranks, loopback;
    tl_u2* const* xg;         // [nranks] device table: every rank's exchange granules [2][kOsMaxRanks][D], mapped here
    unsigned long long* stamps = nullptr;  // tools/tl_lab (TL_STAMPS builds): [nwg][L][kTlStamps] s_memrealtime
};
constexpr int kTlStamps = 20;
#ifdef TL_STAMPS
#define TL_STAMPL(lay, k) \
    if (a.stamps && threadIdx.x == 0) a.stamps[((size_t)blockIdx.x * a.L + (lay)) * kTlStamps + (k)] = __builtin_amdgcn_s_memrealtime()
#define TL_STAMP(k) \
    if (a.stamps && threadIdx.x == 0) a.stamps[((size_t)blockIdx.x * a.L + l) * kTlStamps + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define TL_STAMPL(lay, k)
#define TL_STAMP(k)
#endif

struct TlSmem {
    float xs[kTlMaxX];        // the op's input vector (normalised for q/k/v and gate/up)
    float part[kTlPartMax];   // GEMV partial sums; the attention's wave partials and the merge's split partials
    float rows[kTlMaxRows];   // the op's row sums (<= 256 rows per workgroup per op at the supported shapes)
    float xres[kTlMaxRows];   // the residual rows this workgroup owns (x, then x1)
    float qv[(kTlMaxG + 2) * kTlHD];  // the kv head's G q rows, then (the split holding pos) this step's K and V rows
    float red[2 * kTlWaves * kTlMaxG + 8];
    unsigned vote[2][kTlWaves];  // tl_any: one flag per wave, double-buffered by call parity
    float vsum[2][kTlWaves];     // tl_any: one partial sum per wave beside its flag (the gathers' sums of squares)
    int dead;
};

// a pointer read from device memory, declared uniform: a buffer resource built from a VGPR pointer makes the compiler
// wrap every load in a waterfall loop (readfirstlane, compare, branch per load)
template <class T>
__device__ __forceinline__ T* tl_uniform(T* p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (T*)(((unsigned long long)hi << 32) | lo);
}

// ---------------------------------------------------------------- granules
__device__ __forceinline__ void tl_put(tl_u2* g, int i, float v, unsigned tag) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(tl_u2{__float_as_uint(v), tag}, rs, 8u * (unsigned)i, 0, 16 /* sc1 */);
}

// block-wide OR with ONE barrier (__syncthreads_or costs three): each wave's ballot, one flag per wave in LDS, read by
// all. The flags alternate between two slots by call parity: a wave writing call k + 2's flags has passed call k + 1's
// barrier, which every wave reaches only after reading call k's.
template <bool SUM = false>
__device__ __forceinline__ bool tl_any(TlSmem& sm, unsigned& vp, bool v, float* sum = nullptr) {
    const unsigned par = vp & 1u;
    ++vp;
    const bool w = __ballot(v) != 0;
    float ws = 0.0f;
    if constexpr (SUM) ws = wave_sum(*sum);
    if ((tl_tid() & 63) == 0) {
        sm.vote[par][tl_tid() >> 6] = w ? 1u : 0u;
        if constexpr (SUM) sm.vsum[par][tl_tid() >> 6] = ws;
    }
    __syncthreads();
    const uint4 f0 = *reinterpret_cast<const uint4*>(&sm.vote[par][0]);
    const uint4 f1 = *reinterpret_cast<const uint4*>(&sm.vote[par][4]);
    if constexpr (SUM) {
        const float4 s0 = *reinterpret_cast<const float4*>(&sm.vsum[par][0]);
        const float4 s1 = *reinterpret_cast<const float4*>(&sm.vsum[par][4]);
        *sum = ((((((s0.x + s0.y) + s0.z) + s0.w) + s1.x) + s1.y) + s1.z) + s1.w;
    }
    return (f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w) != 0;
}

// the bounded-wait give-up of every gather, checked every 1024 passes: true once this one has swept kTlSpin times, or
// another workgroup (or rank) gave up already; then the workgroup skips every later wait and the grid drains
__device__ __forceinline__ bool tl_give_up(TlSmem& sm, unsigned& vp, DevState* st, unsigned pass) {
    if ((pass & 1023u) != 1023u) {
        __builtin_amdgcn_s_sleep(1);
        return false;
    }
    bool give_up = pass >= kTlSpin;
    if (tl_tid() == 0)
        give_up = give_up || (__hip_atomic_load(&st->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & kTlErrWait) != 0;
    if (tl_any(sm, vp, give_up)) {
        if (tl_tid() == 0) {
            __hip_atomic_fetch_or(&st->error, kTlErrWait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            sm.dead = 1;
        }
        __syncthreads();
        return true;
    }
    return false;
}

// n granules g[0 .. n) carrying `tag` into dst[0 .. n) (LDS), all threads, up to 8 per thread per sweep. Branch-free
// sweep (instruction count is what a persistent layer pays for, tools/tl_lab): every pass loads all of the thread's
// granules (indices past n clamped to n - 1) and stores every value; a value stored before its tag arrived is
// overwritten by a later pass, and the loop ends on the pass where every tag matched. (A tag never moves past this
// edge's while the gather runs: its producers' next write needs this workgroup's later output.) The last tl_any's
// barrier publishes dst.
template <bool SS = false>
__device__ __forceinline__ void tl_gather(TlSmem& sm, unsigned& vp, const tl_u2* g, int n, unsigned tag, float* dst, DevState* st,
                                          float* ss = nullptr) {
    if (sm.dead) return;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<tl_u2*>(g), 0, 0x7fffffff, 0x00020000);
    constexpr int kPer = 8;
    const int tid = tl_tid();
    for (int b0 = 0; b0 < n; b0 += kPer * kTlThreads) {
        unsigned off[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) off[j] = (unsigned)min(b0 + tid + j * kTlThreads, n - 1);
        for (unsigned pass = 0;; ++pass) {
            tl_u2 v[kPer];
#pragma unroll
            for (int j = 0; j < kPer; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b64(rs, 8u * off[j], 0, 16 /* sc1 */);
            bool miss = false;
            float sq = 0.0f;  // (SS: RMSNorm's sum of squares of this pass's values; the last pass's is the one kept)
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
                miss |= v[j].y != tag;
                const float x = __uint_as_float(v[j].x);
                dst[off[j]] = x;
                if constexpr (SS) sq += b0 + tid + j * kTlThreads < n ? x * x : 0.0f;
            }
            if constexpr (SS) {
                if (!tl_any<true>(sm, vp, miss, &sq)) {
                    *ss += sq;
                    break;
                }
            } else {
                if (!tl_any(sm, vp, miss)) break;
            }
            if (tl_give_up(sm, vp, st, pass)) return;
        }
    }
}

// two granule sets in one sweep: n1 contiguous from g1, then n2 from g2 (blocks of inner, stride apart), into dst;
// n1 + n2 <= 2 * kTlThreads; branch-free like tl_gather (offsets computed once per call)
__device__ __forceinline__ void tl_gather2(TlSmem& sm, unsigned& vp, const tl_u2* g1, int n1, const tl_u2* g2, int n2, int inner,
                                           int stride, unsigned tag, float* dst, DevState* st) {
    if (sm.dead) return;
    const int n = n1 + n2;
    if (n <= 0) return;
    const auto r1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<tl_u2*>(g1 ? g1 : g2), 0, 0x7fffffff, 0x00020000);
    const auto r2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<tl_u2*>(g2), 0, 0x7fffffff, 0x00020000);
    const int tid = tl_tid();
    int idx[2];
    unsigned off[2];
    bool first[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        idx[j] = min(tid + j * kTlThreads, n - 1);
        first[j] = idx[j] < n1;
        const int k = idx[j] - n1, o = first[j] ? 0 : k / inner;
        off[j] = 8u * (unsigned)(first[j] ? idx[j] : o * stride + (k - o * inner));
    }
    for (unsigned pass = 0;; ++pass) {
        tl_u2 v[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
            v[j] = first[j] ? __builtin_amdgcn_raw_buffer_load_b64(r1, off[j], 0, 16 /* sc1 */)
                            : __builtin_amdgcn_raw_buffer_load_b64(r2, off[j], 0, 16);
        bool miss = false;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            miss |= v[j].y != tag;
            dst[idx[j]] = __uint_as_float(v[j].x);
        }
        if (!tl_any(sm, vp, miss)) break;
        if (tl_give_up(sm, vp, st, pass)) return;
    }
}

// ---------------------------------------------------------------- register-chunk GEMV over LDS-staged input
// An op's rows on this workgroup: nr rows of K columns (K % 8 == 0), row(i) their matrix rows. Vector v of the
// flat (row, 8-column group) sequence: row v / G, group v % G (G = K / 8); thread t holds v = (c kTlCH + j) 512 + t
// of register chunk c. Chunk 0 is issued before the op's input edge (its bytes land while the edge is pending).
template <int CH>
struct TlChunk {
    u32x4 w[CH];
};

// (row, group) of vector v0 = (chunk CH) 512 + tid, then of v0 + 512 j, j < CH, by increments (no division per vector:
// the kernel's loop body has to fit the instruction cache)
struct TlVec {
    int r, g;
};
__device__ __forceinline__ TlVec tl_vec0(int G, int chunk, int CH) {
    const int v = chunk * CH * kTlThreads + tl_tid();
    const int r = v / G;
    return {r, v - r * G};
}
__device__ __forceinline__ void tl_vec_next(TlVec& p, int G, int q512, int r512) {
    p.g += r512;
    p.r += q512;
    if (p.g >= G) {
        p.g -= G;
        p.r += 1;
    }
}

// FIXED: K / 8 divides the 512 threads (K a power of two <= 4096: q/k/v, wo and gate/up at the supported shapes), so a
// thread's column group is fixed and the row advances by a constant; otherwise (down: K = the local FFN width) the
// (row, group) pair is stepped incrementally
template <int CH, bool FIXED, class RowF>
__device__ __forceinline__ void tl_issue(TlChunk<CH>& c, const __half* W, int K, int nr, const RowF& row, int chunk) {
    const int G = K >> 3;
    if (nr <= 0) return;
    // 32-bit byte offsets into the matrix (a shard matrix is < 4 GiB): one buffer resource, no 64-bit address math
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<__half*>(W), 0, 0x7fffffff, 0x00020000);
    const int tid = tl_tid();
    if constexpr (FIXED) {
        const int per = kTlThreads / G, g = tid % G, r0 = chunk * CH * per + tid / G;
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const int r = min(r0 + j * per, nr - 1);  // clamped: a duplicate of a vector in flight, never a branch
            c.w[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, 2u * ((unsigned)row(r) * (unsigned)K + 8u * (unsigned)g), 0,
                                                           2 /* nt: streamed once */);
        }
    } else {
    const int q512 = kTlThreads / G, r512 = kTlThreads - q512 * G;
    TlVec p = tl_vec0(G, chunk, CH);
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const bool in = p.r < nr;
        const unsigned off = 2u * ((unsigned)row(in ? p.r : nr - 1) * (unsigned)K + 8u * (unsigned)(in ? p.g : G - 1));
        c.w[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2);
        tl_vec_next(p, G, q512, r512);
    }
    }
}

__device__ __forceinline__ float tl_dot8(const u32x4& w, const float* x) {  // x: 8 floats (LDS or registers)
    const float4 x0 = *reinterpret_cast<const float4*>(x);
    const float4 x1 = *reinterpret_cast<const float4*>(x + 4);
    const __half2* h = reinterpret_cast<const __half2*>(&w);
    const float2 a = __half22float2(h[0]), b = __half22float2(h[1]), e = __half22float2(h[2]), f = __half22float2(h[3]);
    float s = a.x * x0.x;
    s = fmaf(a.y, x0.y, s);
    s = fmaf(b.x, x0.z, s);
    s = fmaf(b.y, x0.w, s);
    s = fmaf(e.x, x1.x, s);
    s = fmaf(e.y, x1.y, s);
    s = fmaf(f.x, x1.z, s);
    s = fmaf(f.y, x1.w, s);
    return s;
}

template <int CH, bool FIXED>
__device__ __forceinline__ void tl_consume(const TlChunk<CH>& c, int K, int nr, const float* xs, float* part, int chunk,
                                           const float* nw) {
    const int G = K >> 3;
    const int tid = tl_tid();
    if constexpr (FIXED) {
        const int per = kTlThreads / G, g = tid % G, r0 = chunk * CH * per + tid / G;
        // the thread's 8 inputs, once (times their norm weights where the op is RMS-normalised: the row sums are scaled
        // by 1/rms afterwards)
        float xr[8];
        {
            const float4 x0 = *reinterpret_cast<const float4*>(xs + 8 * g), x1 = *reinterpret_cast<const float4*>(xs + 8 * g + 4);
            xr[0] = x0.x, xr[1] = x0.y, xr[2] = x0.z, xr[3] = x0.w, xr[4] = x1.x, xr[5] = x1.y, xr[6] = x1.z, xr[7] = x1.w;
            if (nw) {
#pragma unroll
                for (int e = 0; e < 8; ++e) xr[e] *= nw[e];
            }
        }
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            // clamped like the loads: a vector past the last is a duplicate of it, its dot the same value (no branch)
            const int r = min(r0 + j * per, nr - 1);
            part[r * G + g] = tl_dot8(c.w[j], xr);
        }
    } else {
        const int q512 = kTlThreads / G, r512 = kTlThreads - q512 * G;
        TlVec p = tl_vec0(G, chunk, CH);
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            if (p.r < nr) part[p.r * G + p.g] = tl_dot8(c.w[j], xs + 8 * p.g);
            tl_vec_next(p, G, q512, r512);
        }
    }
}

// the whole op: chunk 0 already issued into c (before the input edge); a larger share's later chunks follow one by
// one (one register set: the TP-4 / TP-8 shards are one chunk per op). Row sums into sm.rows[0 .. nr), each summed
// over its groups in group order by one wave (deterministic).
template <int CH, bool FIXED, class RowF>
__device__ __forceinline__ void tl_gemv(TlSmem& sm, TlChunk<CH>& c, const __half* W, int K, int nr, const RowF& row,
                                        const float* nw = nullptr, float scale = 1.0f) {
    const int G = K >> 3, nch = (nr * G + CH * kTlThreads - 1) / (CH * kTlThreads);
#pragma nounroll
    for (int ch = 0; ch < nch; ++ch) {
        if (ch > 0) tl_issue<CH, FIXED>(c, W, K, nr, row, ch);
        tl_consume<CH, FIXED>(c, K, nr, sm.xs, sm.part, ch, nw);
    }
    __syncthreads();
    const int lane = tl_tid() & 63, wave = tl_tid() >> 6;
    for (int i = wave; i < nr; i += kTlWaves) {
        float s = 0.0f;
        if (G <= 8 * 64) {  // (every op at the supported shapes) independent loads, no loop-carried branch
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int g = lane + 64 * k;
                const float v = sm.part[i * G + min(g, G - 1)];
                s += g < G ? v : 0.0f;
            }
        } else {
            for (int g = lane; g < G; g += 64) s += sm.part[i * G + g];
        }
        s = wave_sum(s);
        if (lane == 0) sm.rows[i] = s * scale;
    }
    __syncthreads();
}

// the norm weights a thread multiplies (w[t + 512 k], k < D / 512, D <= 4096): loaded before the input edge, so the
// RMSNorm after it pays no global round trip
struct TlNormW {
    float w[kTlMaxD / kTlThreads];  // the norm weights of the thread's 8 columns (its fixed group of the D-wide GEMV)
};
__device__ __forceinline__ void tl_issue_norm(TlNormW& n, const float* w, int D) {
    const int g = tl_tid() % (D >> 3);  // D / 8 divides 512 (tpl_check): the thread's column group of every D-wide GEMV
    const float4 a = *reinterpret_cast<const float4*>(w + 8 * g), b = *reinterpret_cast<const float4*>(w + 8 * g + 4);
    n.w[0] = a.x, n.w[1] = a.y, n.w[2] = a.z, n.w[3] = a.w, n.w[4] = b.x, n.w[5] = b.y, n.w[6] = b.z, n.w[7] = b.w;
}

// RMSNorm (rms_kernel.cpp:5-23: y = (x * 1/sqrt(mean(x^2) + eps)) * w) is folded into the D-wide GEMVs: the gather
// sums the squares, the consume multiplies each x by its column's norm weight (kept in registers) and the row sums
// are scaled by 1/rms, so the normalised vector is never written (one LDS pass and two barriers per norm fewer; the
// products round as inv * sum(W x w) instead of sum(W ((x inv) w)): within the parity bar, tests/test_gpu_tp_layers.py)
__device__ __forceinline__ float tl_rms_inv(float ss, int D, float eps) { return 1.0f / sqrtf(ss / (float)D + eps); }

// ---------------------------------------------------------------- residual exchange of this workgroup's rows
// val[i] (LDS sm.rows) = this rank's projection rows r0 + i; out: sm.xres[i] = the new residual rows. Region 0: wo,
// 1: down.
__device__ __forceinline__ void tl_exchange(TlSmem& sm, unsigned& vp, const TlArgs& a, int r0, int nrow, int region, unsigned tag) {
    const int t = tl_tid();
    if (a.mode == 0) {  // one rank: x += projection (EpiStore: resid + acc)
        if (t < nrow) sm.xres[t] = sm.xres[t] + sm.rows[t];
        __syncthreads();
        return;
    }
    // this rank's contribution: the partial, plus the residual on rank 0 (EpiPush / EpiStore under tp)
    const float v = t < nrow ? (a.rank == 0 ? sm.xres[t] + sm.rows[t] : sm.rows[t]) : 0.0f;
    if (a.mode == 1) {  // debug no-comm: the local partial stands in for the sum
        if (t < nrow) sm.xres[t] = v;
        __syncthreads();
        return;
    }
    const size_t D = (size_t)a.D;
    if (t < nrow) {
        for (int p = 0; p < a.nranks; ++p) {
            // slot [rank] of every rank's buffer; loopback (one process, every "peer" this rank): every slot of its own
            tl_u2* dst = a.loopback ? tl_uniform(a.xg[a.rank]) + ((size_t)region * 8 + p) * D
                                    : tl_uniform(a.xg[p]) + ((size_t)region * 8 + a.rank) * D;
            tl_put(dst, r0 + t, v, tag);
        }
        // (no wait for the pushes' acknowledgement before the first poll: the tags tell a value that has not landed,
        // and waiting cost 0.3 us per layer in tools/tl_lab)
    }
    // this workgroup's rows of every rank's slot in its own buffer, summed in rank order
    float* got = sm.part;  // [nranks][nrow], one sweep over every slot
    tl_gather2(sm, vp, nullptr, 0, tl_uniform(a.xg[a.rank]) + (size_t)region * 8 * D + r0, a.nranks * nrow, nrow, (int)D, tag,
               got, a.st);
    if (t < nrow) {
        float s = got[t];
        for (int p = 1; p < a.nranks; ++p) s += got[p * nrow + t];
        sm.xres[t] = s;
    }
    __syncthreads();
}

// ---------------------------------------------------------------- attention item (kv head, split of kTlKS keys)
// mha_kernel.cpp:36-77 for the G query heads of one kv head over keys [s KS, s KS + KS) of the live context, as
// flash-decoding partials (max m, sum l, unnormalised o) merged later (attention.h attn_merge's arithmetic). K and V
// of the split are in registers (issued before the q/k/v edge); the row at pos is this step's, from the E2 granules.
struct TlKV {
    u32x4 k[4], v[4];
};

__device__ __forceinline__ void tl_issue_kv(TlKV& r, const TlArgs& a, int l, int kvh, int s, int pos) {
    const int c = tl_tid() & 15;
    const size_t base = ((size_t)l * a.hkv + kvh) * a.T;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int key = min(s * kTlKS + (int)(tl_tid() >> 4) + 32 * j, pos);
        r.k[j] = load16<true>(a.kc + (base + key) * kTlHD + 8 * c);
        r.v[j] = load16<true>(a.vc + (base + key) * kTlHD + 8 * c);
    }
}

__device__ __forceinline__ u32x4 tl_pack8(const float* p) {
    __half h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = __float2half_rn(p[e]);
    return *reinterpret_cast<const u32x4*>(h);
}

template <int G>
__device__ __forceinline__ void tl_attend(TlSmem& sm, const TlArgs& a, TlKV& r, int kvh, int s, int S, int pos, unsigned tag,
                                          int lay) {
    const int t = tl_tid(), c = t & 15, lane = t & 63, wave = t >> 6;
    const int k0 = s * kTlKS;
    if (pos >= k0 && pos < k0 + kTlKS) {  // this step's row replaces the cache's (fp16, as the cache stores it)
        const int jj = pos - k0 - (t >> 4);
        const u32x4 kn = tl_pack8(sm.qv + G * kTlHD + 8 * c), vn = tl_pack8(sm.qv + (G + 1) * kTlHD + 8 * c);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // selects, not a conditional store (that became an indexed one: scratch)
            const bool hit = jj == 32 * j;
            r.k[j] = hit ? kn : r.k[j];
            r.v[j] = hit ? vn : r.v[j];
        }
    }
    float sc[4][G];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const __half2* kh = reinterpret_cast<const __half2*>(&r.k[j]);
        float kf[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float2 f = __half22float2(kh[e]);
            kf[2 * e] = f.x;
            kf[2 * e + 1] = f.y;
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float* q = sm.qv + g * kTlHD + 8 * c;
            float d = kf[0] * q[0];
#pragma unroll
            for (int e = 1; e < 8; ++e) d = fmaf(kf[e], q[e], d);
            d = group_sum<16>(d);  // the key's 16 lanes hold its 16 chunks
            const int key = k0 + (t >> 4) + 32 * j;
            sc[j][g] = key <= pos ? d * a.scale : -INFINITY;
        }
    }
    TL_STAMPL(lay, 16);
    // split max and sum per q head: a lane's 4 keys, the wave's 4 key groups (lanes 16 apart), then the 8 waves
    float mx[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float m = fmaxf(fmaxf(sc[0][g], sc[1][g]), fmaxf(sc[2][g], sc[3][g]));
        m = stride_max<16>(m);
        if (lane == 0) sm.red[wave * G + g] = m;
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float m = sm.red[g];
        for (int w = 1; w < kTlWaves; ++w) m = fmaxf(m, sm.red[w * G + g]);
        mx[g] = m;  // finite: key k0 <= pos is live
    }
    TL_STAMPL(lay, 17);
    float p[4][G], ls[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float sum = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            p[j][g] = expf(sc[j][g] - mx[g]);  // 0 for masked keys
            sum += p[j][g];
        }
        ls[g] = stride_sum<16>(sum);
    }
    // o partial for dims 8c .. 8c+7: the lane's 4 keys, then the wave's 4 key groups
    float* po = sm.part;  // [waves][G][hd]
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const __half2* vh = reinterpret_cast<const __half2*>(&r.v[j]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float2 f = __half22float2(vh[e]);
                o[2 * e] = fmaf(p[j][g], f.x, o[2 * e]);
                o[2 * e + 1] = fmaf(p[j][g], f.y, o[2 * e + 1]);
            }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = stride_sum<16>(o[e]);
        if (lane < 16) {
#pragma unroll
            for (int e = 0; e < 8; ++e) po[(wave * G + g) * kTlHD + 8 * c + e] = o[e];
        }
    }
    __syncthreads();  // (red[] of the max is read above; the l sums go to red[] below, after this barrier)
    TL_STAMPL(lay, 18);
    if (lane == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) sm.red[kTlWaves * kTlMaxG + wave * G + g] = ls[g];
    }
    __syncthreads();
    // publish (o, m, l) per q head: granules [(kvh G + g) S + s][kTlPart]
    for (int i = t; i < G * kTlPart; i += kTlThreads) {
        const int g = i / kTlPart, d = i - g * kTlPart;
        float v;
        if (d < kTlHD) {
            v = po[g * kTlHD + d];
            for (int w = 1; w < kTlWaves; ++w) v += po[(w * G + g) * kTlHD + d];
        } else if (d == kTlHD) {
            v = sm.red[g];  // the split max of q head g (every wave's lane 0 left it there; no register array indexed
                            // by a runtime g: that went to scratch)
            for (int w2 = 1; w2 < kTlWaves; ++w2) v = fmaxf(v, sm.red[w2 * G + g]);
        } else {
            v = sm.red[kTlWaves * kTlMaxG + g];
            for (int w = 1; w < kTlWaves; ++w) v += sm.red[kTlWaves * kTlMaxG + w * G + g];
        }
        tl_put(a.g_part, ((kvh * G + g) * S + s) * kTlPart + d, v, tag);
    }
    __syncthreads();
}

// the kv head's merge: ns live splits per q head -> attention output rows (attention.h attn_merge: M = max m_s,
// w_s = e^{m_s - M}, out = sum w_s o_s / sum w_s l_s, in split order)
template <int G>
__device__ __forceinline__ void tl_merge(TlSmem& sm, unsigned& vp, const TlArgs& a, int kvh, int S, int ns, unsigned tag_in, unsigned tag_out,
                                         int lay) {
    for (int g = 0; g < G; ++g) {
        const int h = kvh * G + g;
        tl_gather(sm, vp, a.g_part + (size_t)h * S * kTlPart, ns * kTlPart, tag_in, sm.part, a.st);
#ifdef TL_STAMPS
        if (a.stamps && threadIdx.x == 0) a.stamps[((size_t)blockIdx.x * a.L + lay) * kTlStamps + 12] = __builtin_amdgcn_s_memrealtime();
#endif
        // 512 threads: dim d = t & 127, quarter q = t >> 7 takes splits q, q + 4, ...; M over every split (independent
        // broadcast reads), the quarters' sums combined in quarter order (deterministic)
        const int t = tl_tid(), d = t & (kTlHD - 1), q = t >> 7;
        float M = -INFINITY;
        for (int s2 = 0; s2 < ns; ++s2) M = fmaxf(M, sm.part[s2 * kTlPart + kTlHD]);
        float num = 0.0f, den = 0.0f;
        for (int s2 = q; s2 < ns; s2 += kTlThreads / kTlHD) {
            const float w = expf(sm.part[s2 * kTlPart + kTlHD] - M);
            num = fmaf(w, sm.part[s2 * kTlPart + d], num);
            den = fmaf(w, sm.part[s2 * kTlPart + kTlHD + 1], den);
        }
        float* qs = sm.part + kTlMaxSplits * kTlPart;  // [4][hd] numerators, then [4][hd] denominators
        qs[q * kTlHD + d] = num;
        qs[(kTlThreads / kTlHD + q) * kTlHD + d] = den;
        __syncthreads();
        if (t < kTlHD) {
            float n2 = qs[d], d2 = qs[4 * kTlHD + d];
#pragma unroll
            for (int k = 1; k < kTlThreads / kTlHD; ++k) {
                n2 += qs[k * kTlHD + d];
                d2 += qs[(4 + k) * kTlHD + d];
            }
            tl_put(a.g_att, h * kTlHD + d, n2 / d2, tag_out);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- the layer stack
template <int G>
__global__ void __launch_bounds__(kTlThreads) tp_layers_kernel(TlArgs a) {
    __shared__ TlSmem sm;
    const int t = threadIdx.x, w = blockIdx.x, nwg = a.nwg;
    if (t == 0) sm.dead = 0;
    unsigned vp = 0;  // tl_any's call parity (every thread makes the same calls)
    const int pos = a.st->pos;
    const unsigned E = *a.epoch + 1u;
    __syncthreads();
    const int D = a.D, hq = a.hq, hkv = a.hkv, Il = a.Il, T = a.T, L = a.L;
    const int S = (T + kTlKS - 1) / kTlKS, ns = pos / kTlKS + 1;
    const int n_items = hkv * S;
    // this workgroup's rows: x rows [r0, r1) (wo, down, exchange); q/k/v units (2 rows: RoPE pair); gate/up units
    const int r0 = (int)((long long)D * w / nwg), nrow = (int)((long long)D * (w + 1) / nwg) - r0;
    const int Uq = (hq + 2 * hkv) * (kTlHD / 2);
    const int q0 = (int)((long long)Uq * w / nwg), nq = (int)((long long)Uq * (w + 1) / nwg) - q0;
    const int g0 = (int)((long long)Il * w / nwg), ng = (int)((long long)Il * (w + 1) / nwg) - g0;
    auto row_qkv = [&](int i) {
        const int u = q0 + (i >> 1), uh = u / (kTlHD / 2), d = u - uh * (kTlHD / 2);
        return uh * kTlHD + d + (i & 1) * (kTlHD / 2);
    };
    auto row_gu = [&](int i) { return (i & 1) * Il + g0 + (i >> 1); };
    auto row_x = [&](int i) { return r0 + i; };

    for (int l = 0; l < L; ++l) {
        const unsigned tb = (E * (unsigned)L + (unsigned)l) * 8u;
        const __half* W[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) W[k] = tl_uniform(a.w[4 * l + k]);
        // ---- E1 -> RMSNorm -> q/k/v (+ RoPE, K/V cache rows)
        TlChunk<kTlCHQ> c;
        tl_issue<kTlCHQ, true>(c, W[0], D, 2 * nq, row_qkv, 0);
        TlNormW nw;
        tl_issue_norm(nw, a.norms + (size_t)(2 * l) * D, D);
        float rsin = 0.0f, rcos = 1.0f;  // this thread's q/k/v unit's RoPE table entries (rope_kernel.cpp:30-38)
        if (t < nq) {
            const int u = q0 + t, d = u % (kTlHD / 2);
            rsin = a.sin_t[pos * (kTlHD / 2) + d];
            rcos = a.cos_t[pos * (kTlHD / 2) + d];
        }
        TlKV kv;
        const bool attn_item = w < n_items && (w % S) < ns;  // (first item only in registers early)
        if (attn_item) tl_issue_kv(kv, a, l, w / S, w % S, pos);  // (after E1 instead: +0.2-0.5 us per layer)
        float ss = 0.0f;  // sum of squares of x (RMSNorm)
        if (l == 0) {  // the embedding's x, written before this launch
            float sq = 0.0f;
            for (int i = t; i < D; i += kTlThreads) {
                const float v = a.x[i];
                sm.xs[i] = v;
                sq += v * v;
            }
            tl_any<true>(sm, vp, false, &sq);  // (the block sum; its barrier publishes xs)
            ss = sq;
        } else {
            tl_gather<true>(sm, vp, a.g_x, D, tb + 1, sm.xs, a.st, &ss);
        }
        TL_STAMP(0);
        if (t < nrow) sm.xres[t] = sm.xs[r0 + t];
        TL_STAMP(14);
        tl_gemv<kTlCHQ, true>(sm, c, W[0], D, 2 * nq, row_qkv, nw.w, tl_rms_inv(ss, D, a.eps));
        TL_STAMP(15);
        if (t < nq) {  // EpiQKV (rope_kernel.cpp:30-38)
            const int u = q0 + t, uh = u / (kTlHD / 2), d = u - uh * (kTlHD / 2);
            float r0v = sm.rows[2 * t], r1v = sm.rows[2 * t + 1];
            if (uh < hq + hkv) {
                const float fci = rsin, fcr = rcos;
                const float x0 = r0v * fcr - r1v * fci, x1 = r1v * fcr + r0v * fci;
                r0v = x0;
                r1v = x1;
            }
            if (uh >= hq) {  // k or v: this step's cache row
                const bool isk = uh < hq + hkv;
                __half* cache = (isk ? a.kc : a.vc) +
                                (((size_t)l * hkv + (isk ? uh - hq : uh - hq - hkv)) * T + pos) * kTlHD;
                cache[d] = __float2half_rn(r0v);
                cache[d + kTlHD / 2] = __float2half_rn(r1v);
            }
            tl_put(a.g_qkv, uh * kTlHD + d, r0v, tb + 2);
            tl_put(a.g_qkv, uh * kTlHD + d + kTlHD / 2, r1v, tb + 2);
        }
        TL_STAMP(1);
        // ---- attention items, then the merges of the kv heads whose split 0 this workgroup holds
        for (int it = w; it < n_items; it += nwg) {
            const int kvh = it / S, s = it - kvh * S;
            if (s >= ns) continue;
            if (it != w) tl_issue_kv(kv, a, l, kvh, s, pos);
            const bool own_row = pos >= s * kTlKS && pos < s * kTlKS + kTlKS;  // this split holds this step's K / V
            // the G q rows, then (the split holding pos) k and v, hkv * hd apart: one sweep
            tl_gather2(sm, vp, a.g_qkv + (size_t)kvh * G * kTlHD, G * kTlHD, a.g_qkv + (size_t)(hq + kvh) * kTlHD,
                       own_row ? 2 * kTlHD : 0, kTlHD, hkv * kTlHD, tb + 2, sm.qv, a.st);
            TL_STAMP(10);
            tl_attend<G>(sm, a, kv, kvh, s, S, pos, tb + 3, l);
            TL_STAMP(11);
        }
        // (merging in every workgroup instead, no merge edge: +1.3 us per layer, profiles/r6_tl_lab_ab_merge.txt)
        for (int it = w; it < n_items; it += nwg)
            if (it % S == 0) tl_merge<G>(sm, vp, a, it / S, S, ns, tb + 3, tb + 4, l);
        TL_STAMP(2);
        // ---- wo (+ residual, exchange)
        TlChunk<kTlCHO> co;
        tl_issue<kTlCHO, true>(co, W[1], hq * kTlHD, nrow, row_x, 0);
        tl_gather(sm, vp, a.g_att, hq * kTlHD, tb + 4, sm.xs, a.st);
        TL_STAMP(3);
        tl_gemv<kTlCHO, true>(sm, co, W[1], hq * kTlHD, nrow, row_x);
        TL_STAMP(4);
        tl_exchange(sm, vp, a, r0, nrow, 0, tb + 7);
        if (t < nrow) tl_put(a.g_x1, r0 + t, sm.xres[t], tb + 5);
        // ---- E4 -> RMSNorm -> gate/up -> SwiGLU (swiglu_kernel.cpp:12-13: sigmoid(gate) * up; act_mode 1: SiLU)
        // (issued after the exchange and the x1 publish, never before: a store queued behind a CU's 88 KB weight share
        // reaches its readers that much later — 1.3-1.6 us per layer in tools/tl_lab)
        TlChunk<kTlCHG> cg;
        tl_issue<kTlCHG, true>(cg, W[2], D, 2 * ng, row_gu, 0);  // (half of it after E4 instead: no change)
        tl_issue_norm(nw, a.norms + (size_t)(2 * l + 1) * D, D);
        float ss1 = 0.0f;
        tl_gather<true>(sm, vp, a.g_x1, D, tb + 5, sm.xs, a.st, &ss1);

        TL_STAMP(5);
        tl_gemv<kTlCHG, true>(sm, cg, W[2], D, 2 * ng, row_gu, nw.w, tl_rms_inv(ss1, D, a.eps));
        TL_STAMP(6);
        if (t < ng) {
            const float g = sm.rows[2 * t], up = sm.rows[2 * t + 1];
            float s = 1.0f / (1.0f + expf(-g));
            if (a.act_mode) s = g * s;
            tl_put(a.g_act, g0 + t, s * up, tb + 6);
        }
        // ---- E5 -> down (+ residual x1, exchange) -> the next layer's x
        TlChunk<kTlCHD> cd;
        tl_issue<kTlCHD, false>(cd, W[3], Il, nrow, row_x, 0);
        tl_gather(sm, vp, a.g_act, Il, tb + 6, sm.xs, a.st);
        TL_STAMP(7);
        tl_gemv<kTlCHD, false>(sm, cd, W[3], Il, nrow, row_x);
        TL_STAMP(8);
        tl_exchange(sm, vp, a, r0, nrow, 1, tb + 0);
        TL_STAMP(9);
        if (t < nrow) {
            if (l + 1 < L)
                tl_put(a.g_x, r0 + t, sm.xres[t], (E * (unsigned)L + (unsigned)(l + 1)) * 8u + 1u);
            else
                a.x[r0 + t] = sm.xres[t];
        }
        __syncthreads();
    }
    // the next launch's epoch: workgroup 0 ends only after every workgroup has contributed to its last gather, so
    // every workgroup has read this launch's epoch by then
    if (w == 0 && t == 0) *a.epoch = E;
}

}  // namespace sli
