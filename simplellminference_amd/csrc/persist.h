// persist.h — the whole batch-1 decode step (LlamaModel::forward, source/model/model.cpp:40-140, and
// the argmax + state update of predict, :157-183) as ONE persistent launch: one 1024-thread workgroup
// per CU runs every phase of every layer, separated by grid barriers instead of kernel boundaries.
//
// Why: at batch 1 every phase streams its weights once from HBM, and what a kernel
// boundary costs is the HBM stream going idle — the next kernel's loads start only after the previous
// kernel has drained. Here the next phase's first two weight chunks (and the attention's whole K/V
// slice) are issued BEFORE the grid barrier that guards the phase's input, so the stream keeps running
// while the barrier and the input hand-off complete (MI355X_MICROARCH.md price list,
// **prefetch-credit**, **engine-vs-launches**).
//
// Roles inside a workgroup: wave 0 is the control wave — it polls the grid barrier and stages the phase's
// input vector into LDS (RMS-normalised where the reference normalises); it never holds prefetched
// weights, so its poll is not queued behind them (s_waitcnt vmcnt counts in issue order). Waves 1..15
// stream weights (and the K/V slices) and run the epilogues.
//
// Hand-offs between workgroups (MI355X_MICROARCH.md "Valid forms", table row 1; cdna_hip_programming.md
// Guideline 16): every handed-off word is stored write-through (sc1) and drained (s_waitcnt vmcnt(0)) by
// every storing wave before the workgroup barrier that precedes ONE lane's agent-scope arrival add, and
// every load of it is an sc1 load issued after the consumer's poll matched. Every hand-off buffer is
// written at most once per launch (one x per half-layer, one q / new K/V row / attention output / act per
// layer), so no L2 can hold a stale copy of a line that a later phase of the same launch rewrites. The
// grid-barrier and per-head merge counters are zeroed by a memset node before every launch; every spin
// is bounded and gives up with DevState::error bit kPsErrTimeout.
#pragma once
#include "attention.h"
#include "common.h"
#include "gemv.h"
#include "step_state.h"

namespace sli {

constexpr int kPsThreads = 1024;
constexpr int kPsWaves = kPsThreads / 64;  // 16
constexpr int kPsCW = kPsWaves - 1;        // compute waves (1 .. 15)
constexpr int kPsAbortSlot = 63;           // LDS word (in the reduction scratch): a barrier spin gave up
constexpr unsigned kPsSpinLimit = 1u << 22;
constexpr int kPsErrTimeout = 2;           // DevState::error bit
constexpr size_t kPsMinLds = 96 * 1024;    // > 80 KiB: never two workgroups on one CU
constexpr int kPsSyncTop = 0;        // sync word: barrier arrivals of whole shards
constexpr int kPsSyncShard = 32;     // sync word of shard s: kPsSyncShard * (1 + s) (one 128-byte line each)
constexpr int kPsShards = 8;         // workgroup b arrives at shard b % 8
constexpr int kPsSyncHeads = kPsSyncShard * (1 + kPsShards);  // attention split arrivals [L][hkv]
#ifndef SLI_PS_PREFETCH2
#define SLI_PS_PREFETCH2 1
#endif
constexpr bool kPsPrefetch2 = SLI_PS_PREFETCH2;  // both weight chunks before the barrier (else one)
constexpr int kPsU2 = 4;                   // 16-byte vectors per lane per chunk, two-row phases (fits 128 VGPRs)

struct PsLayer {
    const void* qkv;
    const float* qkv_s;
    const void* wo;
    const float* wo_s;
    const void* gu;
    const float* gu_s;
    const void* down;
    const float* down_s;
};

struct PsArgs;
// the args record and the layer table are read through the constant address space (scalar loads)
using PsA = const __attribute__((address_space(4))) PsArgs;
struct PsArgs {
    const PsLayer* layers;  // [L]
    const void* emb;        // [V][D] (tied LM head)
    const float* emb_s;     // int8 row scales or null
    const float* norms;     // [2L+1][D]
    void* kc;               // [L][hkv][T][hd]
    void* vc;
    const float* sin_t;     // [T][hd/2]
    const float* cos_t;
    DevState* st;
    const int32_t* prompt;
    int32_t* hist;
    float* xv;              // [2L+1][D]    residual stream after embedding / each wo / each down
    float* qv;              // [L][hq*hd]   rotated q
    float* kvn;             // [L][2][hkv*hd] this step's rotated k and v rows
    float* part;            // [L][hq][splits][hd + pad] attention split partials
    float* attn;            // [L][hq*hd]   merged attention output
    float* actv;            // [L][Il]      sigmoid(g)*u
    float* logits;          // [v_n]
    unsigned long long* keys;  // [grid] per-workgroup argmax keys
    unsigned* sync;         // grid barrier (kPsSyncTop, kPsSyncShard) and attention split arrivals
                            // (kPsSyncHeads + l*hkv + h); zeroed before every launch
    unsigned long long* stamps;  // diagnostic (tools/ps_stamps.py), null in the product step:
                                 // [phase][workgroup][5] s_memrealtime at entry, poll done, input staged,
                                 // compute done, arrival
    int D, L, T, hd, hq, hkv, Il, V, v_lo, v_n, max_splits;
    float eps, scale;
    int act_mode;
    int wslot;  // LDS float offset of the norm-weight image (the last D floats of the dynamic LDS)
};

// ---------------------------------------------------------------- sc1 accesses
// (p and bytes are wave-uniform; readfirstlane makes that provable, or every buffer access through the
// descriptor becomes a waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ps_rsrc(const void* p, unsigned bytes) {
    const uint64_t u = (uint64_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
    void* q = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, 0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ float4 ps_ld4(__amdgpu_buffer_rsrc_t rs, unsigned off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /* sc1 */));
}
// Every pointer the step reaches is read from device memory (the args record, the layer table), so the
// compiler cannot prove it global; an explicit address-space cast keeps every access a global_ (or
// buffer_) instruction — a flat_ access would count on both vmcnt and lgkmcnt and force vmcnt(0) waits
// behind the prefetched weight stream.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gp(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}
__device__ __forceinline__ float ps_ld(const float* p) {
    return __hip_atomic_load(gp(const_cast<float*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ps_st(float* p, float v) {
    __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one element of a table of T (float / __half / int8) through a global pointer (raw bits: the class
// types cannot be read through an address-space-qualified pointer), and the matching store
template <typename T>
__device__ __forceinline__ float ps_ldt(const T* p, size_t i) {
    if constexpr (sizeof(T) == 2) {
        return __half2float(__ushort_as_half(gp(reinterpret_cast<const unsigned short*>(p))[i]));
    } else if constexpr (sizeof(T) == 1) {
        return (float)(int)gp(reinterpret_cast<const int8_t*>(p))[i];
    } else {
        return gp(reinterpret_cast<const float*>(p))[i];
    }
}
template <typename T>
__device__ __forceinline__ void ps_stt(T* p, size_t i, T v) {
    if constexpr (sizeof(T) == 2) {
        gp(reinterpret_cast<unsigned short*>(p))[i] = __half_as_ushort(v);
    } else {
        gp(p)[i] = v;
    }
}
__device__ __forceinline__ u32x4 ps_ld16(const void* p, bool nt) {
    const __attribute__((address_space(1))) u32x4* q = gp(reinterpret_cast<const u32x4*>(p));
    return nt ? __builtin_nontemporal_load(q) : *q;
}

// diagnostic stamps (only when PsArgs::stamps is set): slot k of this workgroup's record of phase p
__device__ __forceinline__ void ps_stamp(unsigned long long* st, int k) {
    if (st) st[k] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------- grid barrier
struct PsBar {
    unsigned* cnt;   // the sync block
    DevState* st;
    unsigned nwg;
    unsigned k;      // barriers this workgroup has arrived at
    // Two-level arrival (MI355X_MICROARCH.md price list, **fanin**: one word serialises ~12 ns per add):
    // every storing wave drained; then ONE lane adds to its shard (b % 8); the add that completes the
    // shard's round adds to the top word, which the control waves poll.
    __device__ __forceinline__ void arrive() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        ++k;
        if (threadIdx.x == 0) {
            const unsigned s = blockIdx.x % kPsShards;
            const unsigned ns = (nwg - s + kPsShards - 1) / kPsShards;  // workgroups of shard s
            const unsigned prev =
                __hip_atomic_fetch_add(gp(cnt + kPsSyncShard * (1 + s)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev + 1 == k * ns)
                __hip_atomic_fetch_add(gp(cnt + kPsSyncTop), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // control wave: every shard has completed k rounds. Bounded: false = gave up (error recorded).
    __device__ __forceinline__ bool poll() const {
        const unsigned target = k * min(nwg, (unsigned)kPsShards);
        for (unsigned spins = 0;; ++spins) {
            const unsigned v = __hip_atomic_load(gp(cnt + kPsSyncTop), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v >= target) return true;
            if (spins >= kPsSpinLimit) {
                if ((threadIdx.x & 63) == 0)
                    __hip_atomic_fetch_or(gp(&st->error), kPsErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
};

// The control wave waits for the grid barrier and runs `stage` (the phase's input into LDS); every wave
// then meets at the workgroup barrier. Returns false (uniformly) if the barrier spin gave up.
template <class Stage>
__device__ __forceinline__ bool ps_sync_stage(PsBar& bar, float* smem, const Stage& stage,
                                              unsigned long long* stamps = nullptr) {
    int* abort = reinterpret_cast<int*>(smem + kPsAbortSlot);
    if ((threadIdx.x >> 6) == 0) {
        stage.pre(smem);  // inputs that do not depend on the barrier (norm weights), before the poll
        if (bar.poll()) {
            if (threadIdx.x == 0) ps_stamp(stamps, 1);
            stage(smem);
            if (threadIdx.x == 0) ps_stamp(stamps, 2);
        } else if ((threadIdx.x & 63) == 0) {
            *abort = 1;
        }
    }
    __syncthreads();
    return *abort == 0;
}

struct PsNoStage {
    __device__ void pre(float*) const {}
    __device__ void post(float*) const {}
    __device__ void operator()(float*) const {}
};

// Control wave: a handed-off vector x[cols] (sc1 loads) into the swizzled LDS image gemv_chunk reads
// (xswz<G>), RMS-normalised when norm_w != nullptr (rms_kernel.cpp:12-22: sum of squares, / cols,
// + eps, sqrt, 1 / rms, then (x * inv) * w).
// The norm weights a phase multiplies by (rms_kernel.cpp:20-22) are static: the control wave loads the
// NEXT RMS phase's weights into an LDS image of their own (wslot) right after it has staged the current
// phase's input, while the compute waves stream, so no RMS phase waits for them after its barrier.
__device__ __forceinline__ void ps_load_norm(float* smem, int wslot, const float* w, int cols) {
    const int lane = threadIdx.x & 63, n4 = cols >> 2;
    float4* ws4 = reinterpret_cast<float4*>(smem + wslot);
    constexpr int B = 8;
    for (int f0 = 0; f0 < n4; f0 += 64 * B) {
        u32x4 v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) v[j] = ps_ld16(w + 4 * min(f0 + lane + 64 * j, n4 - 1), false);
#pragma unroll
        for (int j = 0; j < B; ++j)
            if (f0 + lane + 64 * j < n4) ws4[f0 + lane + 64 * j] = __builtin_bit_cast(float4, v[j]);
    }
}

template <int G>
struct PsStageVec {
    const float* x;
    const float* norm_w;     // non-null: RMS-normalise with the weights already in LDS at wslot
    float eps;
    int cols;
    int wslot;               // LDS float offset of the norm-weight image
    const float* next_norm;  // the next RMS phase's weights ([D]) to load after staging, or null
    int D;
    __device__ void pre(float*) const {}
    __device__ void post(float* smem) const {
        if (next_norm) ps_load_norm(smem, wslot, next_norm, D);
    }
    __device__ void operator()(float* smem) const {
        const int lane = threadIdx.x & 63;
        const int n4 = cols >> 2;
        float4* xs4 = reinterpret_cast<float4*>(smem + kGemvLdsHead);
        const auto rs = ps_rsrc(x, (unsigned)(sizeof(float) * cols));
        float ss = 0.0f;
        constexpr int B = 8;   // sc1 loads per lane in flight per round trip
        for (int f0 = 0; f0 < n4; f0 += 64 * B) {
            float4 v[B];
#pragma unroll
            for (int j = 0; j < B; ++j) v[j] = ps_ld4(rs, (unsigned)(16 * (f0 + lane + 64 * j)));  // past the end: 0
#pragma unroll
            for (int j = 0; j < B; ++j) {
                const int f = f0 + lane + 64 * j;
                if (f < n4) xs4[xswz<G>(f)] = v[j];
                ss += v[j].x * v[j].x;  // out-of-range vectors read as 0
                ss += v[j].y * v[j].y;
                ss += v[j].z * v[j].z;
                ss += v[j].w * v[j].w;
            }
        }
        if (norm_w == nullptr) return;
        ss = wave_sum(ss);
        const float tep = ss / (float)cols;   // rms_kernel.cpp:17
        const float rms = sqrtf(tep + eps);  // :18
        const float inv = 1.0f / rms;        // :19
        const float4* ws4 = reinterpret_cast<const float4*>(smem + wslot);
        for (int f = lane; f < n4; f += 64) {  // :20-22  y = (x * inv) * w
            const float4 w = ws4[f];
            float4 v = xs4[xswz<G>(f)];
            v.x = (v.x * inv) * w.x;
            v.y = (v.y * inv) * w.y;
            v.z = (v.z * inv) * w.z;
            v.w = (v.w * inv) * w.w;
            xs4[xswz<G>(f)] = v;
        }
    }
};

// ---------------------------------------------------------------- epilogues (handed-off outputs: sc1)
// Fused q/k/v + RoPE (rope_kernel.cpp:30-38) + K/V: the cache row (plain: read by later launches) and
// this step's row for the attention phase (sc1).
template <typename KT>
struct PsEpiQKV {
    float* q_out;
    KT* kc;
    KT* vc;
    float* kn;   // [hkv*hd] this step's k row, then v row at kn + hkv*hd
    const float* rscale;
    const float* sin_t;
    const float* cos_t;
    int pos, hq, hkv, hd, T;
    float pre_s0 = 1.0f, pre_s1 = 1.0f, pre_sin = 0.0f, pre_cos = 1.0f;
    __device__ int units() const { return (hq + 2 * hkv) * (hd / 2); }
    __device__ void rows(int u, int* r) const {
        const int half = hd / 2, uh = u / half, d = u - uh * half;
        r[0] = uh * hd + d;
        r[1] = uh * hd + d + half;
    }
    __device__ void prefetch_a(int u) {
        int r[2];
        rows(u, r);
        const auto sp = gp(rscale ? rscale : sin_t);
        pre_s0 = sp[rscale ? r[0] : 0];
        pre_s1 = sp[rscale ? r[1] : 0];
    }
    __device__ void prefetch_b(int u) {
        const int half = hd / 2, d = u - (u / half) * half;
        pre_sin = gp(sin_t)[pos * half + d];
        pre_cos = gp(cos_t)[pos * half + d];
    }
    __device__ void store(int u, const int*, const float* acc, bool pre) const {
        const int half = hd / 2, uh = u / half, d = u - uh * half;
        float a0 = acc[0], a1 = acc[1];
        if (rscale) {
            int r[2];
            rows(u, r);
            a0 *= pre ? pre_s0 : gp(rscale)[r[0]];
            a1 *= pre ? pre_s1 : gp(rscale)[r[1]];
        }
        if (uh < hq + hkv) {
            const float fci = pre ? pre_sin : gp(sin_t)[pos * half + d], fcr = pre ? pre_cos : gp(cos_t)[pos * half + d];
            const float r0 = a0 * fcr - a1 * fci;
            const float r1 = a1 * fcr + a0 * fci;
            if (uh < hq) {
                ps_st(q_out + (size_t)uh * hd + d, r0);
                ps_st(q_out + (size_t)uh * hd + d + half, r1);
            } else {
                const int h = uh - hq;
                const KT k0 = from_f32<KT>(r0), k1 = from_f32<KT>(r1);
                KT* k = kc + ((size_t)h * T + pos) * hd;
                ps_stt(k, d, k0);
                ps_stt(k, d + half, k1);
                ps_st(kn + (size_t)h * hd + d, to_f32(k0));  // the cache's rounding, as attention reads it
                ps_st(kn + (size_t)h * hd + d + half, to_f32(k1));
            }
        } else {
            const int h = uh - hq - hkv;
            const KT v0 = from_f32<KT>(a0), v1 = from_f32<KT>(a1);
            KT* v = vc + ((size_t)h * T + pos) * hd;
            ps_stt(v, d, v0);
            ps_stt(v, d + half, v1);
            float* vn = kn + (size_t)hkv * hd;
            ps_st(vn + (size_t)h * hd + d, to_f32(v0));
            ps_st(vn + (size_t)h * hd + d + half, to_f32(v1));
        }
    }
    __device__ void finish(float*) {}
};

// y[row] = resid[row] + (sum * rscale[row]) (matmul_kernel.cpp:26 + add_kernel.cpp:5-14)
struct PsEpiStore {
    float* y;
    const float* resid;  // handed off: sc1
    const float* rscale;
    int nrows;
    float pre_r = 0.0f, pre_s = 1.0f;
    __device__ int units() const { return nrows; }
    __device__ void rows(int u, int* r) const { r[0] = min(u, nrows - 1); }
    __device__ void prefetch_a(int u) {
        const int row = min(u, nrows - 1);
        pre_r = ps_ld(resid + row);
        pre_s = rscale ? gp(rscale)[row] : 1.0f;
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int*, const float* v, bool pre) const {
        if (u >= nrows) return;
        const float a = rscale ? v[0] * (pre ? pre_s : gp(rscale)[u]) : v[0];
        ps_st(y + u, (pre ? pre_r : ps_ld(resid + u)) + a);
    }
    __device__ void finish(float*) {}
};

// act = sigmoid(g) * u (swiglu_kernel.cpp:12-13) or SiLU(g) * u
struct PsEpiSwiGLU {
    float* act;
    const float* rscale;
    int inter;
    int silu;
    float pre_s0 = 1.0f, pre_s1 = 1.0f;
    __device__ int units() const { return inter; }
    __device__ void rows(int u, int* r) const {
        r[0] = u;
        r[1] = inter + u;
    }
    __device__ void prefetch_a(int u) {
        if (rscale) {
            pre_s0 = gp(rscale)[u];
            pre_s1 = gp(rscale)[inter + u];
        }
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int*, const float* acc, bool pre) const {
        float g = acc[0], up = acc[1];
        if (rscale) {
            g *= pre ? pre_s0 : gp(rscale)[u];
            up *= pre ? pre_s1 : gp(rscale)[inter + u];
        }
        float t = 1.0f / (1.0f + expf(-g));
        if (silu) t = g * t;
        ps_st(act + u, t * up);
    }
    __device__ void finish(float*) {}
};

// tied LM head (model.cpp:136-139): logits (plain: read by the host) + the workgroup's max argmax key
struct PsEpiLogits {
    float* logits;
    unsigned long long* keys;
    const float* rscale;
    int nrows, vocab_off;
    unsigned long long best = 0;
    float pre_s[2] = {1.0f, 1.0f};
    __device__ int units() const { return (nrows + 1) / 2; }
    __device__ void rows(int u, int* r) const {
        r[0] = min(2 * u, nrows - 1);
        r[1] = min(2 * u + 1, nrows - 1);
    }
    __device__ void prefetch_a(int u) {
        if (rscale) {
            pre_s[0] = gp(rscale)[min(2 * u, nrows - 1)];
            pre_s[1] = gp(rscale)[min(2 * u + 1, nrows - 1)];
        }
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int*, const float* acc, bool pre) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = 2 * u + i;
            if (row < nrows) {
                const float a = rscale ? acc[i] * (pre ? pre_s[i] : gp(rscale)[row]) : acc[i];
                gp(logits)[row] = a;
                const unsigned long long k = argmax_key(a, (unsigned)(row + vocab_off));
                best = k > best ? k : best;
            }
        }
    }
    // every thread of the workgroup: the workgroup's max key, published sc1
    __device__ void finish(float* smem) {
        unsigned long long* red = reinterpret_cast<unsigned long long*>(smem);
        const unsigned long long b = wave_max_u64(best);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long m = 0;
            for (int w = 0; w < kPsWaves; ++w) m = red[w] > m ? red[w] : m;
            __hip_atomic_store(gp(keys + blockIdx.x), m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    }
};

// ---------------------------------------------------------------- one GEMV phase
// gemv_block's schedule on the 15 compute waves of every workgroup: the epilogue's own inputs and the
// first two weight chunks are issued BEFORE the grid barrier that guards the phase input; the control
// wave stages the input; the compute waves stream and reduce; the compute waves' threads run the
// epilogue one unit each; the workgroup arrives at the next barrier.
template <typename WT, int R, int U, class Epi, class Stage>
__device__ __forceinline__ bool ps_gemv(const WT* __restrict__ W, int cols, Epi& epi, const Stage& stage, float* smem,
                                        PsBar& bar, unsigned long long* stamps) {
    if (threadIdx.x == 0) ps_stamp(stamps, 0);
    constexpr int EPV = Vec16<WT>::N;
    constexpr int CV = U * 64;
    const int lane = threadIdx.x & 63;
    const int cw = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) - 1;  // -1: control wave
    const int nvec = cols / EPV;
    const size_t row_bytes = (size_t)cols * sizeof(WT);
    const int nunits = epi.units();
    const int total_waves = gridDim.x * kPsCW;
    const int gw = blockIdx.x * kPsCW + max(cw, 0);
    const int u_begin = gemv_unit_begin(gw, nunits, total_waves);
    const int u_end = gemv_unit_begin(gw + 1, nunits, total_waves);
    const int ub = gemv_unit_begin(blockIdx.x * kPsCW, nunits, total_waves);
    const int ue = gemv_unit_begin((blockIdx.x + 1) * kPsCW, nunits, total_waves);
    const int cpr = (nvec + CV - 1) / CV;
    const int nsteps = cw >= 0 ? (u_end - u_begin) * cpr : 0;
    float* res = smem + kGemvLdsHead + cols;
    const int u_last = max(min(u_end, nunits) - 1, 0);
    const int et = (int)threadIdx.x - 64;  // epilogue thread (compute waves)
    const int pre_unit = max(min(ub + max(et, 0), nunits - 1), 0);

    auto load_step = [&](int u, int c, u32x4 (&w)[U][R]) {
        int rows[R];
        epi.rows(min(u, u_last), rows);
        const int v = (u > u_last ? cpr - 1 : c) * CV + lane;
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int vj = min(v + j * 64, nvec - 1);
#pragma unroll
            for (int r = 0; r < R; ++r)
                w[j][r] = ps_ld16(reinterpret_cast<const char*>(W) + (size_t)rows[r] * row_bytes + (size_t)vj * 16, true);
        }
    };
    auto next = [&](int& u, int& c) {
        if (++c == cpr) {
            c = 0;
            ++u;
        }
    };
    u32x4 wa[U][R], wb[U][R];
    int lu = u_begin, lc = 0, cu = u_begin, cc = 0;
    if (cw >= 0) {
        epi.prefetch_a(pre_unit);  // static inputs, or outputs published before the last barrier
        load_step(lu, lc, wa);
        next(lu, lc);
        if (kPsPrefetch2) {
            load_step(lu, lc, wb);
            next(lu, lc);
        }
        epi.prefetch_b(pre_unit);  // waits only for prefetch_a's loads (issued before the weights)
    }
    if (!ps_sync_stage(bar, smem, stage, stamps)) return false;
    if (cw < 0) stage.post(smem);  // the control wave, while the compute waves stream
    if (!kPsPrefetch2 && cw >= 0) {
        load_step(lu, lc, wb);
        next(lu, lc);
    }
    if (cw >= 0) {
        const float* xs = smem + kGemvLdsHead;
        float acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = 0.0f;
        auto consume_step = [&](int u, int c, const u32x4(&w)[U][R]) {
            const int v = c * CV + lane;
            if ((c + 1) * CV <= nvec)
                gemv_chunk<WT, R, U>(w, xs, v, acc);
            else
                gemv_chunk<WT, R, U, true>(w, xs, v, acc, nvec);
            if (c == cpr - 1) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const float t = wave_sum(acc[r]);
                    if (lane == 0) res[(u - ub) * R + r] = t;
                    acc[r] = 0.0f;
                }
            }
        };
        int k = 0;
        for (; k + 2 < nsteps; k += 2) {
            consume_step(cu, cc, wa);
            next(cu, cc);
            load_step(lu, lc, wa);
            next(lu, lc);
            consume_step(cu, cc, wb);
            next(cu, cc);
            load_step(lu, lc, wb);
            next(lu, lc);
        }
        if (k < nsteps) {
            consume_step(cu, cc, wa);
            next(cu, cc);
            if (k + 1 < nsteps) consume_step(cu, cc, wb);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) ps_stamp(stamps, 3);
    if (et >= 0) {
        for (int u = ub + et; u < ue; u += kPsThreads - 64) {
            int rows[R];
            epi.rows(u, rows);
            epi.store(u, rows, res + (u - ub) * R, u == pre_unit);
        }
    }
    epi.finish(smem);
    bar.arrive();
    if (threadIdx.x == 0) ps_stamp(stamps, 4);
    return true;
}

// ---------------------------------------------------------------- attention phase
// Split-context flash decode (mha_kernel.cpp:36-77 semantics) on the 15 compute waves: a workgroup job is
// (kv head, split of PPWG positions); each compute wave owns PPW consecutive positions, NIT wave-
// instructions of RPI rows. The job's K/V rows below the current position are issued before the grid
// barrier (they were written by earlier launches); this step's row comes from the qkv phase's sc1
// hand-off. Partials are merged in LDS, published sc1, and the head's last-arriving split merges the
// head (attn_merge, split order: deterministic).
// attn_merge (attention.h) on the persistent path: kv head kvh's ns live split partials of this layer
// merged in split order (M = max m_i, out = sum e^{m_i-M} o_i / sum e^{m_i-M} l_i), sc1 loads and stores,
// by every thread of the workgroup; ends with the storing waves drained.
template <int HD, int G>
__device__ __forceinline__ void ps_merge(const float* part, float* out, int kvh, int max_splits, int ns) {
    constexpr int PS = HD + kAttnPartPad;
    constexpr int NS = 16;
    const unsigned bytes = (unsigned)(sizeof(float) * (size_t)G * max_splits * PS);
    const auto rs = ps_rsrc(part + (size_t)kvh * G * max_splits * PS, bytes);
    for (int i = threadIdx.x; i < G * HD; i += kPsThreads) {
        const int g = i / HD, d = i - g * HD;
        const unsigned row0 = (unsigned)(g * max_splits) * PS;
        float M = -INFINITY;
        for (int s0 = 0; s0 < ns; s0 += NS) {
            float mv[NS];
#pragma unroll
            for (int j = 0; j < NS; ++j)
                mv[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                      rs, 4u * (row0 + (unsigned)min(s0 + j, ns - 1) * PS + HD), 0, 16));
#pragma unroll
            for (int j = 0; j < NS; ++j) M = fmaxf(M, mv[j]);
        }
        float o = 0.0f, L = 0.0f;
        for (int s0 = 0; s0 < ns; s0 += NS) {
            float mv[NS], lv[NS], ov[NS];
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const unsigned r = row0 + (unsigned)min(s0 + j, ns - 1) * PS;
                mv[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * (r + HD), 0, 16));
                lv[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * (r + HD + 1), 0, 16));
                ov[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * (r + d), 0, 16));
            }
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                if (s0 + j < ns) {
                    const float w = expf(mv[j] - M);
                    o = fmaf(w, ov[j], o);
                    L = fmaf(w, lv[j], L);
                }
            }
        }
        ps_st(out + (size_t)(kvh * G + g) * HD + d, o / L);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename KT, int HD>
struct PsAttnGeom {
    static constexpr int EPV = Vec16<KT>::N;
    static constexpr int LPR = HD / EPV;
    static constexpr int RPI = 64 / LPR;
    static constexpr int PPWG = kAttnSlots * RPI;                   // positions per job (the launch path's split)
    static constexpr int NIT = (kAttnSlots + kPsCW - 1) / kPsCW;  // wave-instructions per compute wave
    static constexpr int PPW = NIT * RPI;                           // (the last waves of a job run short)
};

template <typename KT, int HD, int G>
__device__ __forceinline__ bool ps_attention(PsA& a, int l, int pos, float* smem, PsBar& bar,
                                             unsigned long long* stamps) {
    if (threadIdx.x == 0) ps_stamp(stamps, 0);
    using Geo = PsAttnGeom<KT, HD>;
    constexpr int EPV = Geo::EPV, LPR = Geo::LPR, RPI = Geo::RPI, NIT = Geo::NIT, PPW = Geo::PPW;
    constexpr int SH = HD + 2;
    const int lane = threadIdx.x & 63;
    const int cw = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) - 1;
    const int sub = lane / LPR, li = lane - sub * LPR;
    const int nsplit = min(pos / Geo::PPWG + 1, a.max_splits);  // live splits of every head
    const int njobs = a.hkv * nsplit;
    const KT* kl = (const KT*)a.kc + (size_t)l * a.hkv * a.T * HD;
    const KT* vl = (const KT*)a.vc + (size_t)l * a.hkv * a.T * HD;
    const float* q = a.qv + (size_t)l * a.hq * HD;
    const float* kn = a.kvn + (size_t)l * 2 * a.hkv * HD;
    const float* vn = kn + (size_t)a.hkv * HD;
    float* part = a.part + (size_t)l * a.hq * a.max_splits * (HD + kAttnPartPad);
    float* out = a.attn + (size_t)l * a.hq * HD;
    float* sh = smem + kGemvLdsHead;  // [kPsCW][G][SH]
    int* last = reinterpret_cast<int*>(smem + kPsAbortSlot - 1);

    bool first = true;
    for (int job = blockIdx.x; ; job += gridDim.x) {
        const bool live = job < njobs;  // uniform
        const int kvh = live ? job / nsplit : 0;
        const int split = live ? job - kvh * nsplit : 0;
        const int t0 = split * Geo::PPWG + max(cw, 0) * PPW;
        const int t_end = min(min(t0 + PPW, (split + 1) * Geo::PPWG), pos + 1);
        const bool live_wave = live && cw >= 0 && t0 < t_end;  // (the last waves of a job may have no rows)
        u32x4 kr[NIT], vr[NIT];
        const KT* kb = kl + (size_t)kvh * a.T * HD + li * EPV;
        const KT* vb = vl + (size_t)kvh * a.T * HD + li * EPV;
        if (live_wave) {  // rows of earlier launches: before the barrier (a stale row pos is replaced below)
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int t = min(t0 + it * RPI + sub, t_end - 1);
                kr[it] = ps_ld16(kb + (size_t)t * HD, false);
                vr[it] = ps_ld16(vb + (size_t)t * HD, false);
            }
        }
        if (first) {
            if (!ps_sync_stage(bar, smem, PsNoStage{}, stamps)) return false;
            first = false;
        }
        if (!live) break;
        float m[G], lsum[G], ov[G][EPV];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            m[g] = -INFINITY;
            lsum[g] = 0.0f;
#pragma unroll
            for (int e = 0; e < EPV; ++e) ov[g][e] = 0.0f;
        }
        if (live_wave) {
            // this step's row: the qkv phase's sc1 hand-off (already rounded to the cache type)
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int t = min(t0 + it * RPI + sub, t_end - 1);
                if (t == pos) {
                    float kf[EPV], vf[EPV];
#pragma unroll
                    for (int e = 0; e < EPV; ++e) {
                        kf[e] = ps_ld(kn + (size_t)kvh * HD + li * EPV + e);
                        vf[e] = ps_ld(vn + (size_t)kvh * HD + li * EPV + e);
                    }
                    kr[it] = Vec16<KT>::pack(kf);
                    vr[it] = Vec16<KT>::pack(vf);
                }
            }
            float qv[G][EPV];
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int e = 0; e < EPV; ++e) qv[g][e] = ps_ld(q + (size_t)(kvh * G + g) * HD + li * EPV + e);
            float s[NIT][G];
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                float kf[EPV];
                Vec16<KT>::unpack(kr[it], kf);
                const bool rl = (t0 + it * RPI + sub) < t_end;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    float d = 0.0f;
#pragma unroll
                    for (int e = 0; e < EPV; ++e) d = fmaf(qv[g][e], kf[e], d);
                    d = group_sum<LPR>(d);
                    s[it][g] = rl ? d * a.scale : -INFINITY;  // mha_kernel.cpp:51-60 (sum * scale)
                    m[g] = fmaxf(m[g], s[it][g]);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g)
                m[g] = stride_max<LPR>(m[g]);
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                float vf[EPV];
                Vec16<KT>::unpack(vr[it], vf);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const float p = expf(s[it][g] - m[g]);
                    lsum[g] += p;
#pragma unroll
                    for (int e = 0; e < EPV; ++e) ov[g][e] = fmaf(p, vf[e], ov[g][e]);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                lsum[g] = stride_sum<LPR>(lsum[g]);
#pragma unroll
                for (int e = 0; e < EPV; ++e) ov[g][e] = stride_sum<LPR>(ov[g][e]);
            }
        }
        if (threadIdx.x == 64) ps_stamp(stamps, 2);  // wave 1's loads landed and scored
        if (cw >= 0 && sub == 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float* row = sh + ((size_t)cw * G + g) * SH;
#pragma unroll
                for (int e = 0; e < EPV; ++e) row[li * EPV + e] = ov[g][e];
                if (li == 0) {
                    row[HD] = m[g];
                    row[HD + 1] = lsum[g];
                }
            }
        }
        __syncthreads();
        // the workgroup's partial (the compute waves' states merged in wave order), published sc1
        for (int i = threadIdx.x; i < G * HD; i += kPsThreads) {
            const int g = i / HD, d = i - g * HD;
            float M = -INFINITY;
#pragma unroll
            for (int w = 0; w < kPsCW; ++w) M = fmaxf(M, sh[((size_t)w * G + g) * SH + HD]);
            float o = 0.0f, L = 0.0f;
#pragma unroll
            for (int w = 0; w < kPsCW; ++w) {
                const float* row = sh + ((size_t)w * G + g) * SH;
                const float c = expf(row[HD] - M);  // dead waves: m = -inf -> 0
                o = fmaf(c, row[d], o);
                L = fmaf(c, row[HD + 1], L);
            }
            float* dst = part + ((size_t)(kvh * G + g) * a.max_splits + split) * (HD + kAttnPartPad);
            ps_st(dst + d, o);
            if (d == 0) {
                ps_st(dst + HD, M);
                ps_st(dst + HD + 1, L);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned* c = a.sync + kPsSyncHeads + (size_t)l * a.hkv + kvh;
            const unsigned prev = __hip_atomic_fetch_add(gp(c), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *last = prev == (unsigned)(nsplit - 1);
        }
        __syncthreads();
        if (threadIdx.x == 0) ps_stamp(stamps, 3);
        if (*last) ps_merge<HD, G>(part, out, kvh, a.max_splits, nsplit);
        __syncthreads();  // sh and `last` are reused by the next job
    }
    if (first && !ps_sync_stage(bar, smem, PsNoStage{}, stamps)) return false;  // (no job at all)
    bar.arrive();
    if (threadIdx.x == 0) ps_stamp(stamps, 4);
    return true;
}

// ---------------------------------------------------------------- the step
template <typename WT>
struct PsU {  // weight vectors in flight per lane per chunk (int8: half, gemv's launch_gemv_u rule)
    static constexpr int H(int u) { return sizeof(WT) == 1 && u >= 2 ? u / 2 : u; }
};

// One phase of the step: p = 0 embedding; p = 1 + 5l + {0 qkv, 1 attention, 2 wo, 3 gate/up, 4 down};
// p = 1 + 5L LM head. Returns false if a barrier spin gave up. Every phase ends with the workgroup's
// arrival at the grid barrier; every phase but the embedding begins by waiting for it.
template <typename WT, typename KT, int HD, int G>
__device__ __forceinline__ bool ps_phase(PsA& a, int p, int pos, float* smem, PsBar& bar) {
    constexpr int GV = Vec16<WT>::N / 4;  // float4 of x per 16-byte weight vector (LDS swizzle)
    const int D = a.D;
    unsigned long long* const stamps = a.stamps ? a.stamps + ((size_t)p * gridDim.x + blockIdx.x) * 5 : nullptr;
    if (p == 0) {  // embedding (emb_kernel.cpp:4-21, token on the device) -> x_0
        const int token = ((const __attribute__((address_space(4))) DevState*)a.st)->token;
        const bool ok = token >= 0 && token < a.V;
        const float s = (ok && a.emb_s) ? gp(a.emb_s)[token] : 1.0f;
        const WT* row = (const WT*)a.emb + (size_t)(ok ? token : 0) * D;
        const int chunk = (D + gridDim.x - 1) / gridDim.x;
        for (int i = blockIdx.x * chunk + threadIdx.x; i < min(D, (blockIdx.x + 1) * chunk); i += kPsThreads)
            ps_st(a.xv + i, ok ? ps_ldt(row, i) * s : 0.0f);
        if ((threadIdx.x >> 6) == 0) ps_load_norm(smem, a.wslot, a.norms, D);  // qkv(0)'s norm weights
        bar.arrive();
        return true;
    }
    if (p == 1 + 5 * a.L) {  // final RMSNorm + tied LM head + argmax keys (model.cpp:131-139)
        PsEpiLogits e{a.logits, a.keys, a.emb_s ? a.emb_s + a.v_lo : nullptr, a.v_n, a.v_lo};
        PsStageVec<GV> st{a.xv + (size_t)(2 * a.L) * D, a.norms + (size_t)(2 * a.L) * D, a.eps, D, a.wslot, nullptr, D};
        return ps_gemv<WT, 2, PsU<WT>::H(kPsU2)>((const WT*)a.emb + (size_t)a.v_lo * D, D, e, st, smem, bar, stamps);
    }
    const int l = (p - 1) / 5;
    const __attribute__((address_space(4))) PsLayer& w = ((const __attribute__((address_space(4))) PsLayer*)a.layers)[l];
    const float* x_in = a.xv + (size_t)(2 * l) * D;
    float* x_mid = a.xv + (size_t)(2 * l + 1) * D;
    float* x_out = a.xv + (size_t)(2 * l + 2) * D;
    switch ((p - 1) - 5 * l) {
        case 0: {  // RMSNorm + [wq; wk; wv] + RoPE + K/V (model.cpp:52-67)
            KT* kc = (KT*)a.kc + (size_t)l * a.hkv * a.T * HD;
            KT* vc = (KT*)a.vc + (size_t)l * a.hkv * a.T * HD;
            PsEpiQKV<KT> e{a.qv + (size_t)l * a.hq * HD, kc, vc, a.kvn + (size_t)l * 2 * a.hkv * HD, w.qkv_s, a.sin_t,
                           a.cos_t, pos, a.hq, a.hkv, HD, a.T};
            PsStageVec<GV> st{x_in, a.norms + (size_t)(2 * l) * D, a.eps, D, a.wslot, a.norms + (size_t)(2 * l + 1) * D, D};
            return ps_gemv<WT, 2, PsU<WT>::H(kPsU2)>((const WT*)w.qkv, D, e, st, smem, bar, stamps);
        }
        case 1: return ps_attention<KT, HD, G>(a, l, pos, smem, bar, stamps);  // model.cpp:70-78
        case 2: {  // wo + residual (model.cpp:80-90)
            PsEpiStore e{x_mid, x_in, w.wo_s, D};
            PsStageVec<GV> st{a.attn + (size_t)l * a.hq * HD, nullptr, 0.0f, a.hq * HD, a.wslot, nullptr, D};
            return ps_gemv<WT, 1, PsU<WT>::H(4)>((const WT*)w.wo, a.hq * HD, e, st, smem, bar, stamps);
        }
        case 3: {  // RMSNorm + [gate; up] + SwiGLU (model.cpp:93-115)
            PsEpiSwiGLU e{a.actv + (size_t)l * a.Il, w.gu_s, a.Il, a.act_mode};
            PsStageVec<GV> st{x_mid, a.norms + (size_t)(2 * l + 1) * D, a.eps, D, a.wslot, a.norms + (size_t)(2 * l + 2) * D, D};
            return ps_gemv<WT, 2, PsU<WT>::H(kPsU2)>((const WT*)w.gu, D, e, st, smem, bar, stamps);
        }
        default: {  // down + residual (model.cpp:118-128)
            PsEpiStore e{x_out, x_mid, w.down_s, D};
            PsStageVec<GV> st{a.actv + (size_t)l * a.Il, nullptr, 0.0f, a.Il, a.wslot, nullptr, D};
            return ps_gemv<WT, 1, PsU<WT>::H(6)>((const WT*)w.down, a.Il, e, st, smem, bar, stamps);
        }
    }
}

// PsArgs lives in device memory (one scalar-cached record), not in the kernel's argument SGPRs: the
// phases read what they need, and nothing but (phase, pos, barrier count) is live across phases.
template <typename WT, typename KT, int HD, int G>
__global__ void __launch_bounds__(kPsThreads) ps_step_kernel(const PsArgs* __restrict__ ap) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    if (threadIdx.x == 0) reinterpret_cast<int*>(smem)[kPsAbortSlot] = 0;
    __syncthreads();
    PsA* ak = (PsA*)ap;
    PsA& a = *ak;
    PsBar bar{a.sync, a.st, gridDim.x, 0};
    const int pos = ((const __attribute__((address_space(4))) DevState*)a.st)->pos;
    const int nphase = 2 + 5 * a.L;
    for (int p = 0; p < nphase; ++p) {
        // opaque per phase: the record's fields are re-read (scalar cache) inside each phase instead of
        // being hoisted out of the loop and held in SGPRs across all of them
        PsA* pa = ak;
        asm volatile("" : "+s"(pa));
        if (!ps_phase<WT, KT, HD, G>(*pa, p, pos, smem, bar)) return;
    }
    if (blockIdx.x != 0) return;
    // argmax over the workgroups' keys, then the decode state (model.cpp:157-183)
    if (!ps_sync_stage(bar, smem, PsNoStage{})) return;
    unsigned long long b = 0;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += kPsThreads) {
        const unsigned long long k = __hip_atomic_load(gp(a.keys + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        b = k > b ? k : b;
    }
    b = wave_max_u64(b);
    unsigned long long* red = reinterpret_cast<unsigned long long*>(smem);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < kPsWaves; ++w) b = red[w] > b ? red[w] : b;
        a.st->key = b;
        finalize_state(a.st, a.prompt, a.hist, a.T);
    }
}

}  // namespace sli
