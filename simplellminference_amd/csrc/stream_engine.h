// stream_engine.h — the whole batch-1 decode step (LlamaModel::forward, source/model/model.cpp:40-140, plus
// the argmax + state update of predict, :157-183) as ONE persistent launch built around a weight stream that
// never waits for a dependency (MI355X_MICROARCH.md price list: **engine-vs-launches**, **prefetch-credit**,
// **ldsdma-fill**, **gather-pass**).
//
// Why: at batch 1 every byte the step reads (weights, the K/V context) is known before the step starts; only
// the small activation vectors depend on the previous op. The launch path (engine.hip) pays, at every one of
// its 161 kernel boundaries, a drained HBM stream (the next kernel's first loads issue only after the
// previous kernel's last wave ends: ramp + tail + boundary ≈ 3-5 µs per launch). Here the
// stream runs across the dependency edges:
//
//   * one workgroup per CU: wave 0 is the LOADER, waves 1..kEsNC are CONSUMERS;
//   * the loader walks this CU's share of every op of the step, in step order (qkv rows, the attention job's
//     K/V rows, wo rows, gate/up rows, down rows per layer, then the LM-head rows), moving 16 KiB slots into
//     an LDS ring by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction, non-temporal) with a
//     counted vmcnt that keeps kEsAhead slots in flight. It waits for nothing but a FREE ring slot, so while
//     the consumers wait for an op's input (an edge), the next op's weights keep arriving;
//   * consumers wait for the op's input edge, stage the input vector into LDS (RMS statistics on the fly),
//     then consume the ring slots: a slot holds kEsNC rows x 128 16-byte vectors (2 KiB per row piece), one
//     row per consumer wave, so a row's partial dot product stays in ONE wave's registers across its pieces
//     (deterministic: wave_sum at the row's last piece). The attention slots hold 16 KiB of one job's K or V
//     rows; each consumer wave owns a fixed run of positions of every slot (online softmax);
//   * edges between CUs: every CU publishes its outputs with write-through (sc1) stores, drains, and adds to
//     the op's arrival counter sharded per XCD (8 words on their own lines: MI355X_MICROARCH.md **fanin**);
//     one consumer wave polls the 8 shards and releases the others through an LDS word
//     (MI355X_MICROARCH.md "Valid forms", hand-off table row 1: sc1 stores, drained before one lane's
//     agent-scope add per workgroup, sc1 loads after the poll matched). Every hand-off buffer is written once
//     per launch (per layer), so no L2 holds a stale copy of a line a later op of the same launch rewrites;
//   * per op, the LAST consumer wave to finish its rows runs the op's epilogue (RoPE + K/V row, SwiGLU,
//     residual add, logits + argmax key) and publishes; the other waves move on to the next edge.
//
// Fused RMSNorm (rms_kernel.cpp:5-23): the staged input is x*w and the row sums are multiplied by
// inv_rms = 1/sqrt(mean(x^2)+eps) in the epilogue (a per-vector scalar commutes with the column sum; the
// oracle normalises first: same value up to fp32 rounding, within the 1e-3 bar).
//
// Every spin is bounded; a timeout sets DevState::error bit kEsErrTimeout (reported by every predict path)
// and the workgroup winds down.
#pragma once
#include "common.h"
#include "step_state.h"

namespace sli {

constexpr int kEsNC = 8;                      // consumer waves
constexpr int kEsThreads = 64 * (kEsNC + 1);  // + the loader wave
constexpr int kEsSlot = 16384;                // bytes per ring slot (16 LDS-DMA wave-instructions)
constexpr int kEsPiece = 128;                 // 16-byte vectors of one row per slot (a consumer wave's share)
constexpr int kEsMaxSlots = 8;
#ifndef SLI_ES_AHEAD
#define SLI_ES_AHEAD 2
#endif
constexpr int kEsAhead = SLI_ES_AHEAD;  // slots the loader keeps in flight beyond the last published one
constexpr int kEsShards = 8;            // arrival-counter shards (blockIdx % 8)
constexpr int kEsShardWords = 16;       // one 64-byte line per shard
constexpr unsigned kEsSpin = 1u << 21;  // bounded spins (x s_sleep: ~ 0.1-1 s)

// LDS control words (u32 slots of the ctl area)
enum : int {
    kEsFull = 0,                       // [kEsMaxSlots] fills landed per slot
    kEsFree = kEsMaxSlots,             // [kEsMaxSlots] consumer-wave releases per slot
    kEsEdgeSeen = 2 * kEsMaxSlots,     // last op whose input edge was observed (+1)
    kEsResDone,                        // consumer waves done with their rows, monotonic over ops
    kEsCbar,                           // consumer barrier arrivals, monotonic
    kEsAbort,                          // a spin gave up
    kEsSumSq = 24,                     // [kEsNC] per-wave partial sums of squares (floats)
    kEsKey = 40,                       // [2] u64 scratch (LM-head key)
    kEsCtlWords = 48
};

// Op numbering: op o = 5*l + k (k: 0 qkv, 1 attention, 2 wo, 3 gate/up, 4 down), o = 5L the LM head. Op o
// waits for edge o-1 (the previous op's outputs on every CU) and arrives at edge o.
enum : int { kEsQkv = 0, kEsAttn, kEsWo, kEsGu, kEsDown, kEsOpsPerLayer };

struct EsLayer {
    const void* qkv;
    const float* qkv_s;
    const void* wo;
    const float* wo_s;
    const void* gu;
    const float* gu_s;
    const void* down;
    const float* down_s;
};

struct EsArgs {
    const EsLayer* layers;  // [L]
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
    float* xv;              // [2L+1][D]  residual stream: embedding, after each wo, after each down
    float* qv;              // [L][hq*hd] rotated q
    float* kvn;             // [L][2][hkv*hd] this step's k and v rows (rounded to the cache type)
    float* part;            // [L][hq][max_splits][hd + 4] attention job partials (o, m, l)
    float* actv;            // [L][Il]
    float* logits;          // [v_n]
    unsigned long long* keys;  // [grid] per-CU argmax keys
    unsigned* edges;        // [5L+1][kEsShards][kEsShardWords] arrival counters, zeroed before each launch
    const void* zero;       // 1 KiB of zeros: the DMA source of padding rows / lanes past a row's end
    unsigned long long* stamps;  // diagnostic: [op][grid][4] s_memrealtime (edge seen, staged, rows done, published)
    int D, L, T, hd, hq, hkv, Il, V, v_lo, v_n;
    int max_splits;         // partial rows per q head (T / ppj rounded up)
    int ppj;                // context positions per attention job (a multiple of the slot's positions)
    float eps, scale;
    int act_mode;
    int slots;              // ring slots
    int lds_xs, lds_res, lds_xres, lds_ctl;  // LDS byte offsets (the ring is at 0)
};
using EsA = const __attribute__((address_space(4))) EsArgs;

// ---------------------------------------------------------------- memory helpers
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* es_gp(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}
__device__ __forceinline__ float es_ld(const float* p) {  // sc1 (L2-coherent) 4-byte load
    return __hip_atomic_load(es_gp(const_cast<float*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void es_st(float* p, float v) {  // sc1 (write-through) 4-byte store
    __hip_atomic_store(es_gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t es_rsrc(const void* p, unsigned bytes) {
    const uint64_t u = (uint64_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, __builtin_amdgcn_readfirstlane(bytes),
                                             0x00020000);
}
__device__ __forceinline__ float4 es_ld4(__amdgpu_buffer_rsrc_t rs, unsigned off) {  // sc1 16-byte load
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /* sc1 */));
}
__device__ __forceinline__ float2 es_ld2(__amdgpu_buffer_rsrc_t rs, unsigned off) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 16));
}
template <typename T>
__device__ __forceinline__ float es_ldt(const T* p, size_t i) {  // one table element (static data: plain)
    if constexpr (sizeof(T) == 2) {
        return __half2float(__ushort_as_half(es_gp(reinterpret_cast<const unsigned short*>(p))[i]));
    } else if constexpr (sizeof(T) == 1) {
        return (float)(int)es_gp(reinterpret_cast<const int8_t*>(p))[i];
    } else {
        return es_gp(reinterpret_cast<const float*>(p))[i];
    }
}
template <typename T>
__device__ __forceinline__ void es_stt(T* p, size_t i, float v) {  // K/V cache element (plain: read next launch)
    if constexpr (sizeof(T) == 2) {
        es_gp(reinterpret_cast<unsigned short*>(p))[i] = __half_as_ushort(__float2half_rn(v));
    } else {
        es_gp(reinterpret_cast<float*>(p))[i] = v;
    }
}
template <typename T>
__device__ __forceinline__ float es_round(float v) {  // the cache type's rounding, as the attention reads it
    if constexpr (sizeof(T) == 2) return __half2float(__float2half_rn(v));
    return v;
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ unsigned lds_ld_acq(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st_rel(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned lds_add(unsigned* p, unsigned v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One LDS-DMA wave-instruction: lane i's 16 bytes at gsrc land at LDS byte address lds + 16 i. Inline asm so
// the compiler neither counts it nor drains it before the loader's own LDS accesses (cdna_hip_programming.md
// §5.7: M0 written in the same statement; the loader counts its vmcnt itself).
__device__ __forceinline__ void es_dma(const void* gsrc, unsigned lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds)
        : "memory");
}
template <int N>
__device__ __forceinline__ void es_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void es_stamp(EsA& a, int op, int k) {
    if (a.stamps) a.stamps[((size_t)op * gridDim.x + blockIdx.x) * 4 + k] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ void es_fail(EsA& a, unsigned* ctl) {
    __hip_atomic_fetch_or(es_gp(&a.st->error), kEsErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds_st_rel(ctl + kEsAbort, 1u);
}

// ---------------------------------------------------------------- op geometry (shared by loader and consumers)
// A GEMV op: NU units of R rows; CU b owns units [b*NU/grid, (b+1)*NU/grid); its rows stream in groups of
// kEsNC rows (kEsNC/R units), each group in P = ceil(nvec/128) pieces = slots.
struct EsGemv {
    const char* W;
    size_t row_bytes;
    int nvec;   // 16-byte vectors per row
    int nu, R;  // units, rows per unit
    int kind;   // row map: 0 plain (unit u = rows u*R ..), 1 qkv RoPE pairs, 2 gate/up pairs
    int half, inter;  // qkv: hd/2; gate/up: Il
    int u0, u1;
    __device__ int pieces() const { return (nvec + kEsPiece - 1) / kEsPiece; }
    __device__ int groups() const { return (u1 - u0) * R > 0 ? ((u1 - u0) * R + kEsNC - 1) / kEsNC : 0; }
    __device__ int row(int u, int r) const {
        if (kind == 1) {
            const int uh = u / half, d = u - uh * half;
            return uh * 2 * half + d + r * half;
        }
        if (kind == 2) return u + r * inter;
        return u * R + r;
    }
    // row of consumer slot c of group g, or -1 (padding)
    __device__ int group_row(int g, int c) const {
        const int u = u0 + g * (kEsNC / R) + c / R;
        return u < u1 ? row(u, c % R) : -1;
    }
};

template <typename WT>
__device__ __forceinline__ EsGemv es_gemv(EsA& a, int op) {
    EsGemv g{};
    const int D = a.D;
    if (op == kEsOpsPerLayer * a.L) {  // tied LM head: rows [v_lo, v_lo + v_n) of the embedding
        g.W = (const char*)a.emb + (size_t)a.v_lo * D * sizeof(WT);
        g.row_bytes = (size_t)D * sizeof(WT);
        g.nvec = D * (int)sizeof(WT) / 16;
        g.nu = a.v_n;
        g.R = 1;
        g.kind = 0;
    } else {
        const int l = op / kEsOpsPerLayer, k = op - l * kEsOpsPerLayer;
        const __attribute__((address_space(4))) EsLayer& w = ((const __attribute__((address_space(4))) EsLayer*)a.layers)[l];
        int cols = D;
        switch (k) {
            case kEsQkv:
                g.W = (const char*)w.qkv;
                g.nu = (a.hq + 2 * a.hkv) * (a.hd / 2);
                g.R = 2;
                g.kind = 1;
                g.half = a.hd / 2;
                break;
            case kEsWo:
                g.W = (const char*)w.wo;
                cols = a.hq * a.hd;
                g.nu = D;
                g.R = 1;
                break;
            case kEsGu:
                g.W = (const char*)w.gu;
                g.nu = a.Il;
                g.R = 2;
                g.kind = 2;
                g.inter = a.Il;
                break;
            default:
                g.W = (const char*)w.down;
                cols = a.Il;
                g.nu = D;
                g.R = 1;
                break;
        }
        g.row_bytes = (size_t)cols * sizeof(WT);
        g.nvec = cols * (int)sizeof(WT) / 16;
    }
    g.u0 = (int)(((long long)blockIdx.x * g.nu) / gridDim.x);
    g.u1 = (int)(((long long)(blockIdx.x + 1) * g.nu) / gridDim.x);
    return g;
}

// Attention geometry: a slot holds PPS positions of one kv head's K (or V) rows; a job = (kv head, split of
// ppj positions) = ppj / PPS slot pairs (K then V); job j of the layer is CU j's (at most one per CU).
template <typename KT, int HD>
struct EsAttnGeo {
    static constexpr int EPV = Vec16<KT>::N;           // elements per 16-byte vector
    static constexpr int RB = HD * (int)sizeof(KT);    // bytes per cached row
    static constexpr int LPR = RB / 16;                // lanes per row
    static constexpr int RPI = 64 / LPR;               // rows per wave-instruction (1 KiB)
    static constexpr int PPS = kEsSlot / RB;           // positions per slot
    static constexpr int PPW = PPS / kEsNC;            // positions per consumer wave per slot (= 2 * RPI)
    static_assert(PPW == 2 * RPI, "two 16-byte vectors per lane per slot");
};

__device__ __forceinline__ int es_nsplit(EsA& a, int pos) { return min(pos / a.ppj + 1, a.max_splits); }

// ---------------------------------------------------------------- the loader (wave 0)
struct EsLoader {
    unsigned ring;   // LDS byte address of slot 0
    unsigned* ctl;
    int S;
    unsigned n = 0;    // slots issued
    unsigned pub = 0;  // slots published (landed and announced)
    __device__ void publish_landed_all() {
        es_wait_vm<0>();
        while (pub < n) {
            lds_st_rel(ctl + kEsFull + pub % S, pub / S + 1);
            ++pub;
        }
    }
    // the slot for fill n is free (every consumer wave released fill n - S); false: abort
    __device__ bool acquire() {
        if (n < (unsigned)S) return true;
        const unsigned k = n % S, need = kEsNC * (n / S);
        if (lds_ld_acq(ctl + kEsFree + k) >= need) return true;
        publish_landed_all();  // never block with landed slots unannounced
        for (unsigned spin = 0;; ++spin) {
            if (lds_ld_acq(ctl + kEsFree + k) >= need) return true;
            if (lds_ld_acq(ctl + kEsAbort) != 0u || spin >= kEsSpin) return false;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __device__ unsigned slot_lds() const { return ring + (n % S) * kEsSlot; }
    // after the 16 DMA of slot n: keep kEsAhead slots in flight, announce the older ones
    __device__ void issued() {
        ++n;
        if (n - pub > (unsigned)kEsAhead) {
            es_wait_vm<16 * kEsAhead>();
            while (n - pub > (unsigned)kEsAhead) {
                lds_st_rel(ctl + kEsFull + pub % S, pub / S + 1);
                ++pub;
            }
        }
    }
};

template <typename WT>
__device__ __forceinline__ bool es_load_gemv(EsA& a, EsLoader& ld, int op) {
    const EsGemv g = es_gemv<WT>(a, op);
    const int lane = threadIdx.x & 63;
    const int P = g.pieces(), G = g.groups();
    const char* zero = (const char*)a.zero + lane * 16;
    for (int gi = 0; gi < G; ++gi) {
        int rows[kEsNC];
#pragma unroll
        for (int c = 0; c < kEsNC; ++c) rows[c] = g.group_row(gi, c);
        for (int p = 0; p < P; ++p) {
            if (!ld.acquire()) return false;
            const unsigned dst = ld.slot_lds();
#pragma unroll
            for (int c = 0; c < kEsNC; ++c) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int j = p * kEsPiece + h * 64 + lane;
                    const char* src = (rows[c] >= 0 && j < g.nvec) ? g.W + (size_t)rows[c] * g.row_bytes + (size_t)j * 16 : zero;
                    es_dma(src, dst + c * 2048 + h * 1024);
                }
            }
            ld.issued();
        }
    }
    return true;
}

template <typename KT, int HD>
__device__ __forceinline__ bool es_load_attn(EsA& a, EsLoader& ld, int l, int pos) {
    using Geo = EsAttnGeo<KT, HD>;
    const int lane = threadIdx.x & 63;
    const int job = blockIdx.x, nsplit = es_nsplit(a, pos);
    if (job >= a.hkv * nsplit) return true;
    const int kvh = job / nsplit, split = job - kvh * nsplit;
    const size_t head = ((size_t)l * a.hkv + kvh) * a.T;
    const char* zero = (const char*)a.zero + lane * 16;
    const int sp = a.ppj / Geo::PPS;
    for (int s = 0; s < sp; ++s) {
        const int t_slot = split * a.ppj + s * Geo::PPS;
        for (int kv = 0; kv < 2; ++kv) {
            const char* base = (const char*)(kv ? a.vc : a.kc) + head * Geo::RB;
            if (!ld.acquire()) return false;
            const unsigned dst = ld.slot_lds();
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = t_slot + i * Geo::RPI + lane / Geo::LPR;  // rows past pos are never read
                const char* src = t <= pos ? base + (size_t)t * Geo::RB + (lane % Geo::LPR) * 16 : zero;
                es_dma(src, dst + i * 1024);
            }
            ld.issued();
        }
    }
    return true;
}

template <typename WT, typename KT, int HD>
__device__ __forceinline__ void es_loader(EsA& a, unsigned* ctl, unsigned ring, int pos) {
    EsLoader ld{ring, ctl, a.slots};
    const int nops = kEsOpsPerLayer * a.L + 1;
    bool ok = true;
    for (int op = 0; ok && op < nops; ++op) {
        const int l = op / kEsOpsPerLayer;
        if (op < nops - 1 && op - l * kEsOpsPerLayer == kEsAttn)
            ok = es_load_attn<KT, HD>(a, ld, l, pos);
        else
            ok = es_load_gemv<WT>(a, ld, op);
    }
    ld.publish_landed_all();  // (also drains every DMA before the wave ends)
}

// ---------------------------------------------------------------- consumer side
struct EsCons {
    unsigned* ctl;
    const char* ring;
    int S;
    int c;            // consumer wave 0 .. kEsNC-1
    unsigned n = 0;   // slots consumed
    unsigned cb = 0;  // consumer barriers passed
    // wait until slot n has landed; false: abort
    __device__ bool wait_full(unsigned& k) {
        k = n % S;
        const unsigned need = n / S + 1;
        for (unsigned spin = 0;; ++spin) {
            if (lds_ld_acq(ctl + kEsFull + k) >= need) return true;
            if (lds_ld_acq(ctl + kEsAbort) != 0u || spin >= kEsSpin) return false;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    // the wave's reads of slot n are complete (the caller waited lgkmcnt(0)): hand it back to the loader
    __device__ void release(unsigned k) {
        if ((threadIdx.x & 63) == 0) lds_add(ctl + kEsFree + k, 1u);
        ++n;
    }
    // all consumer waves (never the loader)
    __device__ bool barrier() {
        ++cb;
        if ((threadIdx.x & 63) == 0) lds_add(ctl + kEsCbar, 1u);
        const unsigned need = cb * kEsNC;
        for (unsigned spin = 0;; ++spin) {
            if (lds_ld_acq(ctl + kEsCbar) >= need) return true;
            if (lds_ld_acq(ctl + kEsAbort) != 0u || spin >= kEsSpin) return false;
            __builtin_amdgcn_s_sleep(1);
        }
    }
};

// Edge o (op o's outputs on every CU): consumer wave 0 polls the 8 shards (sc1), then announces it in LDS; the
// other consumer waves wait for the announcement. false: abort.
__device__ __forceinline__ bool es_wait_edge(EsA& a, EsCons& cs, int e) {
    const int lane = threadIdx.x & 63;
    if (cs.c == 0) {
        const int sh = lane & (kEsShards - 1);
        const unsigned need = (gridDim.x - sh + kEsShards - 1) / kEsShards;
        const unsigned* w = a.edges + ((size_t)e * kEsShards + sh) * kEsShardWords;
        for (unsigned spin = 0;; ++spin) {
            const unsigned v = __hip_atomic_load(es_gp(const_cast<unsigned*>(w)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_ballot_w64(v < need) == 0ull) break;
            if (lds_ld_acq(cs.ctl + kEsAbort) != 0u) return false;
            if (spin >= kEsSpin) {
                if (lane == 0) es_fail(a, cs.ctl);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0) lds_st_rel(cs.ctl + kEsEdgeSeen, (unsigned)e + 1);
        return true;
    }
    for (unsigned spin = 0;; ++spin) {
        if (lds_ld_acq(cs.ctl + kEsEdgeSeen) >= (unsigned)e + 1) return true;
        if (lds_ld_acq(cs.ctl + kEsAbort) != 0u || spin >= kEsSpin) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

// The calling wave has stored (sc1) everything this CU publishes for edge e: drain, then ONE add to this CU's
// shard (the only storing wave is the caller, so its own drain covers every byte of the hand-off).
__device__ __forceinline__ void es_arrive(EsA& a, int e) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) {
        unsigned* w = a.edges + ((size_t)e * kEsShards + (blockIdx.x % kEsShards)) * kEsShardWords;
        __hip_atomic_fetch_add(es_gp(w), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// This wave is done with op o's rows (its LDS results written): true in the wave that finished LAST (it runs
// the op's epilogue; the others move on).
__device__ __forceinline__ bool es_rows_done(EsCons& cs, int o) {
    unsigned prev = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) prev = lds_add(cs.ctl + kEsResDone, 1u);
    prev = __builtin_amdgcn_readfirstlane(prev);
    return prev == (unsigned)(kEsNC * (o + 1) - 1);
}

// ---- input staging: x (fp32, [cols]) into the LDS image xs, optionally times the norm weight w; the sum of
// squares of x over the whole vector is returned (every consumer wave gets the same value). The vector is split
// over the consumer waves in float4s; sc1 loads (a handed-off vector) or plain (the embedding row).
__device__ __forceinline__ float es_inv_rms(float ss, int cols, float eps) {
    const float tep = ss / (float)cols;   // rms_kernel.cpp:17
    const float rms = sqrtf(tep + eps);  // :18
    return 1.0f / rms;                   // :19
}

template <bool NORM>
__device__ __forceinline__ bool es_stage(EsCons& cs, float* xs, const float* x, const float* w, int cols, float* ss_out) {
    const int t = cs.c * 64 + (threadIdx.x & 63), nt = kEsNC * 64, n4 = cols >> 2;
    const auto rs = es_rsrc(x, (unsigned)(sizeof(float) * cols));
    float ss = 0.0f;
    constexpr int B = 4;
    for (int f0 = 0; f0 < n4; f0 += nt * B) {
        float4 v[B], wv[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int f = f0 + t + j * nt;
            v[j] = es_ld4(rs, (unsigned)(16 * f));  // past the end: 0 (buffer range check)
            if constexpr (NORM) wv[j] = reinterpret_cast<const float4*>(w)[min(f, n4 - 1)];
        }
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int f = f0 + t + j * nt;
            ss += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
            if (f < n4) {
                float4 o = v[j];
                if constexpr (NORM) o = make_float4(o.x * wv[j].x, o.y * wv[j].y, o.z * wv[j].z, o.w * wv[j].w);
                reinterpret_cast<float4*>(xs)[f] = o;
            }
        }
    }
    if constexpr (NORM) {
        ss = wave_sum(ss);
        if ((threadIdx.x & 63) == 0) reinterpret_cast<float*>(cs.ctl + kEsSumSq)[cs.c] = ss;
    }
    if (!cs.barrier()) return false;
    if constexpr (NORM) {
        float tot = 0.0f;
#pragma unroll
        for (int i = 0; i < kEsNC; ++i) tot += reinterpret_cast<const float*>(cs.ctl + kEsSumSq)[i];
        *ss_out = tot;
    }
    return true;
}

// ---- GEMV consumption: every row of this CU's share, one row per wave per group, 2 vectors per lane per slot.
// Row sums (unscaled) go to res[local row].
template <typename WT>
__device__ __forceinline__ bool es_consume_gemv(EsCons& cs, const EsGemv& g, const float* xs, float* res) {
    constexpr int EPV = Vec16<WT>::N;
    const int lane = threadIdx.x & 63;
    const int P = g.pieces(), G = g.groups();
    for (int gi = 0; gi < G; ++gi) {
        const int row = g.group_row(gi, cs.c);
        float acc = 0.0f;
        for (int p = 0; p < P; ++p) {
            const int j0 = p * kEsPiece + lane, j1 = j0 + 64;
            // x for this lane's two vectors first (independent of the slot)
            float x0[EPV], x1[EPV];
            {
                const float4* xp0 = reinterpret_cast<const float4*>(xs) + (size_t)min(j0, g.nvec - 1) * (EPV / 4);
                const float4* xp1 = reinterpret_cast<const float4*>(xs) + (size_t)min(j1, g.nvec - 1) * (EPV / 4);
#pragma unroll
                for (int e = 0; e < EPV / 4; ++e) {
                    const float4 a0 = xp0[e], a1 = xp1[e];
                    x0[4 * e] = a0.x, x0[4 * e + 1] = a0.y, x0[4 * e + 2] = a0.z, x0[4 * e + 3] = a0.w;
                    x1[4 * e] = a1.x, x1[4 * e + 1] = a1.y, x1[4 * e + 2] = a1.z, x1[4 * e + 3] = a1.w;
                }
            }
            unsigned k;
            if (!cs.wait_full(k)) return false;
            const char* sl = cs.ring + (size_t)k * kEsSlot + cs.c * 2048 + lane * 16;
            const u32x4 w0 = *reinterpret_cast<const u32x4*>(sl);
            const u32x4 w1 = *reinterpret_cast<const u32x4*>(sl + 1024);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            cs.release(k);
            float wf[EPV];
            Vec16<WT>::unpack(w0, wf);
            float d0 = 0.0f, d1 = 0.0f;
#pragma unroll
            for (int e = 0; e < EPV; ++e) d0 = fmaf(wf[e], x0[e], d0);
            Vec16<WT>::unpack(w1, wf);
#pragma unroll
            for (int e = 0; e < EPV; ++e) d1 = fmaf(wf[e], x1[e], d1);
            acc += (j0 < g.nvec ? d0 : 0.0f) + (j1 < g.nvec ? d1 : 0.0f);
        }
        acc = wave_sum(acc);
        if (lane == 0 && row >= 0) res[gi * kEsNC + cs.c] = acc;  // local row index: group-major
    }
    return true;
}

// local result of unit u (relative to u0), row r: the group-major slot the consumer wrote
__device__ __forceinline__ float es_res(const float* res, const EsGemv& g, int ul, int r) {
    const int lr = ul * g.R + r;  // consumer slot = local row in group-major order
    return res[lr];
}

// ---- attention consumption (mha_kernel.cpp:36-77 semantics: s_t = (q . K_t) * scale for t <= pos, softmax,
// o = sum_t p_t V_t), online softmax per wave over its positions of every slot; the wave's (o, m, l) per q
// head of the kv-head group go to the LDS scratch [kEsNC][G][HD + 2] (lanes of row group 0).
template <typename KT, int HD, int G>
__device__ __forceinline__ bool es_consume_attn(EsA& a, EsCons& cs, int l, int pos, int kvh, int split,
                                                float* scratch) {
    using Geo = EsAttnGeo<KT, HD>;
    constexpr int EPV = Geo::EPV, LPR = Geo::LPR, RPI = Geo::RPI, PPS = Geo::PPS;
    const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane - sub * LPR;
    const float* q = a.qv + (size_t)l * a.hq * HD;
    const float* kn = a.kvn + (size_t)l * 2 * a.hkv * HD + (size_t)kvh * HD;
    const float* vn = kn + (size_t)a.hkv * HD;
    float qf[G][EPV], knf[EPV], vnf[EPV];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < EPV; ++e) qf[g][e] = es_ld(q + (size_t)(kvh * G + g) * HD + li * EPV + e);
#pragma unroll
    for (int e = 0; e < EPV; ++e) {
        knf[e] = es_ld(kn + li * EPV + e);
        vnf[e] = es_ld(vn + li * EPV + e);
    }
    float m[G], ls[G], o[G][EPV];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        m[g] = -INFINITY;
        ls[g] = 0.0f;
#pragma unroll
        for (int e = 0; e < EPV; ++e) o[g][e] = 0.0f;
    }
    const int sp = a.ppj / PPS;
    for (int s = 0; s < sp; ++s) {
        const int tw = split * a.ppj + s * PPS + cs.c * (2 * RPI) + sub;  // vector i: position tw + i * RPI
        unsigned k;
        if (!cs.wait_full(k)) return false;
        const char* sl = cs.ring + (size_t)k * kEsSlot + cs.c * 2048 + lane * 16;
        u32x4 kr[2] = {*reinterpret_cast<const u32x4*>(sl), *reinterpret_cast<const u32x4*>(sl + 1024)};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        cs.release(k);
        float sc[2][G];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = tw + i * RPI;
            float kf[EPV];
            Vec16<KT>::unpack(kr[i], kf);
#pragma unroll
            for (int e = 0; e < EPV; ++e) kf[e] = t == pos ? knf[e] : kf[e];  // this step's row: the hand-off
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float d = 0.0f;
#pragma unroll
                for (int e = 0; e < EPV; ++e) d = fmaf(qf[g][e], kf[e], d);
                d = group_sum<LPR>(d);
                sc[i][g] = t <= pos ? d * a.scale : -INFINITY;  // mha_kernel.cpp:51-60 (sum * scale)
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float mx = stride_max<LPR>(fmaxf(sc[0][g], sc[1][g]));
            const float mn = fmaxf(m[g], mx);
            const float corr = mn == -INFINITY ? 1.0f : expf(m[g] - mn);
            ls[g] *= corr;
#pragma unroll
            for (int e = 0; e < EPV; ++e) o[g][e] *= corr;
            m[g] = mn;
        }
        if (!cs.wait_full(k)) return false;
        sl = cs.ring + (size_t)k * kEsSlot + cs.c * 2048 + lane * 16;
        u32x4 vr[2] = {*reinterpret_cast<const u32x4*>(sl), *reinterpret_cast<const u32x4*>(sl + 1024)};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        cs.release(k);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = tw + i * RPI;
            float vf[EPV];
            Vec16<KT>::unpack(vr[i], vf);
#pragma unroll
            for (int e = 0; e < EPV; ++e) vf[e] = t == pos ? vnf[e] : vf[e];
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const float p = t <= pos ? expf(sc[i][g] - m[g]) : 0.0f;
                ls[g] += p;
#pragma unroll
                for (int e = 0; e < EPV; ++e) o[g][e] = fmaf(p, vf[e], o[g][e]);
            }
        }
    }
    // every lane of a row holds the same p: reduce across the row groups only
#pragma unroll
    for (int g = 0; g < G; ++g) {
        ls[g] = stride_sum<LPR>(ls[g]);
#pragma unroll
        for (int e = 0; e < EPV; ++e) o[g][e] = stride_sum<LPR>(o[g][e]);
    }
    if (sub == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float* row = scratch + ((size_t)cs.c * G + g) * (HD + 2);
#pragma unroll
            for (int e = 0; e < EPV; ++e) row[li * EPV + e] = o[g][e];
            if (li == 0) {
                row[HD] = m[g];
                row[HD + 1] = ls[g];
            }
        }
    }
    return true;
}

// the job's partial: the consumer waves' states merged in wave order, published (sc1) for the wo staging
template <int HD, int G>
__device__ __forceinline__ void es_attn_publish(EsA& a, int l, int kvh, int split, const float* scratch) {
    const int lane = threadIdx.x & 63;
    for (int i = lane; i < G * HD; i += 64) {
        const int g = i / HD, d = i - g * HD;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < kEsNC; ++w) M = fmaxf(M, scratch[((size_t)w * G + g) * (HD + 2) + HD]);
        float ov = 0.0f, L = 0.0f;
#pragma unroll
        for (int w = 0; w < kEsNC; ++w) {
            const float* row = scratch + ((size_t)w * G + g) * (HD + 2);
            const float cw = expf(row[HD] - M);  // a wave without live positions: m = -inf -> 0
            ov = fmaf(cw, row[d], ov);
            L = fmaf(cw, row[HD + 1], L);
        }
        float* dst = a.part + (((size_t)l * a.hq + kvh * G + g) * a.max_splits + split) * (HD + kAttnPartPad);
        es_st(dst + d, ov);
        if (d == 0) {
            es_st(dst + HD, M);
            es_st(dst + HD + 1, L);
        }
    }
}

// wo's input: every q head's job partials merged in split order (M = max m_s, out = sum e^{m_s-M} o_s /
// sum e^{m_s-M} l_s: the launch path's attn_merge arithmetic), by all consumer waves, into xs
template <int HD>
__device__ __forceinline__ bool es_stage_merge(EsA& a, EsCons& cs, int l, int pos, float* xs) {
    constexpr int PS = HD + kAttnPartPad, NSB = 8;
    const int t = cs.c * 64 + (threadIdx.x & 63), nt = kEsNC * 64;
    const int n4 = a.hq * HD / 4, ns = es_nsplit(a, pos);
    const float* base = a.part + (size_t)l * a.hq * a.max_splits * PS;
    const auto rs = es_rsrc(base, (unsigned)(sizeof(float) * (size_t)a.hq * a.max_splits * PS));
    for (int f = t; f < n4; f += nt) {
        const int h = f / (HD / 4), d4 = f - h * (HD / 4);
        const unsigned row0 = (unsigned)(h * a.max_splits) * PS;
        float M = -INFINITY;
        float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float L = 0.0f;
        for (int s0 = 0; s0 < ns; s0 += NSB) {
            float2 ml[NSB];
            float4 ov[NSB];
#pragma unroll
            for (int j = 0; j < NSB; ++j) {
                const unsigned r = row0 + (unsigned)min(s0 + j, ns - 1) * PS;
                ml[j] = es_ld2(rs, 4u * (r + HD));
                ov[j] = es_ld4(rs, 4u * r + 16u * d4);
            }
            float Mb = M;
#pragma unroll
            for (int j = 0; j < NSB; ++j)
                if (s0 + j < ns) Mb = fmaxf(Mb, ml[j].x);
            if (Mb != M) {  // rescale what has been summed so far (a later batch raised the max)
                const float cr = M == -INFINITY ? 0.0f : expf(M - Mb);
                acc = make_float4(acc.x * cr, acc.y * cr, acc.z * cr, acc.w * cr);
                L *= cr;
                M = Mb;
            }
#pragma unroll
            for (int j = 0; j < NSB; ++j) {
                if (s0 + j < ns) {
                    const float w = expf(ml[j].x - M);
                    acc.x = fmaf(w, ov[j].x, acc.x);
                    acc.y = fmaf(w, ov[j].y, acc.y);
                    acc.z = fmaf(w, ov[j].z, acc.z);
                    acc.w = fmaf(w, ov[j].w, acc.w);
                    L = fmaf(w, ml[j].y, L);
                }
            }
        }
        reinterpret_cast<float4*>(xs)[f] = make_float4(acc.x / L, acc.y / L, acc.z / L, acc.w / L);
    }
    return cs.barrier();
}

// ---------------------------------------------------------------- epilogues (the op's last consumer wave)
// Fused q/k/v + RoPE (rope_kernel.cpp:30-38) + K/V: the cache row (plain: read by later launches) and this
// step's rows for the attention (sc1, rounded to the cache type as the attention reads the cache).
template <typename KT>
__device__ __forceinline__ void es_epi_qkv(EsA& a, const EsGemv& g, const float* res, int l, int pos, float inv) {
    const int lane = threadIdx.x & 63, half = a.hd / 2;
    const float* rs = ((const __attribute__((address_space(4))) EsLayer*)a.layers)[l].qkv_s;
    float* q = a.qv + (size_t)l * a.hq * a.hd;
    float* kn = a.kvn + (size_t)l * 2 * a.hkv * a.hd;
    KT* kc = (KT*)a.kc + (size_t)l * a.hkv * a.T * a.hd;
    KT* vc = (KT*)a.vc + (size_t)l * a.hkv * a.T * a.hd;
    for (int ul = lane; ul < g.u1 - g.u0; ul += 64) {
        const int u = g.u0 + ul, uh = u / half, d = u - uh * half;
        const int r0 = uh * a.hd + d, r1 = r0 + half;
        float a0 = res[2 * ul] * inv, a1 = res[2 * ul + 1] * inv;
        if (rs) {
            a0 *= rs[r0];
            a1 *= rs[r1];
        }
        if (uh < a.hq + a.hkv) {
            const float fci = a.sin_t[pos * half + d], fcr = a.cos_t[pos * half + d];
            const float x0 = a0 * fcr - a1 * fci;
            const float x1 = a1 * fcr + a0 * fci;
            if (uh < a.hq) {
                es_st(q + (size_t)uh * a.hd + d, x0);
                es_st(q + (size_t)uh * a.hd + d + half, x1);
            } else {
                const int h = uh - a.hq;
                KT* kr = kc + ((size_t)h * a.T + pos) * a.hd;
                es_stt(kr, d, x0);
                es_stt(kr, d + half, x1);
                es_st(kn + (size_t)h * a.hd + d, es_round<KT>(x0));
                es_st(kn + (size_t)h * a.hd + d + half, es_round<KT>(x1));
            }
        } else {
            const int h = uh - a.hq - a.hkv;
            KT* vr = vc + ((size_t)h * a.T + pos) * a.hd;
            es_stt(vr, d, a0);
            es_stt(vr, d + half, a1);
            float* vn = kn + (size_t)a.hkv * a.hd;
            es_st(vn + (size_t)h * a.hd + d, es_round<KT>(a0));
            es_st(vn + (size_t)h * a.hd + d + half, es_round<KT>(a1));
        }
    }
}

// act = sigmoid(g) * u (swiglu_kernel.cpp:12-13) or SiLU(g) * u
__device__ __forceinline__ void es_epi_gu(EsA& a, const EsGemv& g, const float* res, int l, float inv) {
    const int lane = threadIdx.x & 63;
    const float* rs = ((const __attribute__((address_space(4))) EsLayer*)a.layers)[l].gu_s;
    float* act = a.actv + (size_t)l * a.Il;
    for (int ul = lane; ul < g.u1 - g.u0; ul += 64) {
        const int u = g.u0 + ul;
        float gv = res[2 * ul] * inv, up = res[2 * ul + 1] * inv;
        if (rs) {
            gv *= rs[u];
            up *= rs[a.Il + u];
        }
        float t = 1.0f / (1.0f + expf(-gv));
        if (a.act_mode) t = gv * t;
        es_st(act + u, t * up);
    }
}

// y[row] = resid[row] + sum * rscale[row] (matmul_kernel.cpp:26 + add_kernel.cpp:5-14); the CU's rows of the
// residual stream live in LDS (xres): wo and down own the same rows on every CU
__device__ __forceinline__ void es_epi_resid(const EsGemv& g, const float* res, const float* rs, float* xres, float* y) {
    const int lane = threadIdx.x & 63;
    for (int ul = lane; ul < g.u1 - g.u0; ul += 64) {
        const int u = g.u0 + ul;
        const float v = rs ? res[ul] * rs[u] : res[ul];
        const float x = xres[ul] + v;
        xres[ul] = x;
        es_st(y + u, x);
    }
}

// tied LM head (model.cpp:136-139) + the argmax: logits (plain: read by the host), this CU's max key (sc1);
// the last CU to arrive reduces every CU's key and advances the decode state (model.cpp:157-183)
__device__ __forceinline__ void es_epi_lm(EsA& a, const EsGemv& g, const float* res, float inv) {
    const int lane = threadIdx.x & 63;
    unsigned long long best = 0;
    for (int ul = lane; ul < g.u1 - g.u0; ul += 64) {
        const int u = g.u0 + ul;
        float v = res[ul] * inv;
        if (a.emb_s) v *= a.emb_s[a.v_lo + u];
        a.logits[u] = v;
        const unsigned long long k = argmax_key(v, (unsigned)(a.v_lo + u));
        best = k > best ? k : best;
    }
    best = wave_max_u64(best);
    if (lane == 0)
        __hip_atomic_store(es_gp(a.keys + blockIdx.x), best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned prev = 0;
    if (lane == 0) {
        unsigned* w = a.edges + (size_t)kEsOpsPerLayer * a.L * kEsShards * kEsShardWords;
        prev = __hip_atomic_fetch_add(es_gp(w), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev != gridDim.x - 1) return;
    unsigned long long b = 0;
    for (int i = lane; i < (int)gridDim.x; i += 64) {
        const unsigned long long k =
            __hip_atomic_load(es_gp(a.keys + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        b = k > b ? k : b;
    }
    b = wave_max_u64(b);
    if (lane == 0) {
        a.st->key = b;
        finalize_state(a.st, a.prompt, a.hist, a.T);
    }
}

// ---------------------------------------------------------------- the consumer waves' op loop
template <typename WT, typename KT, int HD, int G>
__device__ __forceinline__ void es_consumer(EsA& a, unsigned* ctl, char* smem, int c, int pos, int token) {
    EsCons cs{ctl, smem, a.slots, c};
    float* xs = reinterpret_cast<float*>(smem + a.lds_xs);
    float* res = reinterpret_cast<float*>(smem + a.lds_res);
    float* xres = reinterpret_cast<float*>(smem + a.lds_xres);
    const int D = a.D, lane = threadIdx.x & 63;
    const int t = c * 64 + lane, nt = kEsNC * 64;
    // layer 0's input: the embedding row (emb_kernel.cpp:4-21; token on the device, a static table: no edge),
    // staged as x * w_norm0 with its sum of squares, and this CU's rows of the residual stream
    float inv = 0.0f;
    {
        const bool ok = token >= 0 && token < a.V;
        const float s = (ok && a.emb_s) ? a.emb_s[token] : 1.0f;
        const WT* row = (const WT*)a.emb + (size_t)(ok ? token : 0) * D;
        float ss = 0.0f;
        for (int i = t; i < D; i += nt) {
            const float x = ok ? es_ldt(row, i) * s : __builtin_nanf("");
            ss += x * x;
            xs[i] = x * a.norms[i];
        }
        ss = wave_sum(ss);
        if (lane == 0) reinterpret_cast<float*>(ctl + kEsSumSq)[c] = ss;
        const int r0 = (int)(((long long)blockIdx.x * D) / gridDim.x), r1 = (int)(((long long)(blockIdx.x + 1) * D) / gridDim.x);
        for (int i = r0 + t; i < r1; i += nt) xres[i - r0] = ok ? es_ldt(row, i) * s : __builtin_nanf("");
        if (!cs.barrier()) return;
        float tot = 0.0f;
#pragma unroll
        for (int i = 0; i < kEsNC; ++i) tot += reinterpret_cast<const float*>(ctl + kEsSumSq)[i];
        inv = es_inv_rms(tot, D, a.eps);
    }
    const int nops = kEsOpsPerLayer * a.L + 1;
    for (int op = 0; op < nops; ++op) {
        const int l = op / kEsOpsPerLayer, k = op - l * kEsOpsPerLayer;
        const bool lm = op == nops - 1;
        if (op > 0 && !es_wait_edge(a, cs, op - 1)) return;
        if (c == 0 && lane == 0) es_stamp(a, op, 0);
        if (!lm && k == kEsAttn) {
            const int nsplit = es_nsplit(a, pos), job = blockIdx.x;
            const bool has = job < a.hkv * nsplit;
            const int kvh = has ? job / nsplit : 0, split = has ? job - kvh * nsplit : 0;
            if (has && !es_consume_attn<KT, HD, G>(a, cs, l, pos, kvh, split, xs)) return;
            if (es_rows_done(cs, op)) {
                if (has) es_attn_publish<HD, G>(a, l, kvh, split, xs);
                es_arrive(a, op);
                if (lane == 0) es_stamp(a, op, 3);
            }
            continue;
        }
        // input staging
        float ss = 0.0f;
        bool ok = true;
        if (lm) {
            ok = es_stage<true>(cs, xs, a.xv + (size_t)(2 * a.L) * D, a.norms + (size_t)(2 * a.L) * D, D, &ss);
            inv = es_inv_rms(ss, D, a.eps);
        } else if (k == kEsQkv) {
            if (op > 0) {
                ok = es_stage<true>(cs, xs, a.xv + (size_t)(2 * l) * D, a.norms + (size_t)(2 * l) * D, D, &ss);
                inv = es_inv_rms(ss, D, a.eps);
            }
        } else if (k == kEsWo) {
            ok = es_stage_merge<HD>(a, cs, l, pos, xs);
        } else if (k == kEsGu) {
            ok = es_stage<true>(cs, xs, a.xv + (size_t)(2 * l + 1) * D, a.norms + (size_t)(2 * l + 1) * D, D, &ss);
            inv = es_inv_rms(ss, D, a.eps);
        } else {
            ok = es_stage<false>(cs, xs, a.actv + (size_t)l * a.Il, nullptr, a.Il, &ss);
        }
        if (!ok) return;
        if (c == 0 && lane == 0) es_stamp(a, op, 1);
        const EsGemv g = es_gemv<WT>(a, op);
        if (!es_consume_gemv<WT>(cs, g, xs, res)) return;
        if (!es_rows_done(cs, op)) continue;
        if (lane == 0) es_stamp(a, op, 2);
        const __attribute__((address_space(4))) EsLayer& w = ((const __attribute__((address_space(4))) EsLayer*)a.layers)[lm ? 0 : l];
        if (lm) {
            es_epi_lm(a, g, res, inv);
            return;
        }
        switch (k) {
            case kEsQkv: es_epi_qkv<KT>(a, g, res, l, pos, inv); break;
            case kEsWo: es_epi_resid(g, res, w.wo_s, xres, a.xv + (size_t)(2 * l + 1) * D); break;
            case kEsGu: es_epi_gu(a, g, res, l, inv); break;
            default: es_epi_resid(g, res, w.down_s, xres, a.xv + (size_t)(2 * l + 2) * D); break;
        }
        es_arrive(a, op);
        if (lane == 0) es_stamp(a, op, 3);
    }
}

// ---------------------------------------------------------------- the step
template <typename WT, typename KT, int HD, int G>
__global__ void __launch_bounds__(kEsThreads) es_step_kernel(const EsArgs* __restrict__ ap) {
    extern __shared__ __attribute__((aligned(1024))) char es_smem[];
    EsA& a = *(EsA*)ap;
    unsigned* ctl = reinterpret_cast<unsigned*>(es_smem + a.lds_ctl);
    if (threadIdx.x < kEsCtlWords) ctl[threadIdx.x] = 0u;
    __syncthreads();  // the only full-workgroup barrier: the loader never joins another one
    const __attribute__((address_space(4))) DevState* st = (const __attribute__((address_space(4))) DevState*)a.st;
    const int pos = st->pos, token = st->token;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (wave == 0)
        es_loader<WT, KT, HD>(a, ctl, lds_addr(es_smem), pos);
    else
        es_consumer<WT, KT, HD, G>(a, ctl, es_smem, wave - 1, pos, token);
}

}  // namespace sli
