// attn_wo.h — decode attention and the K-split wo projection as ONE launch (batch 1, TP 1; SLI_ATTN_WO=1).
//
// The reference runs mha then wo as separate ops (model.cpp:70-83). The launch path ran them as two kernels:
// attention (split-context partials, attention.h) and the wo GEMV, which merges the splits while staging its
// input (gemv.h XStageMerge / EpiKPart). Both stream from HBM — the K/V rows (C1: 33.5 MB per layer) and wo
// (33.5 MB fp16) — so between them sit the attention's tail, a kernel boundary and the wo launch's ramp,
// while wo's weights, which do not depend on the attention, wait. Here workgroup b of one launch:
//   1. runs the attention of its (kv head, context split), and right behind its K/V and q loads issues the
//      loads of its wo rows (attn_publish's pre hook), so the weight stream overlaps the attention;
//   2. publishes its partial write-through (sc1, drained) and adds one arrival to its head group's counter
//      (MI355X_MICROARCH.md hand-off table, row 1: one lane per storing workgroup, agent-scope add; the
//      consumer polls with sc1 loads, its other waves join a workgroup barrier, every load of the handed-off
//      bytes an sc1 load);
//   3. waits until every workgroup of ITS column block's head group has arrived (K-split wo: column block k
//      of wo is the input of heads [k hq / ks, (k + 1) hq / ks)), merges those heads' splits (XStageMerge's
//      arithmetic, split order) into LDS, and finishes its rows from the registers: part[k][d].
// The gate/up and down GEMVs consume part[][] exactly as after the unfused K-split wo (XStageSum /
// EpiStoreSum). Counters are 64-bit and monotonic (never reset; a launch adds group_wgs to every group's
// counter, so a workgroup reads the launch's epoch from its own add). Every wait is bounded (DevState::error
// bit kAwErrTimeout). The host launches it only when the grid fits the chip with one workgroup per CU, so
// every workgroup a wait depends on is resident.
#pragma once
#include "attention.h"
#include "common.h"

namespace sli {

constexpr int kAwErrTimeout = 8;  // DevState::error bit: a fused attention + wo wait gave up
constexpr int kAwThreads = 1024;  // attn_waves(1) == attn_waves(2) == 16

template <typename WT>
struct AttnWoArgs {
    const WT* wo;               // [D][QD]
    const float* wo_s;          // int8 row scales [D], or nullptr
    float* part;                // [ks][D]: column block k's row sums (EpiKPart's layout)
    unsigned long long* cnt;    // [ks] arrivals per head group, monotonic
    int* err;                   // &DevState::error
    int D, QD, ks;
    int heads_per_k;            // q heads per column block: hq / ks
    int group_wgs;              // arrivals per head group per launch: (hkv / ks) * max_splits
    int dbg = 0;                // SLI_DEBUG_AW bits (diagnosis): 1 weights after the publish, 2 x_k -> dbg_x,
                                // timing only (wrong results): 4 no wait, 8 no merge loads
    float* dbg_x = nullptr;     // [ks][QD / ks] merged inputs (dbg & 2)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t aw_rsrc(const void* p, unsigned bytes) {
    const uint64_t u = (uint64_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
    void* q = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, 0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ float4 aw_ld4(__amdgpu_buffer_rsrc_t rs, unsigned off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /* sc1 */));
}

// grid: n_kv_heads * max_splits workgroups (<= CUs) of 1024 threads; RW wo rows per wave, NVL 16-byte vectors
// of each row per lane (a row is QD / ks columns); dynamic LDS: QD / ks floats
template <typename KT, typename WT, int HD, int G, int RW, int NVL>
__global__ void __launch_bounds__(kAwThreads) attn_wo_kernel(AttnArgs<KT> a, AttnWoArgs<WT> w) {
    static_assert(attn_waves(G) == 16, "the fused launch runs 16-wave attention workgroups");
    extern __shared__ __attribute__((aligned(16))) float aw_x[];
    constexpr int EPV = Vec16<WT>::N;
    constexpr int SW = (G * HD + 63) / 64;  // waves that store the partial: their weight loads go after it
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int kvh = blockIdx.x / a.max_splits, split = blockIdx.x - kvh * a.max_splits;
    const int u0 = blockIdx.x * 16 * RW;  // this workgroup's K-split wo units (k-major: u = k D + d)
    const int k = u0 / w.D;               // its column block
    const int C = w.QD / w.ks;
    const size_t row_bytes = (size_t)w.QD * sizeof(WT);

    u32x4 wr[RW][NVL];
    auto issue = [&]() {
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int d = u0 + wave * RW + r - k * w.D;
            const char* base = reinterpret_cast<const char*>(w.wo) + (size_t)d * row_bytes + (size_t)k * C * sizeof(WT);
#pragma unroll
            for (int j = 0; j < NVL; ++j) wr[r][j] = load16<true>(base + (size_t)(lane + 64 * j) * 16);
        }
    };
    bool issued = false;
    const bool late = (w.dbg & 1) != 0;
    auto pre = [&]() {
        if (wave >= SW && !late) issue();
        issued = !late;
    };
    a.defer_merge = 3;
    attn_publish<KT, HD, G, 16, attn_late_v(G)>(a, kvh, split, pre);
    if (!issued || wave < SW) issue();  // the storing waves (or a workgroup past the live context): now

    // arrival + wait for column block k's head group
    __shared__ int aw_flag;
    if (threadIdx.x == 0) {
        const int g_att = (kvh * G) / w.heads_per_k;
        const unsigned long long old = __hip_atomic_fetch_add(w.cnt + g_att, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long target = (old / (unsigned long long)w.group_wgs + 1ull) * (unsigned long long)w.group_wgs;
        int ok = 1;
        for (unsigned spins = 0; !(w.dbg & 4) && __hip_atomic_load(w.cnt + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spins) {
            __builtin_amdgcn_s_sleep(1);
            if (spins > (1u << 22)) {
                __hip_atomic_fetch_or(w.err, kAwErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
        }
        aw_flag = ok;
    }
    __syncthreads();

    // merge column block k's heads (XStageMerge's arithmetic, split order), sc1 loads of the partials
    constexpr int PS = HD + kAttnPartPad;
    const int pos = attn_pos(a, kvh);
    const int ns = min(pos / AttnGeom<KT, HD>::PPWG + 1, a.max_splits);
    const int h0 = k * w.heads_per_k;
    const auto rs = aw_rsrc(a.part, (unsigned)(sizeof(float) * (size_t)(h0 + w.heads_per_k) * a.max_splits * PS));
    const int n4 = (w.dbg & 8) ? 0 : C >> 2;
    for (int f = threadIdx.x; f < n4; f += kAwThreads) {
        const int h = h0 + f / (HD / 4), d4 = f - (f / (HD / 4)) * (HD / 4);
        const unsigned row0 = (unsigned)(h * a.max_splits) * PS;
        float M = -INFINITY;
        for (int s0 = 0; s0 < ns; s0 += 8) {
            float4 ml[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) ml[j] = aw_ld4(rs, 4u * (row0 + (unsigned)min(s0 + j, ns - 1) * PS + HD));
#pragma unroll
            for (int j = 0; j < 8; ++j) M = fmaxf(M, ml[j].x);  // clamped duplicates leave the max
        }
        float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float L = 0.0f;
        for (int s0 = 0; s0 < ns; s0 += 8) {
            float4 ml[8], ov[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const unsigned r = row0 + (unsigned)min(s0 + j, ns - 1) * PS;
                ml[j] = aw_ld4(rs, 4u * (r + HD));
                ov[j] = aw_ld4(rs, 4u * (r + 4 * d4));
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (s0 + j < ns) {
                    const float c = expf(ml[j].x - M);
                    o.x = fmaf(c, ov[j].x, o.x);
                    o.y = fmaf(c, ov[j].y, o.y);
                    o.z = fmaf(c, ov[j].z, o.z);
                    o.w = fmaf(c, ov[j].w, o.w);
                    L = fmaf(c, ml[j].y, L);
                }
            }
        }
        reinterpret_cast<float4*>(aw_x)[f] = make_float4(o.x / L, o.y / L, o.z / L, o.w / L);
        if ((w.dbg & 2) && (blockIdx.x % (gridDim.x / w.ks)) == 0)
            reinterpret_cast<float4*>(w.dbg_x + (size_t)k * C)[f] = make_float4(o.x / L, o.y / L, o.z / L, o.w / L);
    }
    __syncthreads();

    // this wave's RW rows from the registers: part[k][d] = (W[d][block k] . x_k) * rscale[d]
    float acc[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int j = 0; j < NVL; ++j) {
        const int v = lane + 64 * j;
        float xv[EPV];
        const float4* xp = reinterpret_cast<const float4*>(aw_x) + v * (EPV / 4);
#pragma unroll
        for (int e = 0; e < EPV / 4; ++e) {
            const float4 t = xp[e];
            xv[4 * e] = t.x;
            xv[4 * e + 1] = t.y;
            xv[4 * e + 2] = t.z;
            xv[4 * e + 3] = t.w;
        }
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            float wf[EPV];
            Vec16<WT>::unpack(wr[r][j], wf);
#pragma unroll
            for (int e = 0; e < EPV; ++e) acc[r] = fmaf(wf[e], xv[e], acc[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        const float t = wave_sum(acc[r]);
        const int u = u0 + wave * RW + r;
        if (lane == 0) w.part[u] = w.wo_s ? t * w.wo_s[u - k * w.D] : t;
    }
}

}  // namespace sli
