// qkv_attn.h — one layer's q/k/v GEMV (+ RoPE + K/V cache row) and its split decode attention as ONE launch,
// batch 1 (the reference's model.cpp:70-84 matmul / rope / mha sequence; the kernels are gemv.h gemv_block with
// EpiQKV and attention.h attn_publish).
//
// Why: on a tensor-parallel shard the launches are latency-bound (TP-8 q/k/v 7.7 us and
// attention 6.2 us per layer for 3.85 + 3.57 us of stream floor). The attention's K/V rows below the current
// position were written by earlier launches, so nothing stops them streaming while the q/k/v GEMV runs; only q
// and this step's K/V row depend on it.
//
// Grid: [0, n_attn) are the attention workgroups (kv head, split), dispatched first so their K/V loads are in
// flight from the start of the launch; [n_attn, grid) run the q/k/v GEMV (gemv_block with OFFS). The GEMV's
// epilogue stores q and a fp32 copy of this step's K/V rows (rounded to the cache type) write-through (sc1),
// drains, and adds its units to its kv heads' counters (one add per workgroup and head, spread over counters on
// separate lines: attention.h kAttnHandSub); each attention wave waits (bounded) for its
// kv head's (G + 2) * hd / 2 units, replaces the stale row at pos with the hand-off and reads q by sc1 loads
// (the hand-off pattern of persist.h, MI355X_MICROARCH.md "Valid forms" row 1). The head's last live attention
// workgroup zeroes the counters, so no memset node is needed between launches.
//
// Only the GEMV workgroups are waited on, and they wait on nothing, so the launch drains whatever the
// residency: the attention workgroups take at most a quarter of the grid capacity (the launcher refuses more),
// and the GEMV grid is sized to the CUs they leave free. Round 3 measured the other arrangement (the GEMV
// workgroups running the attention items after their own work, one 128-VGPR kernel) 3.5-4.5 us per layer
// slower at TP 1 (profiles/r3_qkv_attn_ab.txt); at TP 1 the attention grid (256 workgroups at C1) is too large
// for this launch anyway, so it runs on TP shards and small models only.
#pragma once
#include "attention.h"
#include "gemv.h"

namespace sli {

template <typename KT>
struct EpiQKVHand : EpiQKV<KT> {
    float* hand_kv;    // [2][hkv][hd]: this step's k rows, then v rows (cache-rounded fp32), sc1
    unsigned* count;   // attention.h attn_hand_words(hkv): units landed per kv head (kAttnHandSub counters each)
    int g;             // q heads per kv head
    int my_kvh = -1;   // the kv head of this thread's stored units, and their count (added in finish)
    unsigned my_n = 0;
    __device__ void arrive(int kvh, unsigned n) const {
        __hip_atomic_fetch_add(attn_hand_sub(count, kvh, blockIdx.x % kAttnHandSub), n, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ void store(int u, const int* r, const float* acc) {
        const int hq = this->hq, hkv = this->hkv, hd = this->hd, half = hd / 2;
        const int uh = u / half, d = u - uh * half;
        const bool pre = u == this->pre_u;
        float a0 = acc[0], a1 = acc[1];
        if (this->rscale) {
            a0 *= pre ? this->pre_s0 : this->rscale[r[0]];
            a1 *= pre ? this->pre_s1 : this->rscale[r[1]];
        }
        const int pos = pre ? this->pre_pos : *this->pos_dev;
        auto st = [](float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
        int kvh;
        if (uh < hq + hkv) {  // q or k: rotate (rope_kernel.cpp:30-38)
            const float fci = pre ? this->pre_sin : this->sin_t[pos * half + d];
            const float fcr = pre ? this->pre_cos : this->cos_t[pos * half + d];
            const float r0 = a0 * fcr - a1 * fci;
            const float r1 = a1 * fcr + a0 * fci;
            if (uh < hq) {
                float* q = this->q_out + (size_t)uh * hd;
                st(q + d, r0);
                st(q + d + half, r1);
                kvh = uh / g;
            } else {
                kvh = uh - hq;
                const KT k0 = from_f32<KT>(r0), k1 = from_f32<KT>(r1);
                KT* k = this->kc + ((size_t)kvh * this->T + pos) * hd;
                k[d] = k0;  // the cache row: read by later launches
                k[d + half] = k1;
                float* kn = hand_kv + (size_t)kvh * hd;
                st(kn + d, to_f32(k0));
                st(kn + d + half, to_f32(k1));
            }
        } else {
            kvh = uh - hq - hkv;
            const KT v0 = from_f32<KT>(a0), v1 = from_f32<KT>(a1);
            KT* v = this->vc + ((size_t)kvh * this->T + pos) * hd;
            v[d] = v0;
            v[d + half] = v1;
            float* vn = hand_kv + ((size_t)hkv + kvh) * hd;
            st(vn + d, to_f32(v0));
            st(vn + d + half, to_f32(v1));
        }
        if (kvh != my_kvh && my_n) {  // a thread's second head (not at the launcher's shapes): its own add
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            arrive(my_kvh, my_n);
            my_n = 0;
        }
        my_kvh = kvh;
        ++my_n;
    }
    // every thread: its stores drained, the workgroup's units counted per kv head in LDS (the reduction scratch in
    // front of the staged x; hkv <= 64 at every shape the launcher takes), one device-scope add per kv head
    __device__ void finish(float* smem) {
        unsigned* c = reinterpret_cast<unsigned*>(smem);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if ((int)threadIdx.x < this->hkv) c[threadIdx.x] = 0;
        __syncthreads();
        if (my_n) atomicAdd(c + my_kvh, my_n);
        __syncthreads();
        if ((int)threadIdx.x < this->hkv && c[threadIdx.x]) arrive(threadIdx.x, c[threadIdx.x]);
    }
};

// Chain: the wo GEMV's input stage when wo runs in the same launch, behind the attention (qkv_attn_wo_kernel). Its
// first weight steps are issued before it waits (kLate: gemv_block issues it after them); wave 0 waits (bounded) for
// every kv head's merged output (the heads' last attention workgroups count them after their sc1 stores drained),
// and the threads that hold a float4 of the input read it by sc1 (only those: every workgroup reads the same lines).
// The last workgroup past the wait zeroes the counters.
template <int G>
struct XStageHand {
    static constexpr bool kLate = true;
    unsigned* done;   // kv heads merged
    unsigned* seen;   // wo workgroups past their wait
    unsigned expect;  // kv heads
    unsigned nseen;   // wo workgroups
    int* err;
    float4 xr[kGemvStageV4];
    __device__ __forceinline__ void issue(const GemvIn& in) {
        if (threadIdx.x < 64) {
            for (unsigned spins = 0; __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < expect;
                 ++spins) {
                if (spins >= kAttnHandSpin) {
                    __hip_atomic_fetch_or(err, kAttnErrHand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0 &&
            __hip_atomic_fetch_add(seen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nseen - 1) {
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(seen, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const int n4 = in.cols >> 2;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in.x), 0, (unsigned)(in.cols * 4), 0x00020000);
#pragma unroll
        for (int k = 0; k < kGemvStageV4; ++k) {
            const int i = (int)threadIdx.x + k * kGemvThreads;
            if (i < n4) xr[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * i, 0, 16 /* sc1 */));
        }
    }
    __device__ __forceinline__ void commit(float* smem, const GemvIn& in) {
        float4* xs4 = reinterpret_cast<float4*>(smem + kGemvLdsHead);
        const int n4 = in.cols >> 2;
#pragma unroll
        for (int k = 0; k < kGemvStageV4; ++k) {
            const int i = (int)threadIdx.x + k * kGemvThreads;
            if (i < n4) xs4[xswz<G>(i)] = xr[k];
        }
    }
};

// the attention role of the fused launches: split partials, the head's last workgroup merges (and, in a chain,
// counts the merged head for the wo workgroups)
template <typename KT, int HD, int G>
__device__ __forceinline__ void qkv_attn_role(const AttnArgs<KT>& a) {
    const int kvh = blockIdx.x / a.max_splits;
    if (attn_publish<KT, HD, G, attn_waves(G), attn_late_v(G), true>(a, kvh, blockIdx.x - kvh * a.max_splits)) {
        attn_merge<HD, G>(a.part, a.out, kvh, a.max_splits, attn_live_splits<KT, HD, G>(a, kvh), 0, kGemvThreads);
        if (a.chain_done) {  // every thread's sc1 stores drained (attn_merge): one arrival for the head
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_fetch_add(a.chain_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <typename WT, int U, typename KT, int HD, int G>
__global__ void __launch_bounds__(kGemvThreads) qkv_attn_kernel(const WT* __restrict__ W, GemvIn in,
                                                                 EpiQKVHand<KT> epi_in, AttnArgs<KT> a) {
    static_assert(attn_waves(G) * 64 == kGemvThreads, "the attention workgroups must be GEMV-sized (G <= 2)");
    if ((int)blockIdx.x < in.blk0) {
        qkv_attn_role<KT, HD, G>(a);
        return;
    }
    EpiQKVHand<KT> epi = epi_in;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    XStage<Vec16<WT>::N / 4> stage;
    gemv_block<WT, 2, U, true, EpiQKVHand<KT>, XStage<Vec16<WT>::N / 4>, 2, true, true>(W, in, epi, stage, smem);
}

// The chain: attention [0, n_attn), q/k/v GEMV [n_attn, wo.blk0), then the wo GEMV [wo.blk0, grid). The wo workgroups
// are dispatched as the q/k/v workgroups retire, stream their first weight steps while the attention finishes, and
// wait for the merged heads (XStageHand). Every wait is on lower-indexed workgroups, which never wait on higher ones.
template <typename WT, int U, typename KT, int HD, int G, class WoEpi, int UO>
__global__ void __launch_bounds__(kGemvThreads)
    qkv_attn_wo_kernel(const WT* __restrict__ W, GemvIn in, EpiQKVHand<KT> epi_in, AttnArgs<KT> a,
                       const WT* __restrict__ Wo, GemvIn in_wo, WoEpi wo_epi_in, XStageHand<Vec16<WT>::N / 4> wo_stage) {
    static_assert(attn_waves(G) * 64 == kGemvThreads, "the attention workgroups must be GEMV-sized (G <= 2)");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    if ((int)blockIdx.x < in.blk0) {
        qkv_attn_role<KT, HD, G>(a);
        return;
    }
    if ((int)blockIdx.x < in_wo.blk0) {
        EpiQKVHand<KT> epi = epi_in;  // (in.blk1 = in_wo.blk0: the q/k/v partition ends where wo's workgroups begin)
        XStage<Vec16<WT>::N / 4> stage;
        gemv_block<WT, 2, U, true, EpiQKVHand<KT>, XStage<Vec16<WT>::N / 4>, 2, true, true>(W, in, epi, stage, smem);
        return;
    }
    WoEpi epi = wo_epi_in;
    XStageHand<Vec16<WT>::N / 4> stage = wo_stage;
    gemv_block<WT, 1, UO, true, WoEpi, XStageHand<Vec16<WT>::N / 4>, 2, false, true>(Wo, in_wo, epi, stage, smem);
}

// Launch, or hipErrorNotSupported when the shape does not qualify (the caller then runs the two launches):
// G <= 2, hd 64 / 128, and an attention grid of at most a quarter of the persistent GEMV grid (TP shards and
// small models; every TP-1 preset's is larger). a: the attention's arguments as mha_launch builds them, hand_* filled in.
// dry: only the answer (hipSuccess: it would launch).
template <typename WT, typename KT>
hipError_t launch_qkv_attn(const WT* W, const GemvIn& in_, const EpiQKVHand<KT>& e, const AttnArgs<KT>& a, int units,
                           int hd, hipStream_t s, bool dry = false) {
    constexpr int UW = std::is_same<WT, int8_t>::value ? 2 : 4;
    const int g = e.g;
    const int n_attn = a.n_kv_heads * a.max_splits;
    const int maxb = gemv_max_blocks();
    // the attention's share of the grid: at most 1 / qa_div of the CUs (SLI_QKV_ATTN_DIV, default 4; A/B knob)
    static const int qa_div = [] {
        const char* e = getenv("SLI_QKV_ATTN_DIV");
        return e && atoi(e) >= 2 ? atoi(e) : 4;
    }();
    if ((g != 1 && g != 2) || (hd != 64 && hd != 128) || qa_div * n_attn > maxb || a.n_kv_heads > kGemvLdsHead)
        return hipErrorNotSupported;
    const GemvSplit sp = gemv_split<WT, 4>(units, in_.cols);  // (CS 1 runs the split instantiation unsplit)
    if (dry) return hipSuccess;  // (sli_model_fused_qkv_attn: would launch)
    GemvIn in = in_;
    in.csplit = sp.cs;
    in.cw = kGemvThreads / 64;
    in.blk0 = n_attn;
    const int grid_g = std::min(gemv_blocks(units, sp.cs), maxb - n_attn);
    const size_t lds = gemv_lds_bytes(in.cols) + sizeof(float) * gemv_res_floats(units, grid_g, 2, sp.cs);
    const dim3 grid(n_attn + grid_g), blk(kGemvThreads);
#define SLI_QA(U_, HD_, G_) hipLaunchKernelGGL((qkv_attn_kernel<WT, U_, KT, HD_, G_>), grid, blk, lds, s, W, in, e, a)
#define SLI_QA_G(U_, HD_) \
    do {                  \
        if (g == 1)       \
            SLI_QA(U_, HD_, 1); \
        else              \
            SLI_QA(U_, HD_, 2); \
    } while (0)
#define SLI_QA_HD(U_)  \
    do {               \
        if (hd == 128) \
            SLI_QA_G(U_, 128); \
        else           \
            SLI_QA_G(U_, 64); \
    } while (0)
    if (sp.u == UW) {
        SLI_QA_HD(UW);
    } else if (UW > 2 && sp.u == 2) {
        SLI_QA_HD(2);
    } else {
        SLI_QA_HD(1);
    }
#undef SLI_QA_HD
#undef SLI_QA_G
#undef SLI_QA
    return hipGetLastError();
}

// The chain launch (q/k/v + attention + wo), fp16 weights: hipErrorNotSupported where launch_qkv_attn would refuse,
// where wo's GEMV would be column-split, or where the grid outgrows the per-workgroup exchange's flag slots.
// a.defer_merge must be 0 (the heads' last workgroups merge) and a.chain_done set; done / seen: two counters on
// separate lines, zero between launches.
template <typename KT, class WoEpi>
hipError_t launch_qkv_attn_wo(const __half* W, const GemvIn& in_, const EpiQKVHand<KT>& e, const AttnArgs<KT>& a,
                              int units, int hd, const __half* Wo, const GemvIn& in_wo_, const WoEpi& wo_epi,
                              int wo_units, unsigned* done, unsigned* seen, int max_grid, hipStream_t s,
                              bool dry = false) {
    const int g = e.g;
    const int n_attn = a.n_kv_heads * a.max_splits;
    const int maxb = gemv_max_blocks();
    if ((g != 1 && g != 2) || (hd != 64 && hd != 128) || 4 * n_attn > maxb || a.n_kv_heads > kGemvLdsHead ||
        a.defer_merge != 0 || !a.chain_done)
        return hipErrorNotSupported;
    const GemvSplit sp = gemv_split<__half, 4>(units, in_.cols);
    if (gemv_split<__half, 2>(wo_units, in_wo_.cols).cs != 1) return hipErrorNotSupported;
    const int grid_g = std::min(gemv_blocks(units, sp.cs), maxb - n_attn);
    const int grid_o = gemv_balanced_blocks(wo_units);
    if (n_attn + grid_g + grid_o > max_grid) return hipErrorNotSupported;
    if (dry) return hipSuccess;
    GemvIn in = in_;
    in.csplit = sp.cs;
    in.cw = kGemvThreads / 64;
    in.blk0 = n_attn;
    in.blk1 = n_attn + grid_g;
    GemvIn in_wo = in_wo_;
    in_wo.csplit = 1;
    in_wo.cw = gemv_wave_count<__half>(wo_units, grid_o);
    in_wo.blk0 = n_attn + grid_g;
    const XStageHand<2> st{done, seen, (unsigned)a.n_kv_heads, (unsigned)grid_o, a.hand_err};
    const size_t lds =
        std::max(gemv_lds_bytes(in.cols) + sizeof(float) * gemv_res_floats(units, grid_g, 2, sp.cs),
                 gemv_lds_bytes(in_wo.cols) + sizeof(float) * gemv_res_floats(wo_units, grid_o, 1));
    const dim3 grid(n_attn + grid_g + grid_o), blk(kGemvThreads);
#define SLI_QAW(U_, HD_, G_)                                                                                         \
    hipLaunchKernelGGL((qkv_attn_wo_kernel<__half, U_, KT, HD_, G_, WoEpi, 2>), grid, blk, lds, s, W, in, e, a, Wo, \
                       in_wo, wo_epi, st)
#define SLI_QAW_G(U_, HD_) \
    do {                   \
        if (g == 1)        \
            SLI_QAW(U_, HD_, 1); \
        else               \
            SLI_QAW(U_, HD_, 2); \
    } while (0)
#define SLI_QAW_HD(U_) \
    do {               \
        if (hd == 128) \
            SLI_QAW_G(U_, 128); \
        else           \
            SLI_QAW_G(U_, 64); \
    } while (0)
    if (sp.u == 4) {
        SLI_QAW_HD(4);
    } else if (sp.u == 2) {
        SLI_QAW_HD(2);
    } else {
        SLI_QAW_HD(1);
    }
#undef SLI_QAW_HD
#undef SLI_QAW_G
#undef SLI_QAW
    return hipGetLastError();
}

}  // namespace sli
