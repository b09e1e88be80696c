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
// (MI355X_MICROARCH.md "Valid forms" row 1). The head's last live attention
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

// the attention role of the fused launch: split partials, the head's last workgroup merges
template <typename KT, int HD, int G>
__device__ __forceinline__ void qkv_attn_role(const AttnArgs<KT>& a) {
    const int kvh = blockIdx.x / a.max_splits;
    if (attn_publish<KT, HD, G, attn_waves(G), attn_late_v(G), true>(a, kvh, blockIdx.x - kvh * a.max_splits))
        attn_merge<HD, G>(a.part, a.out, kvh, a.max_splits, attn_live_splits<KT, HD, G>(a, kvh), 0, kGemvThreads);
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
    // the attention's share of the grid: at most a quarter of the CUs (half measured slower at TP 2: the q/k/v
    // GEMV's grid shrinks more than the attention gains, profiles/r4_qkv_attn_tp.txt)
    if ((g != 1 && g != 2) || (hd != 64 && hd != 128) || 4 * n_attn > maxb || a.n_kv_heads > kGemvLdsHead)
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

}  // namespace sli
