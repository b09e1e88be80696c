// gemv.h — weight-streaming GEMV for batch-1 decode on gfx950 (the reference's matmul_f32_kernel,
// source/kernel/cuda/matmul_kernel.cu:5-38, and its callers' surrounding ops, re-designed):
//
//   * one wave64 owns R output rows at a time and streams their weights with 16-byte (dwordx4) loads,
//     U vectors per row in flight per lane before any use (HBM-bound: load straight to VGPRs, no LDS
//     round trip for W — cdna_hip_programming.md §5, 'GEMV / M <= 16' row);
//   * the input vector is staged once per workgroup in LDS as fp32, optionally RMS-normalised in the
//     prologue (fused RMSNorm, rms_kernel.cpp:5-23 semantics);
//   * fp32 accumulation for f32 / f16 / int8 weights (int8: per-row scale applied to the row sum);
//   * the epilogue functor decides which rows form a unit and what happens to the R row sums
//     (plain store, residual add, RoPE + KV-cache write, SwiGLU, logits + argmax keys).
// Grid-stride over units so a launch is sized to the chip, not to the matrix.
#pragma once
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace sli {

struct GemvIn {
    const float* x;       // [cols] fp32 input vector
    const float* norm_w;  // nullptr: plain; else fused RMSNorm weight [cols]
    float eps;
    int cols;
    unsigned long long* stamps = nullptr;  // diagnostic (tools/gemv_lab): per-wave s_memrealtime x4
    int csplit = 1;  // column parts per unit (gemv_block): a unit's rows split over up to csplit waves
    int cw = 16;     // waves per workgroup that stream (gemv_wave_count); the others only shadow loads
    int blk0 = 0;    // workgroups in front of the GEMV's own in the grid (qkv_attn.h: the attention's); OFFS only
    int blk1 = 0;    // OFFS: the end of the GEMV's workgroups (0: the grid's end)
};

constexpr int kGemvThreads = 1024;  // one persistent 16-wave workgroup per CU: x staged once per CU
constexpr int kGemvLdsHead = 64;  // floats of reduction scratch in front of the staged x

inline size_t gemv_lds_bytes(int cols) { return sizeof(float) * (size_t)(kGemvLdsHead + cols); }

constexpr int kGemvStageV4 = 4;  // float4 of x per thread: 1024 threads x 4 x 4 = 16384 columns

// The prologue is split into issue (global loads into registers) and commit (normalise, write LDS) so
// the kernel can issue its input loads FIRST, its weight loads second, and wait only for the input:
// s_waitcnt vmcnt counts in issue order, so an input load issued after the weights would wait for the
// whole first weight chunk (measured: x staged 6-11 us into a 10-30 us launch), and no wave could
// start consuming weights until every wave's first chunk had landed.
// LDS layout of the staged x: float4 f of the input lives at slot xswz<G>(f), G = float4s per 16-byte
// weight vector (fp32 1, fp16 2, int8 4). Lane l of a GEMV wave reads the G float4s of weight vector
// v = base + l; unswizzled, the 16 lanes of a ds_read_b128 group (MI355X_MICROARCH.md §LDS:
// {0-3,12-15,20-27}, ...) hit only 16/G distinct 16-byte slots of the 256-byte bank row (fp16 2-way,
// int8 4-way conflicts). XOR-ing the float4 index inside its vector with bits of v>>(4/G) spreads
// every group over all 16 slots; 8 contiguous writers of the staging store share one key, so the
// ds_write_b128 groups stay conflict-free.
template <int G>
__device__ __forceinline__ int xswz(int f) {
    return G == 1 ? f : f ^ ((f >> 4) & (G - 1));
}

// Stages that wait for their input inside issue() (kLate = true) are issued after the first weight steps.
template <class S, class = void>
struct StageLate {
    static constexpr bool value = false;
};
template <class S>
struct StageLate<S, std::void_t<decltype(S::kLate)>> {
    static constexpr bool value = S::kLate;
};
template <class S>
__host__ __device__ constexpr bool stage_late() {
    return StageLate<S>::value;
}

template <int G>
struct XStage {
    float4 xr[kGemvStageV4];
    float4 wr[kGemvStageV4];
    __device__ __forceinline__ void issue(const GemvIn& in) {
        const int tid = threadIdx.x, nt = kGemvThreads, n4 = in.cols >> 2;
        const float4* x4 = reinterpret_cast<const float4*>(in.x);
        // unconditional (clamped) loads: a load under a branch would make the weight waits conservative
        const float4* w4 = reinterpret_cast<const float4*>(in.norm_w ? in.norm_w : in.x);
#pragma unroll
        for (int k = 0; k < kGemvStageV4; ++k) {
            xr[k] = x4[min(tid + k * nt, n4 - 1)];
            wr[k] = w4[min(tid + k * nt, n4 - 1)];
        }
    }
    // x (optionally RMS-normalised, rms_kernel.cpp:5-23) into LDS; the caller then barriers. Stores are
    // unconditional too (clamped rounds rewrite the last vector with its own value).
    __device__ __forceinline__ void commit(float* smem, const GemvIn& in) {
        float* red = smem;
        float4* xs4 = reinterpret_cast<float4*>(smem + kGemvLdsHead);
        const int tid = threadIdx.x, nt = kGemvThreads, n4 = in.cols >> 2;
        if (in.norm_w == nullptr) {
#pragma unroll
            for (int k = 0; k < kGemvStageV4; ++k) xs4[xswz<G>(min(tid + k * nt, n4 - 1))] = xr[k];
            return;
        }
        float ss = 0.0f;
#pragma unroll
        for (int k = 0; k < kGemvStageV4; ++k) {
            const float m = tid + k * nt < n4 ? 1.0f : 0.0f;
            ss += m * (xr[k].x * xr[k].x);
            ss += m * (xr[k].y * xr[k].y);
            ss += m * (xr[k].z * xr[k].z);
            ss += m * (xr[k].w * xr[k].w);
        }
        ss = wave_sum(ss);
        if ((tid & 63) == 0) red[tid >> 6] = ss;
        __syncthreads();
        if (tid == 0) {
            float t = 0.0f;
            for (int w = 0; w < (nt >> 6); ++w) t += red[w];
            const float tep = t / (float)in.cols;  // rms_kernel.cpp:17
            const float rms = sqrtf(tep + in.eps);  // :18
            red[32] = 1.0f / rms;                   // :19
        }
        __syncthreads();
        const float inv = red[32];
#pragma unroll
        for (int k = 0; k < kGemvStageV4; ++k) {  // :20-22  y = (x * inv) * w
            float4 o;
            o.x = (xr[k].x * inv) * wr[k].x;
            o.y = (xr[k].y * inv) * wr[k].y;
            o.z = (xr[k].z * inv) * wr[k].z;
            o.w = (xr[k].w * inv) * wr[k].w;
            xs4[xswz<G>(min(tid + k * nt, n4 - 1))] = o;
        }
    }
};


// The wo GEMV's input staged straight from the attention's split partials (attention.h, defer_merge): for
// every head h and dim d, out = (sum_s e^{m_s - M} o_s) / (sum_s e^{m_s - M} l_s) over the ns live splits in
// split order, M = max_s m_s — attn_merge's arithmetic, so the result is bit-identical to the attention
// kernel's own last-arriver merge, without that merge's serial tail (an arrival counter, a second round
// trip to the partials and a store) inside the attention launch. The partials are loaded with the input
// loads, before the weight stream, like XStage's x (NS splits in flight per thread, the rest from memory).
struct AttnMergeIn {
    const float* part;       // [heads][max_splits][hd + kAttnPartPad]
    const int32_t* pos_dev;  // the live context: ns = min(pos / ppwg + 1, max_splits)
    int max_splits, ppwg, hd;
    // K-split wo (EpiKPart): the launch's units are ksplit blocks of kunits (k-major), a workgroup's units all lie
    // in one block k, and it stages (merges) only the heads of input quarter k: in.cols / hd heads from head
    // k * in.cols / hd on. ksplit 1: the whole input.
    int ksplit = 1, kunits = 0;
};

template <int G, int NS = 8>
struct XStageMerge {
    AttnMergeIn am;
    float4 ov[NS];
    float2 ml[NS];
    int pos = 0;
    int h0 = 0;  // first head of this workgroup's input (K-split wo)
    __device__ __forceinline__ const float* row(int f, int s) const {
        const int h = h0 + f / (am.hd >> 2);
        return am.part + ((size_t)h * am.max_splits + min(s, am.max_splits - 1)) * (am.hd + kAttnPartPad);
    }
    __device__ __forceinline__ void issue(const GemvIn& in) {
        if (am.ksplit > 1) {  // the block k of the workgroup's first unit (gemv_block's balanced partition)
            const int nw = kGemvThreads >> 6;
            const int ub = (int)(((unsigned)(blockIdx.x * nw) * (unsigned)(am.ksplit * am.kunits)) / (unsigned)(gridDim.x * nw));
            h0 = (ub / am.kunits) * (in.cols / am.hd);
        }
        const int f = min((int)threadIdx.x, (in.cols >> 2) - 1);  // the first round of the input
        const int d4 = f % (am.hd >> 2);
        pos = *am.pos_dev;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const float* r = row(f, s);
            ov[s] = reinterpret_cast<const float4*>(r)[d4];
            ml[s] = *reinterpret_cast<const float2*>(r + am.hd);
        }
    }
    struct Acc {
        float M;
        float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float L = 0.0f;
        __device__ __forceinline__ void add(float2 lm, float4 v) {
            const float w = expf(lm.x - M);
            o.x = fmaf(w, v.x, o.x);
            o.y = fmaf(w, v.y, o.y);
            o.z = fmaf(w, v.z, o.z);
            o.w = fmaf(w, v.w, o.w);
            L = fmaf(w, lm.y, L);
        }
        __device__ __forceinline__ float4 out() const { return make_float4(o.x / L, o.y / L, o.z / L, o.w / L); }
    };
    // the first round: splits < NS from the registers (unrolled and predicated: no dynamic register index)
    __device__ __forceinline__ float4 merge_regs(int f, int ns) const {
        const int d4 = f % (am.hd >> 2);
        float M = -INFINITY;
#pragma unroll
        for (int s = 0; s < NS; ++s)
            if (s < ns) M = fmaxf(M, ml[s].x);
        for (int s = NS; s < ns; ++s) M = fmaxf(M, row(f, s)[am.hd]);
        Acc a{M};
#pragma unroll
        for (int s = 0; s < NS; ++s)
            if (s < ns) a.add(ml[s], ov[s]);
        for (int s = NS; s < ns; ++s)
            a.add(*reinterpret_cast<const float2*>(row(f, s) + am.hd), reinterpret_cast<const float4*>(row(f, s))[d4]);
        return a.out();
    }
    // later rounds (inputs wider than 4 * kGemvThreads): straight from memory
    __device__ __forceinline__ float4 merge_mem(int f, int ns) const {
        const int d4 = f % (am.hd >> 2);
        float M = -INFINITY;
        for (int s = 0; s < ns; ++s) M = fmaxf(M, row(f, s)[am.hd]);
        Acc a{M};
        for (int s = 0; s < ns; ++s)
            a.add(*reinterpret_cast<const float2*>(row(f, s) + am.hd), reinterpret_cast<const float4*>(row(f, s))[d4]);
        return a.out();
    }
    __device__ __forceinline__ void commit(float* smem, const GemvIn& in) {
        float4* xs4 = reinterpret_cast<float4*>(smem + kGemvLdsHead);
        const int n4 = in.cols >> 2;
        const int ns = min(pos / am.ppwg + 1, am.max_splits);
        if ((int)threadIdx.x < n4) xs4[xswz<G>(threadIdx.x)] = merge_regs(threadIdx.x, ns);
        for (int f = threadIdx.x + kGemvThreads; f < n4; f += kGemvThreads) xs4[xswz<G>(f)] = merge_mem(f, ns);
    }
};

// The input x + p_0 + ... + p_{NP-1} (the K-split wo's partial row sums, EpiKPart, added in that order), then
// optionally RMS-normalised like XStage (rms_kernel.cpp:5-23): the gate/up GEMV of a layer whose wo ran K-split
// stages the residual stream x1 = x + wo . attn (model.cpp:86-90) itself. One round only: cols <= 4 *
// kGemvThreads (the host checks), so every input float4 and its partials are one thread's registers (a thread
// past the input repeats the last float4 with the same value).
template <int G, int NP>
struct XStageSum {
    const float* parts;  // [NP][cols]
    float4 xr, wr, pr[NP];
    __device__ __forceinline__ void issue(const GemvIn& in) {
        const int f = min((int)threadIdx.x, (in.cols >> 2) - 1);
        xr = reinterpret_cast<const float4*>(in.x)[f];
        wr = reinterpret_cast<const float4*>(in.norm_w ? in.norm_w : in.x)[f];
#pragma unroll
        for (int k = 0; k < NP; ++k) pr[k] = reinterpret_cast<const float4*>(parts + (size_t)k * in.cols)[f];
    }
    __device__ __forceinline__ void commit(float* smem, const GemvIn& in) {
        float* red = smem;
        float4* xs4 = reinterpret_cast<float4*>(smem + kGemvLdsHead);
        const int tid = threadIdx.x, n4 = in.cols >> 2, f = min(tid, n4 - 1);
        float4 v = xr;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            v.x += pr[k].x;
            v.y += pr[k].y;
            v.z += pr[k].z;
            v.w += pr[k].w;
        }
        if (in.norm_w == nullptr) {
            xs4[xswz<G>(f)] = v;
            return;
        }
        const float m = tid < n4 ? 1.0f : 0.0f;
        float ss = m * (v.x * v.x);
        ss += m * (v.y * v.y);
        ss += m * (v.z * v.z);
        ss += m * (v.w * v.w);
        ss = wave_sum(ss);
        if ((tid & 63) == 0) red[tid >> 6] = ss;
        __syncthreads();
        if (tid == 0) {
            float t = 0.0f;
            for (int w = 0; w < (kGemvThreads >> 6); ++w) t += red[w];
            const float tep = t / (float)in.cols;  // rms_kernel.cpp:17
            const float rms = sqrtf(tep + in.eps);  // :18
            red[32] = 1.0f / rms;                   // :19
        }
        __syncthreads();
        const float inv = red[32];
        float4 o;  // :20-22  y = (x * inv) * w
        o.x = (v.x * inv) * wr.x;
        o.y = (v.y * inv) * wr.y;
        o.z = (v.z * inv) * wr.z;
        o.w = (v.w * inv) * wr.w;
        xs4[xswz<G>(f)] = o;
    }
};

// One-shot staging for callers that have nothing to overlap it with.
template <int G = 1>
__device__ __forceinline__ void gemv_stage_x(float* smem, const GemvIn& in) {
    XStage<G> st;
    st.issue(in);
    st.commit(smem, in);
}

// acc[r] += sum over the U vectors (64 lanes apart, starting at vector index v) of W[r] . x.
// MASK: vectors at index >= nvec contribute nothing (their loads were clamped in range by the caller).
template <typename WT, int R, int U, bool MASK = false>
__device__ __forceinline__ void gemv_chunk(const u32x4 (&w)[U][R], const float* xs, int v, float* acc,
                                           int nvec = 0) {
    constexpr int EPV = Vec16<WT>::N;
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const int vj = v + j * 64;
        if (MASK && vj >= nvec) continue;
        float xv[EPV];
        constexpr int G = EPV / 4;
        const float4* xp = reinterpret_cast<const float4*>(xs) + vj * G;
        const int key = ((vj * G) >> 4) & (G - 1);  // xswz<G>
#pragma unroll
        for (int e = 0; e < G; ++e) {
            float4 t = xp[e ^ key];
            xv[4 * e] = t.x;
            xv[4 * e + 1] = t.y;
            xv[4 * e + 2] = t.z;
            xv[4 * e + 3] = t.w;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            float wf[EPV];
            Vec16<WT>::unpack(w[j][r], wf);
#pragma unroll
            for (int e = 0; e < EPV; ++e) acc[r] = fmaf(wf[e], xv[e], acc[r]);
        }
    }
}

// Units of workgroup b: [b*W*N/G, (b+1)*W*N/G) for W waves per workgroup, G workgroups (32-bit math:
// grid waves x units stays below 2^32 for every supported shape).
__device__ __forceinline__ int gemv_unit_begin(int gwave, int nunits, int total_waves) {
    return (int)(((unsigned)gwave * (unsigned)nunits) / (unsigned)total_waves);
}

// Result slots in LDS behind the staged x: R floats per (unit, column part) of the workgroup.
inline size_t gemv_res_floats(int units, int grid, int R, int csplit = 1) {
    return (size_t)R * csplit * ((size_t)units / grid + 2);
}

// Wave-level schedule. Wave gw of the grid owns units [gw*N/W, (gw+1)*N/W) (balanced: sizes differ by at
// most one); a unit is R rows chosen by the epilogue, streamed in chunks of U 16-byte vectors per row
// per lane. The wave's work is the flat sequence of (unit, chunk) steps; the next step's loads
// are issued before the current step is consumed (two register buffers), so each wave keeps a chunk in
// flight while it computes.
//
// Straight-line memory order, no global access inside the loop but weight loads: every weight load is
// unconditional (positions clamped to the wave's last step; a wave without units loads a valid row it
// never uses), and finished row sums go to LDS, not to global memory. s_waitcnt vmcnt counts loads and
// stores together in issue order, so a conditional load or store anywhere in the sequence forces the
// compiler to a conservative vmcnt(0) at the next use of the weights — measured: the x prologue waited
// for the first weight chunk (staged 4-6 us into a 10-30 us launch). The epilogue (residual reads,
// RoPE, K/V writes, logits) runs once per workgroup after the loop, one thread per unit.
// Prologue order: input loads, first weight chunk, input commit + barrier (see XStage).
template <typename WT, int R, int U, bool NT, class Epi, class Stage, int NB = 2, bool SPLIT = false, bool OFFS = false>
__device__ __forceinline__ void gemv_block(const WT* __restrict__ W, const GemvIn& in, Epi& epi, Stage& stage,
                                           float* smem) {
    const float* xs = smem + kGemvLdsHead;

    constexpr int EPV = Vec16<WT>::N;
    constexpr int CV = U * 64;  // vectors per row per chunk
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwaves = kGemvThreads >> 6;  // compile-time: blockDim.x is a dispatch-packet load
    const int nvec = in.cols / EPV;
    const size_t row_bytes = (size_t)in.cols * sizeof(WT);
    const int nunits = epi.units();
    // OFFS: the GEMV is workgroups [in.blk0, gridDim.x) of a launch it shares (qkv_attn.h)
    const int bx = OFFS ? (int)blockIdx.x - in.blk0 : (int)blockIdx.x;
    const int total_waves = (OFFS ? (in.blk1 > 0 ? in.blk1 : (int)gridDim.x) - in.blk0 : (int)gridDim.x) * nwaves;
    const int ub = gemv_unit_begin(bx * nwaves, nunits, total_waves);  // workgroup's first unit
    const int ue = gemv_unit_begin((bx + 1) * nwaves, nunits, total_waves);
    const int cpr = (nvec + CV - 1) / CV;  // chunks per row
    // Column split (small matrices, e.g. tensor-parallel shards): a unit's rows are cut into CS parts of
    // cpp chunks; the workgroup's (unit, part) items are balanced over its waves and the parts' row sums
    // are added in part order in the epilogue. CS = 1: one item per unit, the whole row per wave.
    const int CS = SPLIT ? in.csplit : 1;  // compile-time 1 unless the launch split the columns
    const int cpp = (cpr + CS - 1) / CS;  // chunks per part (a part past the row end is all masked)
    const int ni = (ue - ub) * CS;       // the workgroup's items
    // in.cw streaming waves share the items; a wave past them has none and repeats the loads of wave
    // (wave - cw)'s first steps (L2 hits on lines in flight), so no load sits behind a branch
    const int cw = in.cw;
    const bool idle = wave >= cw;
    const int wq = idle ? wave - cw : wave;
    const int ib = (int)(((unsigned)wq * (unsigned)ni) / (unsigned)cw);
    const int ie = idle ? ib : (int)(((unsigned)(wq + 1) * (unsigned)ni) / (unsigned)cw);
    const int nsteps = (ie - ib) * cpp;
    float* res = smem + kGemvLdsHead + in.cols;

    const unsigned long long t_entry = in.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long t_staged = 0;
    // (a LATE stage (qkv_attn.h XStageHand) waits for its input inside issue(): it is issued after the first
    // weight steps, so the weights stream during the wait)
    if constexpr (!stage_late<Stage>()) stage.issue(in);
    // the epilogue's own inputs for this thread's unit (the store loop's first unit): in flight with the
    // input, landed long before the stream ends instead of a round trip after it
    const int pre_unit = max(min(ub + (int)threadIdx.x, nunits - 1), 0);
    epi.prefetch_a(pre_unit);
    __builtin_amdgcn_sched_barrier(0);  // keep every input load ahead of the weight loads

    // A step is (item, chunk of its part); the position (u, p, cc) advances incrementally. The load
    // position saturates at the wave's last step (a wave without items loads a valid row it never uses).
    struct Pos {
        int it, u, p, cc;
    };
    const int it_last = max(ie - 1, ib);
    const Pos last{it_last, min(ub + it_last / CS, nunits - 1), it_last - (it_last / CS) * CS, cpp - 1};
    // A load past the wave's last step (its last round when the step count is not a multiple of NB, or the
    // first rounds of a wave with fewer than NB steps) reads the matrix's first chunk instead of repeating its
    // own last step: that repeat was issued after the first copy had landed, so it went back to HBM (int8
    // down at 7B, 3 chunks per row: FETCH_SIZE 1.10x the algorithmic bytes), while the first chunk of the
    // launch is L2-resident on every XCD after its first read. Unconditional either way (only the address
    // is selected). SLI_GEMV_DUP_LOADS=1: the round-2 behaviour (A/B).
#ifndef SLI_GEMV_DUP_LOADS
#define SLI_GEMV_DUP_LOADS 0
#endif
    const Pos dummy = SLI_GEMV_DUP_LOADS ? last : Pos{0, 0, 0, 0};
    auto load_step = [&](const Pos& q, u32x4 (&w)[U][R]) {
        const Pos& a = q.it > it_last ? dummy : q;
        int rows[R];
        epi.rows(min(a.u, nunits - 1), rows);
        const int v = (a.p * cpp + a.cc) * CV + lane;
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int vj = min(v + j * 64, nvec - 1);  // clamp, never branch around a load
#pragma unroll
            for (int r = 0; r < R; ++r)
                w[j][r] = load16<NT>(reinterpret_cast<const char*>(W) + (size_t)rows[r] * row_bytes + (size_t)vj * 16);
        }
    };
    auto next = [&](Pos& q) {
        if (++q.cc == cpp) {
            q.cc = 0;
            ++q.it;
            if (++q.p == CS) {
                q.p = 0;
                ++q.u;
            }
        }
    };
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
    auto consume_step = [&](const Pos& q, const u32x4(&w)[U][R]) {
        const int c = q.p * cpp + q.cc;
        const int v = c * CV + lane;
        if ((c + 1) * CV <= nvec)
            gemv_chunk<WT, R, U>(w, xs, v, acc);
        else
            gemv_chunk<WT, R, U, true>(w, xs, v, acc, nvec);
        if (q.cc == cpp - 1) {  // item complete: its R partial row sums go to LDS
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const float t = wave_sum(acc[r]);
                if (lane == 0) res[((q.u - ub) * CS + q.p) * R + r] = t;
                acc[r] = 0.0f;
            }
        }
    };

    // NB register buffers (steps), all in flight before the input is committed. Every load is
    // unconditional: a position past the wave's last step is clamped to that step, so the extra load
    // duplicates one issued just before it (an in-flight miss to the same lines) and is never consumed;
    // no clamped load is ever issued after its data was consumed (a fresh HBM round trip at the end of
    // every wave).
    u32x4 wbuf[NB][U][R];
    const Pos first{ib, ub + ib / CS, ib - (ib / CS) * CS, 0};
    Pos lq = first;  // next step to load
    Pos cq = first;  // next step to consume
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        load_step(lq, wbuf[b]);
        next(lq);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (stage_late<Stage>()) stage.issue(in);
    stage.commit(smem, in);
    __syncthreads();
    epi.prefetch_b(pre_unit);
    t_staged = in.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    int k = 0;
    for (; k + NB < nsteps; k += NB) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            consume_step(cq, wbuf[b]);
            next(cq);
            load_step(lq, wbuf[b]);  // step k + b + NB, or a duplicate of the wave's last step
            next(lq);
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (k + b < nsteps) {
            consume_step(cq, wbuf[b]);
            next(cq);
        }
    }
    __syncthreads();
    for (int u = ub + (int)threadIdx.x; u < ue; u += kGemvThreads) {
        int rows[R];
        epi.rows(u, rows);
        const float* ru = res + (size_t)(u - ub) * CS * R;
        float v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            v[r] = ru[r];
            for (int p = 1; p < CS; ++p) v[r] += ru[p * R + r];  // part order: deterministic
        }
        epi.store(u, rows, v);
    }
    epi.finish(smem);
    if (in.stamps && lane == 0) {
        unsigned long long* p = in.stamps + ((size_t)bx * nwaves + wave) * 4;
        p[0] = t_entry;
        p[1] = t_staged;
        p[2] = __builtin_amdgcn_s_memrealtime();
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        p[3] = (unsigned long long)max(nsteps, 1) | ((unsigned long long)(xcc & 15) << 32);  // diagnostic: XCD
    }
}

template <typename WT, int R, int U, bool NT, class Epi, int NB = 2, bool SPLIT = false>
__global__ void __launch_bounds__(kGemvThreads) gemv_kernel(const WT* __restrict__ W, GemvIn in, Epi epi_in) {
    Epi epi = epi_in;  // mutable per-thread copy (EpiLogits keeps a running key)
    extern __shared__ __attribute__((aligned(16))) float smem[];
    XStage<Vec16<WT>::N / 4> stage;
    gemv_block<WT, R, U, NT, Epi, XStage<Vec16<WT>::N / 4>, NB, SPLIT>(W, in, epi, stage, smem);
}

// the wo GEMV with its input merged from the attention's split partials (XStageMerge)
template <typename WT, int R, int U, bool NT, class Epi, int NS = 8, int NB = 2>
__global__ void __launch_bounds__(kGemvThreads) gemv_merge_kernel(const WT* __restrict__ W, GemvIn in, Epi epi_in,
                                                                  AttnMergeIn am) {
    Epi epi = epi_in;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    XStageMerge<Vec16<WT>::N / 4, NS> stage{am};
    gemv_block<WT, R, U, NT, Epi, XStageMerge<Vec16<WT>::N / 4, NS>, NB>(W, in, epi, stage, smem);
}

// a GEMV whose input is x plus NP partial vectors (XStageSum)
template <typename WT, int R, int U, bool NT, class Epi, int NP, int NB = 2>
__global__ void __launch_bounds__(kGemvThreads) gemv_sum_kernel(const WT* __restrict__ W, GemvIn in, Epi epi_in,
                                                                const float* parts) {
    Epi epi = epi_in;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    XStageSum<Vec16<WT>::N / 4, NP> stage{parts};
    gemv_block<WT, R, U, NT, Epi, XStageSum<Vec16<WT>::N / 4, NP>, NB>(W, in, epi, stage, smem);
}

// Row-by-row fallback for shapes the vector kernel cannot take (cols*sizeof(WT) not a multiple of 16
// or a misaligned base): one wave per row, scalar loads. Only the op-level API reaches it.
template <typename WT>
__global__ void __launch_bounds__(kGemvThreads)
    gemv_scalar_kernel(const WT* __restrict__ W, const float* __restrict__ x, const float* rscale, float* y, int rows,
                       int cols, float scale) {
    const int lane = threadIdx.x & 63;
    const int nwaves = blockDim.x >> 6;
    for (int r = blockIdx.x * nwaves + (threadIdx.x >> 6); r < rows; r += gridDim.x * nwaves) {
        const WT* wr = W + (size_t)r * cols;
        float acc = 0.0f;
        for (int c = lane; c < cols; c += 64) acc = fmaf(to_f32(wr[c]), x[c], acc);
        acc = wave_sum(acc);
        if (lane == 0) y[r] = rscale ? (acc * rscale[r]) * scale : acc * scale;
    }
}

// ---------------------------------------------------------------- epilogues
// Common shape: units(), rows(u, rows[R]), store(u, rows, v[R]) (one thread per unit, final row sums),
// finish(smem) (every thread of the workgoup).

// y[row] = resid[row] + (sum * rscale[row]) * scale     (resid / rscale optional)
// matmul_kernel.cpp:26 (sum*scale) fused with add_kernel.cpp:5-14 (residual add, model.cpp:86-90/124-128).
template <int R>
struct EpiStore {
    float* y;
    const float* resid;
    const float* rscale;
    float scale;
    int nrows;
    int pre_u = -1;  // unit whose residual / row scales were prefetched at kernel entry
    float pre_r[R] = {}, pre_s[R] = {};
    __device__ int units() const { return (nrows + R - 1) / R; }
    __device__ void rows(int u, int* r) const {
#pragma unroll
        for (int i = 0; i < R; ++i) r[i] = min(u * R + i, nrows - 1);
    }
    // Entry prefetch (issued before the weight stream, consumed after it): unconditional loads from
    // selected valid pointers, so no branch makes the compiler's vmcnt waits conservative.
    __device__ void prefetch_a(int u) {
        pre_u = u;
        const float* rp = resid ? resid : y;
        const float* sp = rscale ? rscale : y;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = min(u * R + i, nrows - 1);
            pre_r[i] = rp[row];
            pre_s[i] = sp[row];
        }
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int*, const float* v) const {
        const bool pre = u == pre_u;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = u * R + i;
            if (row < nrows) {
                float a = rscale ? v[i] * (pre ? pre_s[i] : rscale[row]) : v[i];
                a = a * scale;
                y[row] = resid ? (pre ? pre_r[i] : resid[row]) + a : a;
            }
        }
    }
    __device__ void finish(float*) const {}
};

// EpiStore whose residual is x + p_0 + ... + p_{NP-1} (the K-split wo's partials, summed in XStageSum's order,
// so the residual is bit-identical to the x1 the gate/up GEMV normalised): y[row] = x1[row] + sum * rscale[row].
template <int R, int NP>
struct EpiStoreSum {
    float* y;
    const float* resid;  // x
    const float* parts;  // [NP][nrows]
    const float* rscale;
    int nrows;
    int pre_u = -1;
    float pre_r[R] = {}, pre_s[R] = {};
    __device__ int units() const { return (nrows + R - 1) / R; }
    __device__ void rows(int u, int* r) const {
#pragma unroll
        for (int i = 0; i < R; ++i) r[i] = min(u * R + i, nrows - 1);
    }
    __device__ float x1(int row) const {
        float v = resid[row];
#pragma unroll
        for (int k = 0; k < NP; ++k) v += parts[(size_t)k * nrows + row];
        return v;
    }
    __device__ void prefetch_a(int u) {
        pre_u = u;
        const float* sp = rscale ? rscale : resid;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = min(u * R + i, nrows - 1);
            pre_r[i] = x1(row);
            pre_s[i] = sp[row];
        }
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int*, const float* v) const {
        const bool pre = u == pre_u;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = u * R + i;
            if (row < nrows) {
                const float a = rscale ? v[i] * (pre ? pre_s[i] : rscale[row]) : v[i];
                y[row] = (pre ? pre_r[i] : x1(row)) + a;
            }
        }
    }
    __device__ void finish(float*) const {}
};

// K-split wo (model.cpp:80-83 without the residual add): the [D][QD] weight read as a [D * ks][QD / ks] matrix
// (row d * ks + k = columns [k QD / ks, (k + 1) QD / ks) of row d, the same bytes), unit u = (k = u / D, d = u % D)
// so a workgroup's units share one k; part[k][d] = (row sum) * rscale[d]. The residual add moves to the consumers
// (XStageSum, EpiStoreSum).
struct EpiKPart {
    float* part;  // [ks][D]
    const float* rscale;
    int D, ks;
    int pre_u = -1;
    float pre_s = 1.0f;
    __device__ int units() const { return D * ks; }
    __device__ void rows(int u, int* r) const {
        const int k = u / D;
        r[0] = (u - k * D) * ks + k;
    }
    __device__ void prefetch_a(int u) {
        pre_u = u;
        const int k = u / D;
        pre_s = rscale ? rscale[u - k * D] : 1.0f;
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int*, const float* v) const {
        const int k = u / D;
        const float s = rscale ? (u == pre_u ? pre_s : rscale[u - k * D]) : 1.0f;
        part[u] = v[0] * s;
    }
    __device__ void finish(float*) const {}
};

// Fused q/k/v projection + RoPE + KV-cache write (model.cpp:54-67): a unit is the RoPE pair of rows
// {d, d+hd/2} of one head of the fused [q; k; v] weight, so the rotation (rope_kernel.cpp:31-38) is
// applied to the two row sums in registers and K/V go straight into the head-major cache
// [kv_head][T][hd] of this layer.
template <typename KT>
struct EpiQKV {
    float* q_out;              // [hq*hd]
    KT* kc;                    // layer base, head-major [hkv][T][hd]
    KT* vc;
    const float* rscale;       // int8 row scales of the fused rows (nullable)
    const int32_t* pos_dev;
    const float* sin_t;        // [T][hd/2]
    const float* cos_t;
    int hq, hkv, hd, T;
    int pre_u = -1, pre_pos = 0;  // entry prefetch: position, row scales; then the RoPE table entries
    float pre_s0 = 1.0f, pre_s1 = 1.0f, pre_sin = 0.0f, pre_cos = 1.0f;
    __device__ int units() const { return (hq + 2 * hkv) * (hd / 2); }
    __device__ void prefetch_a(int u) {
        pre_u = u;
        pre_pos = *pos_dev;
        int r[2];
        rows(u, r);
        // without row scales: an unconditional load of a known-valid element (sin_t[0]), never a row
        // index into the [T][hd/2] table
        const float* sp = rscale ? rscale : sin_t;
        pre_s0 = sp[rscale ? r[0] : 0];
        pre_s1 = sp[rscale ? r[1] : 0];
    }
    // after the input commit (the position has landed with the input): the table row of this position
    __device__ void prefetch_b(int u) {
        const int half = hd / 2;
        const int d = u - (u / half) * half;
        pre_sin = sin_t[pre_pos * half + d];
        pre_cos = cos_t[pre_pos * half + d];
    }
    __device__ void rows(int u, int* r) const {
        const int half = hd / 2;
        const int uh = u / half;
        const int d = u - uh * half;
        r[0] = uh * hd + d;
        r[1] = uh * hd + d + half;
    }
    __device__ void store(int u, const int* r, const float* acc) const {
        const int half = hd / 2;
        const int uh = u / half;
        const int d = u - uh * half;
        const bool pre = u == pre_u;
        float a0 = acc[0], a1 = acc[1];
        if (rscale) {
            a0 *= pre ? pre_s0 : rscale[r[0]];
            a1 *= pre ? pre_s1 : rscale[r[1]];
        }
        const int pos = pre ? pre_pos : *pos_dev;
        if (uh < hq + hkv) {  // q or k: rotate (rope_kernel.cpp:30-38)
            const float fci = pre ? pre_sin : sin_t[pos * half + d], fcr = pre ? pre_cos : cos_t[pos * half + d];
            const float r0 = a0 * fcr - a1 * fci;
            const float r1 = a1 * fcr + a0 * fci;
            if (uh < hq) {
                float* q = q_out + (size_t)uh * hd;
                q[d] = r0;
                q[d + half] = r1;
            } else {
                KT* k = kc + ((size_t)(uh - hq) * T + pos) * hd;
                k[d] = from_f32<KT>(r0);
                k[d + half] = from_f32<KT>(r1);
            }
        } else {
            KT* v = vc + ((size_t)(uh - hq - hkv) * T + pos) * hd;
            v[d] = from_f32<KT>(a0);
            v[d + half] = from_f32<KT>(a1);
        }
    }
    __device__ void finish(float*) const {}
};

// Fused gate/up projection + activation (model.cpp:99-115): fused weight rows [gate(I); up(I)], unit =
// {gate i, up i}; act = sigmoid(g)*u (swiglu_kernel.cpp:12-13) or SiLU(g)*u.
struct EpiSwiGLU {
    float* act;
    const float* rscale;
    int inter;  // I (local)
    int silu;
    int pre_u = -1;
    float pre_s0 = 1.0f, pre_s1 = 1.0f;
    __device__ int units() const { return inter; }
    __device__ void rows(int u, int* r) const {
        r[0] = u;
        r[1] = inter + u;
    }
    __device__ void prefetch_a(int u) {
        pre_u = u;
        const float* sp = rscale ? rscale : act;
        pre_s0 = sp[rscale ? u : 0];
        pre_s1 = sp[rscale ? inter + u : 0];
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int* r, const float* acc) const {
        const bool pre = u == pre_u;
        float g = acc[0], up = acc[1];
        if (rscale) {
            g *= pre ? pre_s0 : rscale[r[0]];
            up *= pre ? pre_s1 : rscale[r[1]];
        }
        float t = 1.0f / (1.0f + expf(-g));
        if (silu) t = g * t;
        act[u] = t * up;
    }
    __device__ void finish(float*) const {}
};

// LM head (model.cpp:136-139, tied to the embedding) + first stage of the device argmax: logits are
// stored and each workgroup writes the max orderable key of the rows it owned to keys[blockIdx.x]
// (deterministic two-stage reduction; no atomics on one word).
template <int R>
struct EpiLogits {
    float* logits;
    unsigned long long* keys;
    const float* rscale;
    int nrows;
    int vocab_off;
    unsigned long long best;
    int pre_u = -1;
    float pre_s[R] = {};
    __device__ int units() const { return (nrows + R - 1) / R; }
    __device__ void rows(int u, int* r) const {
#pragma unroll
        for (int i = 0; i < R; ++i) r[i] = min(u * R + i, nrows - 1);
    }
    __device__ void prefetch_a(int u) {
        pre_u = u;
        const float* sp = rscale ? rscale : logits;
#pragma unroll
        for (int i = 0; i < R; ++i) pre_s[i] = sp[min(u * R + i, nrows - 1)];
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int*, const float* acc) {
        const bool pre = u == pre_u;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = u * R + i;
            if (row < nrows) {
                const float a = rscale ? acc[i] * (pre ? pre_s[i] : rscale[row]) : acc[i];
                logits[row] = a;
                const unsigned long long k = argmax_key(a, (unsigned)(row + vocab_off));
                best = k > best ? k : best;
            }
        }
    }
    __device__ void finish(float* smem) {
        unsigned long long* red = reinterpret_cast<unsigned long long*>(smem);
        best = wave_max_u64(best);
        __syncthreads();
        const int wave = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) red[wave] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long b = 0;
            for (int w = 0; w < (kGemvThreads >> 6); ++w) b = red[w] > b ? red[w] : b;
            keys[blockIdx.x] = b;
        }
    }
};

}  // namespace sli

namespace sli {

constexpr int kGemvMaxCols = 16384 - kGemvLdsHead;  // x staged in 64 KiB of LDS (<= kGemvThreads*4*kGemvStageV4)
// persistent grid: one workgroup per CU of the current device (MI355X: 8 XCDs x 32 CUs = 256)
// one persistent workgroup per CU; SLI_DEBUG_GEMV_MAX_BLOCKS caps it (tests: rank processes sharing one GPU
// under the per-workgroup exchange, whose grids must fit the device together)
inline int gemv_max_blocks() {
    static const int cap = [] {
        const char* e = getenv("SLI_DEBUG_GEMV_MAX_BLOCKS");
        return e ? atoi(e) : 0;
    }();
    return cap > 0 ? std::min(cap, device_cus()) : device_cus();
}

// Grid: enough workgroups for every (unit, column part) item to have a wave, capped at the persistent
// size; the balanced schedule in gemv_block spreads the items over whatever grid this returns.
inline int gemv_blocks(int units, int csplit = 1) {
    const int maxb = gemv_max_blocks();
    const int items = units * csplit;
    int b = (items + (kGemvThreads / 64) - 1) / (kGemvThreads / 64);
    b = b < units ? b : units;  // every workgroup owns at least one unit
    return b < maxb ? (b > 0 ? b : 1) : maxb;
}

// Wave-balanced grid for unsplit launches. A wave owns whole units, so at the full grid the waves differ by one
// unit, and when units / waves is far from an integer the waves with one unit fewer finish early and the
// launch's tail streams on part of the chip (gate/up at 7B: 11008 units on 4096 waves = 2.69, 31 % of the
// waves idle for the last third). The smallest grid at which no wave holds more units than at the full grid
// gives every wave (nearly) the same count; it is taken when it keeps >= 7/8 of the workgroups, so each
// CU's share of the HBM stream stays under its per-CU fetch rate (gate/up: 230 workgroups, 31.4 -> 29.0 us,
// C1 358 -> 368 tok/s; qkv at 1.5 units per wave would need 192 workgroups: measured slower, 17.9 -> 20.5 us;
// profiles/r3_gemv_balance_ab.txt).
inline int gemv_balanced_blocks(int units) {
    const int b = gemv_blocks(units);
    const int w = kGemvThreads / 64;
    const int k = (units + b * w - 1) / (b * w);  // most units of a wave at the full grid
    const int g = (units + k * w - 1) / (k * w);
    // only where the full grid's tail is real (>= 8 % more unit slots than units; the LM head's 2.4 % measured
    // slower at 250 workgroups: 41.2 -> 43-44 us)
    return (g < b && 8 * g >= 7 * b && 100LL * k * b * w >= 108LL * units) ? g : b;
}

// Streaming waves per workgroup: with u units per workgroup and 16 waves, waves hold ceil(u / 16) or one
// fewer; when that leaves waves idle for a whole unit (qkv at 7B: 24 units per workgroup = 1.5 per wave,
// half the waves stream for half the launch), ceil(u / k) waves of k units each can take all of them.
// Measured (profiles/r3_gemv_balance_ab.txt): int8 qkv 12.8 -> 12.4 us with 12 waves of 2 units, C3 +0.8 %;
// fp16 qkv 18.1 -> 21.2 us (12 waves keep 3/4 of the bytes in flight per CU, and fp16 needs them) — so
// int8 weights only (the launch sites pass the weight type).
template <typename WT>
inline int gemv_wave_count(int units, int grid) {
    if (!std::is_same<WT, int8_t>::value) return kGemvThreads / 64;
    const int w = kGemvThreads / 64;
    const int upw = (units + grid - 1) / grid;  // most units of a workgroup
    const int k = (upw + w - 1) / w;
    const int c = (upw + k - 1) / k;
    return c >= w / 2 ? c : w;
}

// NS: split partials a thread loads with its input (every live split of a context up to NS * ppwg
// positions in one batch; more splits are read from memory one by one during the merge)
// weight steps in flight per wave while the merge staging runs (A/B knob)
#ifndef SLI_WO_NB
#define SLI_WO_NB 2
#endif
template <typename WT, int R, int U, bool NT, class Epi, int NS = 8, int NB = SLI_WO_NB>
hipError_t launch_gemv_merge(const WT* W, const GemvIn& in_, const Epi& epi, const AttnMergeIn& am, int units,
                             hipStream_t s) {
    if (in_.csplit != 1) return hipErrorInvalidValue;  // the merge-staged wo GEMV runs unsplit
    const int grid = gemv_balanced_blocks(units);
    GemvIn in = in_;
    in.cw = gemv_wave_count<WT>(units, grid);
    const size_t lds = gemv_lds_bytes(in.cols) + sizeof(float) * gemv_res_floats(units, grid, R);
    hipLaunchKernelGGL((gemv_merge_kernel<WT, R, U, NT, Epi, NS, NB>), dim3(grid), dim3(kGemvThreads), lds, s, W, in,
                       epi, am);
    return hipGetLastError();
}

// K-split wo: the grid must keep every workgroup's units inside one block k (gemv_block's partition b * N / g):
// g = ks * m with m dividing D, so each workgroup holds D / m units of one k. 0 if no such grid fits the chip.
inline int gemv_ksplit_grid(int D, int ks) {
    const int maxb = gemv_max_blocks();
    for (int m = maxb / ks; m >= 1; --m)
        if (D % m == 0) return ks * m;
    return 0;
}
template <typename WT, int R, int U, bool NT, class Epi, int NS = 8, int NB = SLI_WO_NB>
hipError_t launch_gemv_merge_ks(const WT* W, const GemvIn& in_, const Epi& epi, const AttnMergeIn& am, int grid,
                                hipStream_t s) {
    const int units = am.ksplit * am.kunits;
    if (in_.csplit != 1 || grid <= 0 || grid % am.ksplit || am.kunits % (grid / am.ksplit)) return hipErrorInvalidValue;
    GemvIn in = in_;
    in.cw = gemv_wave_count<WT>(units, grid);
    const size_t lds = gemv_lds_bytes(in.cols) + sizeof(float) * gemv_res_floats(units, grid, R);
    hipLaunchKernelGGL((gemv_merge_kernel<WT, R, U, NT, Epi, NS, NB>), dim3(grid), dim3(kGemvThreads), lds, s, W, in,
                       epi, am);
    return hipGetLastError();
}
template <typename WT, int R, int U, bool NT, class Epi, int NP, int NB = 2>
hipError_t launch_gemv_sum(const WT* W, const GemvIn& in_, const Epi& epi, const float* parts, int units,
                           hipStream_t s) {
    if (in_.csplit != 1 || in_.cols > 4 * kGemvThreads) return hipErrorInvalidValue;  // XStageSum: one round
    GemvIn in = in_;
    const int grid = gemv_balanced_blocks(units);
    in.cw = gemv_wave_count<WT>(units, grid);
    const size_t lds = gemv_lds_bytes(in.cols) + sizeof(float) * gemv_res_floats(units, grid, R);
    hipLaunchKernelGGL((gemv_sum_kernel<WT, R, U, NT, Epi, NP, NB>), dim3(grid), dim3(kGemvThreads), lds, s, W, in,
                       epi, parts);
    return hipGetLastError();
}

template <typename WT, int R, int U, bool NT, class Epi, int NB = 2, bool SPLIT = false>
hipError_t launch_gemv(const WT* W, const GemvIn& in_, const Epi& epi, int units, hipStream_t s) {
    if (!SPLIT && in_.csplit != 1) return hipErrorInvalidValue;  // a split needs the SPLIT instantiation
    GemvIn in = in_;
    const int grid = in.csplit == 1 ? gemv_balanced_blocks(units) : gemv_blocks(units, in.csplit);
    in.cw = in.csplit == 1 ? gemv_wave_count<WT>(units, grid) : kGemvThreads / 64;
    const size_t lds = gemv_lds_bytes(in.cols) + sizeof(float) * gemv_res_floats(units, grid, R, in.csplit);
    hipLaunchKernelGGL((gemv_kernel<WT, R, U, NT, Epi, NB, SPLIT>), dim3(grid), dim3(kGemvThreads), lds, s, W, in,
                       epi);
    return hipGetLastError();
}

// Vectors in flight per lane: the per-shape U (fp16, tools/gemv_lab) halved for int8, whose 16-byte
// vector holds twice the columns: the same columns per chunk, two chunks per 4096-column row instead of
// one, so a wave's second buffer streams while the first is consumed (measured C3: 414 -> 447 tok/s;
// a quarter U: 431).
//
// Small matrices (tensor-parallel shards: TP-8 q/k/v has 768 two-row units for 4096 waves) split each
// unit's rows over CS column parts (gemv.h gemv_block): CS = the power of two that gives every wave of the
// chip an item, at the widest U whose chunks still cover CS parts per row (U, then 2, then 1). Full-size
// matrices (every TP-1 projection) keep CS = 1.
struct GemvSplit {
    int cs, u;  // column parts per unit, vectors per lane per chunk
};
template <typename WT, int U>
inline GemvSplit gemv_split(int units, int cols) {
    constexpr int UW = std::is_same<WT, int8_t>::value && U >= 2 ? U / 2 : U;
    const int waves = gemv_max_blocks() * (kGemvThreads / 64);
    int need = 1;
    while (need < 8 && units * need < waves) need *= 2;
    const int nvec = cols / Vec16<WT>::N;
    auto cpr = [&](int u) { return (nvec + 64 * u - 1) / (64 * u); };
    if (need == 1) return {1, UW};
    if (need <= cpr(UW)) return {need, UW};
    if (UW > 2 && need <= cpr(2)) return {need, 2};
    return {std::max(1, std::min(need, cpr(1))), 1};
}
template <typename WT, int R, int U, bool NT, class Epi>
hipError_t launch_gemv_u(const WT* W, const GemvIn& in_, const Epi& epi, int units, hipStream_t s) {
    constexpr int UW = std::is_same<WT, int8_t>::value && U >= 2 ? U / 2 : U;
    GemvIn in = in_;
    const GemvSplit sp = gemv_split<WT, U>(units, in.cols);
    in.csplit = sp.cs;
    if (sp.cs == 1) return launch_gemv<WT, R, UW, NT>(W, in, epi, units, s);
    if (sp.u == UW) return launch_gemv<WT, R, UW, NT, Epi, 2, true>(W, in, epi, units, s);
    if constexpr (UW > 2) {
        if (sp.u == 2) return launch_gemv<WT, R, 2, NT, Epi, 2, true>(W, in, epi, units, s);
    }
    return launch_gemv<WT, R, 1, NT, Epi, 2, true>(W, in, epi, units, s);
}

}  // namespace sli
