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
#include "common.h"

namespace sli {

struct GemvIn {
    const float* x;       // [cols] fp32 input vector
    const float* norm_w;  // nullptr: plain; else fused RMSNorm weight [cols]
    float eps;
    int cols;
};

constexpr int kGemvThreads = 256;
constexpr int kGemvLdsHead = 64;  // floats of reduction scratch in front of the staged x

inline size_t gemv_lds_bytes(int cols) { return sizeof(float) * (size_t)(kGemvLdsHead + cols); }

// Stage x (optionally RMS-normalised) into LDS. All LDS lives in one dynamic array (G17: no static
// __shared__ in front of the dynamic region, so the b128 reads stay 16-byte aligned).
__device__ __forceinline__ void gemv_stage_x(float* smem, const GemvIn& in) {
    float* red = smem;
    float* xs = smem + kGemvLdsHead;
    const int tid = threadIdx.x;
    const int nt = blockDim.x;
    if (in.norm_w == nullptr) {
        for (int c = tid; c < in.cols; c += nt) xs[c] = in.x[c];
        return;
    }
    float ss = 0.0f;
    for (int c = tid; c < in.cols; c += nt) {
        float v = in.x[c];
        xs[c] = v;
        ss += v * v;
    }
    ss = wave_sum(ss);
    const int wave = tid >> 6;
    if ((tid & 63) == 0) red[wave] = ss;
    __syncthreads();
    if (tid == 0) {
        float t = 0.0f;
        for (int w = 0; w < (nt >> 6); ++w) t += red[w];
        float tep = t / (float)in.cols;   // rms_kernel.cpp:17
        float rms = sqrtf(tep + in.eps);  // :18
        red[32] = 1.0f / rms;             // :19
    }
    __syncthreads();
    const float inv = red[32];
    for (int c = tid; c < in.cols; c += nt) xs[c] = (xs[c] * inv) * in.norm_w[c];  // :20-22
}

template <typename WT, int R, int U, bool NT, class Epi>
__global__ void __launch_bounds__(kGemvThreads) gemv_kernel(const WT* __restrict__ W, GemvIn in, Epi epi_in) {
    Epi epi = epi_in;  // mutable per-thread copy (EpiLogits keeps a running key)
    extern __shared__ __attribute__((aligned(16))) float smem[];
    gemv_stage_x(smem, in);
    __syncthreads();
    const float* xs = smem + kGemvLdsHead;

    constexpr int EPV = Vec16<WT>::N;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nwaves = blockDim.x >> 6;
    const int cols = in.cols;
    const int nvec = cols / EPV;
    const size_t row_bytes = (size_t)cols * sizeof(WT);
    const int nunits = epi.units();

    for (int u = blockIdx.x * nwaves + wave; u < nunits; u += gridDim.x * nwaves) {
        int rows[R];
        epi.rows(u, rows);
        const char* wp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) wp[r] = reinterpret_cast<const char*>(W) + (size_t)rows[r] * row_bytes;
        float acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = 0.0f;

        int v = lane;
        for (; v + (U - 1) * 64 < nvec; v += U * 64) {
            u32x4 w[U][R];
#pragma unroll
            for (int j = 0; j < U; ++j)
#pragma unroll
                for (int r = 0; r < R; ++r) w[j][r] = load16<NT>(wp[r] + (size_t)(v + j * 64) * 16);
#pragma unroll
            for (int j = 0; j < U; ++j) {
                float xv[EPV];
                const float4* xp = reinterpret_cast<const float4*>(xs + (size_t)(v + j * 64) * EPV);
#pragma unroll
                for (int e = 0; e < EPV / 4; ++e) {
                    float4 t = xp[e];
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
        for (; v < nvec; v += 64) {
            u32x4 w[R];
#pragma unroll
            for (int r = 0; r < R; ++r) w[r] = load16<NT>(wp[r] + (size_t)v * 16);
            float xv[EPV];
            const float4* xp = reinterpret_cast<const float4*>(xs + (size_t)v * EPV);
#pragma unroll
            for (int e = 0; e < EPV / 4; ++e) {
                float4 t = xp[e];
                xv[4 * e] = t.x;
                xv[4 * e + 1] = t.y;
                xv[4 * e + 2] = t.z;
                xv[4 * e + 3] = t.w;
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float wf[EPV];
                Vec16<WT>::unpack(w[r], wf);
#pragma unroll
                for (int e = 0; e < EPV; ++e) acc[r] = fmaf(wf[e], xv[e], acc[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
        epi.store(u, rows, acc, lane);
    }
    epi.finish(smem);
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
// Common shape: units(), rows(u, rows[R]), store(u, rows, acc[R], lane), finish(smem).

// y[row] = resid[row] + (sum * rscale[row]) * scale     (resid / rscale optional)
// matmul_kernel.cpp:26 (sum*scale) fused with add_kernel.cpp:5-14 (residual add, model.cpp:86-90/124-128).
template <int R>
struct EpiStore {
    float* y;
    const float* resid;
    const float* rscale;
    float scale;
    int nrows;
    __device__ int units() const { return (nrows + R - 1) / R; }
    __device__ void rows(int u, int* r) const {
#pragma unroll
        for (int i = 0; i < R; ++i) r[i] = min(u * R + i, nrows - 1);
    }
    __device__ void store(int u, const int*, const float* acc, int lane) const {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = u * R + i;
            if (lane == i && row < nrows) {
                float a = rscale ? acc[i] * rscale[row] : acc[i];
                a = a * scale;
                y[row] = resid ? resid[row] + a : a;
            }
        }
    }
    __device__ void finish(float*) const {}
};

// Fused q/k/v projection + RoPE + KV-cache write (model.cpp:54-67): rows of the fused [q; k; v] weight
// are taken as RoPE pairs {d, d+1, d+hd/2, d+1+hd/2} of one head, so the rotation
// (rope_kernel.cpp:31-38) happens on the row sums in registers and K/V go straight into the
// head-major cache [kv_head][T][hd] of this layer.
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
    __device__ int units() const { return (hq + 2 * hkv) * (hd / 4); }
    __device__ void rows(int u, int* r) const {
        const int per = hd / 4;
        const int uh = u / per;
        const int d = (u - uh * per) * 2;
        const int base = uh * hd;
        r[0] = base + d;
        r[1] = base + d + 1;
        r[2] = base + d + hd / 2;
        r[3] = base + d + 1 + hd / 2;
    }
    __device__ void store(int u, const int* r, const float* acc, int lane) const {
        if (lane != 0) return;
        const int per = hd / 4;
        const int uh = u / per;
        const int d = (u - uh * per) * 2;
        float a0 = acc[0], a1 = acc[1], a2 = acc[2], a3 = acc[3];
        if (rscale) {
            a0 *= rscale[r[0]];
            a1 *= rscale[r[1]];
            a2 *= rscale[r[2]];
            a3 *= rscale[r[3]];
        }
        const int pos = *pos_dev;
        if (uh < hq + hkv) {  // q or k: rotate (rope_kernel.cpp:30-38)
            const float s0 = sin_t[pos * (hd / 2) + d], c0 = cos_t[pos * (hd / 2) + d];
            const float s1 = sin_t[pos * (hd / 2) + d + 1], c1 = cos_t[pos * (hd / 2) + d + 1];
            const float r0 = a0 * c0 - a2 * s0, r2 = a2 * c0 + a0 * s0;
            const float r1 = a1 * c1 - a3 * s1, r3 = a3 * c1 + a1 * s1;
            if (uh < hq) {
                float* q = q_out + (size_t)uh * hd;
                q[d] = r0;
                q[d + 1] = r1;
                q[d + hd / 2] = r2;
                q[d + 1 + hd / 2] = r3;
            } else {
                KT* k = kc + ((size_t)(uh - hq) * T + pos) * hd;
                k[d] = from_f32<KT>(r0);
                k[d + 1] = from_f32<KT>(r1);
                k[d + hd / 2] = from_f32<KT>(r2);
                k[d + 1 + hd / 2] = from_f32<KT>(r3);
            }
        } else {
            KT* v = vc + ((size_t)(uh - hq - hkv) * T + pos) * hd;
            v[d] = from_f32<KT>(a0);
            v[d + 1] = from_f32<KT>(a1);
            v[d + hd / 2] = from_f32<KT>(a2);
            v[d + 1 + hd / 2] = from_f32<KT>(a3);
        }
    }
    __device__ void finish(float*) const {}
};

// Fused gate/up projection + activation (model.cpp:99-115): fused weight rows [gate(I); up(I)], unit =
// {gate i, gate i+1, up i, up i+1}; act = sigmoid(g)*u (swiglu_kernel.cpp:12-13) or SiLU(g)*u.
struct EpiSwiGLU {
    float* act;
    const float* rscale;
    int inter;  // I (local), even
    int silu;
    __device__ int units() const { return inter / 2; }
    __device__ void rows(int u, int* r) const {
        r[0] = 2 * u;
        r[1] = 2 * u + 1;
        r[2] = inter + 2 * u;
        r[3] = inter + 2 * u + 1;
    }
    __device__ void store(int u, const int* r, const float* acc, int lane) const {
        if (lane != 0) return;
        float g0 = acc[0], g1 = acc[1], u0 = acc[2], u1 = acc[3];
        if (rscale) {
            g0 *= rscale[r[0]];
            g1 *= rscale[r[1]];
            u0 *= rscale[r[2]];
            u1 *= rscale[r[3]];
        }
        float t0 = 1.0f / (1.0f + expf(-g0));
        float t1 = 1.0f / (1.0f + expf(-g1));
        if (silu) {
            t0 = g0 * t0;
            t1 = g1 * t1;
        }
        act[2 * u] = t0 * u0;
        act[2 * u + 1] = t1 * u1;
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
    __device__ int units() const { return (nrows + R - 1) / R; }
    __device__ void rows(int u, int* r) const {
#pragma unroll
        for (int i = 0; i < R; ++i) r[i] = min(u * R + i, nrows - 1);
    }
    __device__ void store(int u, const int*, const float* acc, int lane) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = u * R + i;
            if (row < nrows) {
                const float a = rscale ? acc[i] * rscale[row] : acc[i];
                if (lane == i) logits[row] = a;
                const unsigned long long k = argmax_key(a, (unsigned)(row + vocab_off));
                best = k > best ? k : best;
            }
        }
    }
    __device__ void finish(float* smem) {
        unsigned long long* red = reinterpret_cast<unsigned long long*>(smem);
        __syncthreads();
        const int wave = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) red[wave] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long b = 0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) b = red[w] > b ? red[w] : b;
            keys[blockIdx.x] = b;
        }
    }
};

}  // namespace sli

namespace sli {

constexpr int kGemvMaxCols = 16384 - kGemvLdsHead;  // x staged in <= 64 KiB of LDS
constexpr int kGemvMaxBlocks = 1024;                 // 4 workgroups per CU, grid-stride beyond

inline int gemv_blocks(int units) {
    int b = (units + (kGemvThreads / 64) - 1) / (kGemvThreads / 64);
    return b < kGemvMaxBlocks ? (b > 0 ? b : 1) : kGemvMaxBlocks;
}

template <typename WT, int R, int U, bool NT, class Epi>
hipError_t launch_gemv(const WT* W, const GemvIn& in, const Epi& epi, int units, hipStream_t s) {
    hipLaunchKernelGGL((gemv_kernel<WT, R, U, NT, Epi>), dim3(gemv_blocks(units)), dim3(kGemvThreads),
                       gemv_lds_bytes(in.cols), s, W, in, epi);
    return hipGetLastError();
}

}  // namespace sli
