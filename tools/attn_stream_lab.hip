// attn_stream_lab.hip — diagnostic: the LDS-streamed decode attention (tools/attn_stream.h) against the
// register-staged kernel (csrc/attention.h) on the C1 (MHA, ctx 2048) and C4 (batch 8 x GQA-4, ctx 4096)
// shapes: merged outputs compared, then both timed over NL distinct K/V caches in a replayed hipGraph
// (the merge launch included for both).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/attn_stream_lab.hip -o tools/attn_stream_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "attn_stream.h"

using namespace sli;

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void fill_h(__half* p, size_t n, unsigned seed, float scale) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        p[i] = __float2half(((float)(h & 0xFFFF) / 65536.0f - 0.5f) * scale);
    }
}

// the ring pipeline alone (same issue / counted wait / barrier as attn_stream_kernel, a single LDS
// read per chunk instead of the attention): what LDS-DMA streaming costs on its own
template <int D, int W, int P>
__global__ void __launch_bounds__(64 * W) dma_ring_kernel(const char* base, long long per_wg, float* sink) {
    constexpr int CH = W * P * 1024;
    __shared__ __attribute__((aligned(1024))) char ring[D][CH];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const char* b = base + per_wg * blockIdx.x;
    const int nch = (int)(per_wg / CH);
    auto issue = [&](int c) {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int piece = wave * P + j;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(b + (long long)c * CH + piece * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void*)(&ring[c % D][piece * 1024]), 16, 0, 0);
        }
    };
#pragma unroll
    for (int c = 0; c < D - 1; ++c)
        if (c < nch) issue(c);
    float acc = 0.0f;
    for (int c = 0; c < nch; ++c) {
        as_wait_chunk<D, P>(min(D - 2, nch - 1 - c));
        __builtin_amdgcn_s_barrier();
        if (c + D - 1 < nch) issue(c + D - 1);
        acc += reinterpret_cast<const float*>(ring[c % D])[threadIdx.x];
    }
    if (acc == 1.2345f) sink[threadIdx.x] = acc;
}

template <int U>
__global__ void __launch_bounds__(1024) reg_stream_kernel(const char* base, long long per_wg, float* sink) {
    const char* b = base + per_wg * blockIdx.x;
    const int nvec = (int)(per_wg / 16);
    float acc = 0.0f;
    for (int v = threadIdx.x; v < nvec; v += U * 1024) {
        u32x4 w[U];
#pragma unroll
        for (int j = 0; j < U; ++j) w[j] = load16<false>(b + (size_t)min(v + j * 1024, nvec - 1) * 16);
#pragma unroll
        for (int j = 0; j < U; ++j) acc += __uint_as_float(w[j].x ^ w[j].w);
    }
    if (acc == 1.2345f) sink[threadIdx.x] = acc;
}

static void dma_bench() {
    const long long bytes = 64ll << 20;  // 64 MiB, one pass
    const int NL = 6;
    std::vector<char*> buf(NL);
    for (auto& p : buf) {
        CK(hipMalloc(&p, bytes));
        CK(hipMemset(p, 1, bytes));
    }
    float* sink;
    CK(hipMalloc(&sink, 4096));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto time_it = [&](auto fn) {
        for (int l = 0; l < NL; ++l) fn(l);
        CK(hipStreamSynchronize(s));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < 4; ++r)
            for (int l = 0; l < NL; ++l) fn(l);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return 1000.0 * ms / (4 * NL);
    };
    auto rep = [&](const char* n, double us) { printf("stream 64 MiB %-28s %7.2f us %6.0f GB/s\n", n, us, bytes / (us * 1e3)); };
    rep("reg U=8 grid 256", time_it([&](int l) { hipLaunchKernelGGL(reg_stream_kernel<8>, dim3(256), dim3(1024), 0, s, buf[l], bytes / 256, sink); }));
    rep("dma ring D8 W4 P2 grid 256", time_it([&](int l) { hipLaunchKernelGGL((dma_ring_kernel<8, 4, 2>), dim3(256), dim3(256), 0, s, buf[l], bytes / 256, sink); }));
    rep("dma ring D8 W8 P1 grid 256", time_it([&](int l) { hipLaunchKernelGGL((dma_ring_kernel<8, 8, 1>), dim3(256), dim3(512), 0, s, buf[l], bytes / 256, sink); }));
    rep("dma ring D16 W4 P2 grid 256", time_it([&](int l) { hipLaunchKernelGGL((dma_ring_kernel<16, 4, 1>), dim3(256), dim3(256), 0, s, buf[l], bytes / 256, sink); }));
    rep("dma ring D4 W4 P2 grid 512", time_it([&](int l) { hipLaunchKernelGGL((dma_ring_kernel<4, 4, 2>), dim3(512), dim3(256), 0, s, buf[l], bytes / 512, sink); }));
    rep("dma ring D8 W16 P1 grid 256", time_it([&](int l) { hipLaunchKernelGGL((dma_ring_kernel<8, 16, 1>), dim3(256), dim3(1024), 0, s, buf[l], bytes / 256, sink); }));
    for (auto p : buf) CK(hipFree(p));
    CK(hipFree(sink));
    CK(hipStreamDestroy(s));
}

template <int G, int D, int W, int P>
static void run(const char* name, int nkv, int T, int pos, int NL, int ppwg) {
    constexpr int HD = 128;
    using Geo = AttnGeom<__half, HD>;
    const int H = nkv * G;
    const int splits_old = (T + Geo::PPWG - 1) / Geo::PPWG;
    const int splits_new = (T + ppwg - 1) / ppwg;
    const size_t per = (size_t)nkv * T * HD;
    std::vector<__half*> K(NL), V(NL);
    for (int l = 0; l < NL; ++l) {
        CK(hipMalloc(&K[l], per * 2));
        CK(hipMalloc(&V[l], per * 2));
        fill_h<<<1024, 256>>>(K[l], per, 3 + l, 2.0f);
        fill_h<<<1024, 256>>>(V[l], per, 7 + l, 2.0f);
    }
    __half* qh;
    float *q, *out0, *out1, *part;
    unsigned* cnt;
    CK(hipMalloc(&q, sizeof(float) * H * HD));
    CK(hipMalloc(&qh, sizeof(__half) * H * HD));
    CK(hipMalloc(&out0, sizeof(float) * H * HD));
    CK(hipMalloc(&out1, sizeof(float) * H * HD));
    const int smax = std::max(splits_old, splits_new);
    CK(hipMalloc(&part, sizeof(float) * (size_t)H * smax * (HD + kAttnPartPad)));
    CK(hipMalloc(&cnt, sizeof(unsigned) * nkv));
    CK(hipMemset(cnt, 0, sizeof(unsigned) * nkv));
    fill_h<<<64, 256>>>(qh, (size_t)H * HD, 99, 0.5f);
    std::vector<__half> hq(H * HD);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hq.data(), qh, hq.size() * 2, hipMemcpyDeviceToHost));
    std::vector<float> fq(H * HD);
    for (int i = 0; i < H * HD; ++i) fq[i] = __half2float(hq[i]);
    CK(hipMemcpy(q, fq.data(), fq.size() * 4, hipMemcpyHostToDevice));
    auto args = [&](int l, float* out, int splits, int pp, int defer) {
        AttnArgs<__half> a{q, K[l], V[l], HD, (long long)T * HD, part, out, cnt, nullptr, pos, nkv, splits,
                           1.0f / sqrtf((float)HD), nkv, 0};
        a.ppwg = pp;
        a.defer_merge = defer;
        return a;
    };
    auto old_k = [&](int l, hipStream_t s) {
        hipLaunchKernelGGL((attn_partial_kernel<__half, HD, G>), dim3(nkv * splits_old), dim3(64 * attn_waves(G)), 0, s,
                           args(l, out0, splits_old, 0, 2));
        hipLaunchKernelGGL((attn_merge_kernel<__half, HD, G>), dim3(nkv), dim3(kAttnMergeThreads), 0, s,
                           args(l, out0, splits_old, 0, 2));
    };
    auto new_k = [&](int l, hipStream_t s) {
        hipLaunchKernelGGL((attn_stream_kernel<__half, HD, G, D, W, P>), dim3(nkv * splits_new), dim3(64 * W), 0, s,
                           args(l, out1, splits_new, ppwg, 2));
        hipLaunchKernelGGL((attn_merge_kernel<__half, HD, G>), dim3(nkv), dim3(kAttnMergeThreads), 0, s,
                           args(l, out1, splits_new, ppwg, 2));
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    old_k(0, s);
    new_k(0, s);
    CK(hipStreamSynchronize(s));
    std::vector<float> h0(H * HD), h1(H * HD);
    CK(hipMemcpy(h0.data(), out0, h0.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), out1, h1.size() * 4, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    for (int i = 0; i < H * HD; ++i) {
        md = std::max(md, (double)fabsf(h0[i] - h1[i]));
        mx = std::max(mx, (double)fabsf(h0[i]));
    }
    auto time_it = [&](auto fn) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        for (int l = 0; l < NL; ++l) fn(l, s);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int reps = 10;
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        return 1000.0 * ms / (reps * NL);
    };
    const double bytes = 2.0 * nkv * (pos + 1.0) * HD * 2;
    const double t0 = time_it(old_k), t1 = time_it(new_k);
    {  // stamps of one streamed launch (after a cold launch on another cache): entry spread, first chunk, loop, merge
        const int nb = nkv * splits_new;
        unsigned long long* st;
        CK(hipMalloc(&st, 8 * 4 * nb));
        CK(hipMemset(st, 0, 8 * 4 * nb));
        AttnArgs<__half> aa = args(NL - 1, out1, splits_new, ppwg, 2);
        aa.stamps = st;
        new_k(0, s);
        hipLaunchKernelGGL((attn_stream_kernel<__half, HD, G, D, W, P>), dim3(nb), dim3(64 * W), 0, s, aa);
        CK(hipStreamSynchronize(s));
        std::vector<unsigned long long> h(4 * nb);
        CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t00 = ~0ull, te = 0;
        double e = 0, f = 0, lp = 0, mg = 0;
        for (int i = 0; i < nb; ++i) t00 = std::min(t00, h[4 * i]);
        for (int i = 0; i < nb; ++i) {
            e = std::max(e, (h[4 * i] - t00) * 0.01);
            f += (h[4 * i + 1] - h[4 * i]) * 0.01;
            lp += (h[4 * i + 2] - h[4 * i + 1]) * 0.01;
            mg += (h[4 * i + 3] - h[4 * i + 2]) * 0.01;
            te = std::max(te, h[4 * i + 3]);
        }
        printf("    stamps: entry spread %.2f, entry->chunk0 %.2f, loop %.2f, merge+store %.2f, span %.2f us\n", e,
               f / nb, lp / nb, mg / nb, (te - t00) * 0.01);
        CK(hipFree(st));
    }
    printf("%-3s G=%d D=%d W=%2d P=%d ppwg=%4d: max|out diff| %.2e (max|out| %.2e) | register-staged %6.2f us %5.0f GB/s | "
           "LDS-streamed %6.2f us %5.0f GB/s (grid %d)\n",
           name, G, D, W, P, ppwg, md, mx, t0, bytes / (t0 * 1e3), t1, bytes / (t1 * 1e3), nkv * splits_new);
    fflush(stdout);
    for (int l = 0; l < NL; ++l) {
        CK(hipFree(K[l]));
        CK(hipFree(V[l]));
    }
    CK(hipFree(q));
    CK(hipFree(qh));
    CK(hipFree(out0));
    CK(hipFree(out1));
    CK(hipFree(part));
    CK(hipFree(cnt));
    CK(hipStreamDestroy(s));
}

int main() {
    run<1, 8, 4, 2>("C1", 32, 2048, 2047, 8, 256);
    run<1, 4, 16, 1>("C1", 32, 2048, 2047, 8, 256);
    run<1, 8, 8, 1>("C1", 32, 2048, 2047, 8, 256);
    run<1, 4, 8, 1>("C1", 32, 2048, 2047, 8, 128);
    run<4, 4, 16, 1>("C4", 64, 4096, 4095, 3, 1024);
    run<4, 8, 8, 1>("C4", 64, 4096, 4095, 3, 1024);
    run<4, 4, 8, 1>("C4", 64, 4096, 4095, 3, 512);
    run<4, 4, 4, 2>("C4", 64, 4096, 4095, 3, 512);
    return 0;
}
