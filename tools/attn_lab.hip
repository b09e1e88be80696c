// attn_lab.hip — diagnostic: the split-context decode attention (csrc/attention.h) on the C1 (MHA, ctx
// 2048) and C4 (batch 8 x GQA-4, ctx 4096) shapes at chosen waves per workgroup, timed over NL distinct
// K/V caches inside a replayed hipGraph (no Infinity-Cache re-reads), with per-workgroup phase stamps.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/attn_lab.hip -o tools/attn_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../simplellminference_amd/csrc/attention.h"

using namespace sli;

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void fill_h(__half* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        p[i] = __float2half(((float)(h & 0xFFFF) / 65536.0f - 0.5f) * 2.0f);
    }
}

template <int G, int WAVES, bool LATE_V = false>
static void run(const char* name, int nkv, int T, int pos, int NL) {
    constexpr int HD = 128;
    using Geo = AttnGeom<__half, HD>;
    const int splits = (T + Geo::PPWG - 1) / Geo::PPWG;
    const size_t per = (size_t)nkv * T * HD;
    std::vector<__half*> K(NL), V(NL);
    for (int l = 0; l < NL; ++l) {
        CK(hipMalloc(&K[l], per * 2));
        CK(hipMalloc(&V[l], per * 2));
        fill_h<<<1024, 256>>>(K[l], per, 3 + l);
        fill_h<<<1024, 256>>>(V[l], per, 7 + l);
    }
    float *q, *out, *part;
    unsigned* cnt;
    unsigned long long* st;
    const int H = nkv * G;
    CK(hipMalloc(&q, sizeof(float) * H * HD));
    CK(hipMalloc(&out, sizeof(float) * H * HD));
    CK(hipMalloc(&part, sizeof(float) * (size_t)H * splits * (HD + kAttnPartPad)));
    CK(hipMalloc(&cnt, sizeof(unsigned) * nkv));
    CK(hipMemset(cnt, 0, sizeof(unsigned) * nkv));
    CK(hipMemset(q, 0, sizeof(float) * H * HD));
    const int blocks = nkv * splits;
    CK(hipMalloc(&st, sizeof(unsigned long long) * 4 * blocks));
    CK(hipDeviceSynchronize());
    auto args = [&](int l, unsigned long long* stamps) {
        AttnArgs<__half> a{q, K[l], V[l], HD, (long long)T * HD, part, out, cnt, nullptr, pos, nkv, splits,
                           1.0f / sqrtf((float)HD), nkv, 0, stamps};
        return a;
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int l = 0; l < NL; ++l)
        hipLaunchKernelGGL((attn_partial_kernel<__half, HD, G, WAVES, LATE_V>), dim3(blocks), dim3(64 * WAVES), 0, s,
                           args(l, nullptr));
    CK(hipStreamSynchronize(s));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    for (int l = 0; l < NL; ++l)
        hipLaunchKernelGGL((attn_partial_kernel<__half, HD, G, WAVES, LATE_V>), dim3(blocks), dim3(64 * WAVES), 0, s,
                           args(l, nullptr));
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
    const double us = 1000.0 * ms / (reps * NL);
    const double bytes = 2.0 * nkv * (pos + 1.0) * HD * 2;
    // stamps of one launch
    CK(hipMemset(st, 0, sizeof(unsigned long long) * 4 * blocks));
    hipLaunchKernelGGL((attn_partial_kernel<__half, HD, G, WAVES, LATE_V>), dim3(blocks), dim3(64 * WAVES), 0, s, args(1, st));
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(4 * blocks);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, tend = 0;
    double c_sum = 0, p_sum = 0, m_sum = 0, ent = 0;
    int nm = 0;
    for (int i = 0; i < blocks; ++i) t0 = std::min(t0, h[4 * i]);
    for (int i = 0; i < blocks; ++i) {
        ent = std::max(ent, (double)(h[4 * i] - t0));
        c_sum += h[4 * i + 1] - h[4 * i];
        p_sum += h[4 * i + 2] - h[4 * i + 1];
        if (h[4 * i + 3]) {
            m_sum += h[4 * i + 3] - h[4 * i + 2];
            ++nm;
        }
        tend = std::max(tend, std::max(h[4 * i + 2], h[4 * i + 3]));
    }
    printf("%-5s G=%d WAVES=%2d%s blocks=%5d  %7.2f us  %6.0f GB/s | entry spread %.2f, load+compute %.2f, "
           "merge+publish %.2f, last-arriver merge %.2f (%d), span %.2f us\n",
           name, G, WAVES, LATE_V ? " lateV" : "", blocks, us, bytes / (us * 1e3), ent / 100, c_sum / blocks / 100, p_sum / blocks / 100,
           nm ? m_sum / nm / 100 : 0.0, nm, (tend - t0) / 100.0);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(s));
    for (int l = 0; l < NL; ++l) {
        CK(hipFree(K[l]));
        CK(hipFree(V[l]));
    }
    CK(hipFree(q));
    CK(hipFree(out));
    CK(hipFree(part));
    CK(hipFree(cnt));
    CK(hipFree(st));
}

int main() {
    run<1, 16>("C1", 32, 2048, 2047, 8);
    run<1, 8>("C1", 32, 2048, 2047, 8);
    run<1, 4>("C1", 32, 2048, 2047, 8);
    run<4, 4>("C4", 64, 4096, 4095, 3);
    run<4, 8>("C4", 64, 4096, 4095, 3);
    run<4, 16>("C4", 64, 4096, 4095, 3);
    run<4, 4, true>("C4", 64, 4096, 4095, 3);
    run<4, 8, true>("C4", 64, 4096, 4095, 3);
    run<1, 16, true>("C1", 32, 2048, 2047, 8);
    run<1, 4, true>("C1", 32, 2048, 2047, 8);
    return 0;
}
