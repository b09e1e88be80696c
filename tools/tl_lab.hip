// tl_lab.hip — the persistent layer stack (csrc/tp_layers.h) alone on one GPU, at a C2 TP-8 rank's shapes
// (Llama-2-7B / 8: D 4096, 4 q and 4 kv heads of 128, FFN 1376, 32 layers, ctx 2048 at position 2047), with
// per-phase stamps (built with TL_STAMPS). Weights / cache are hashed noise: timing only (the engine's tests hold the
// arithmetic to the oracle, tests/test_gpu_tp_layers.py).
//
//   tl_lab [-m 0|1|2] [-L layers] [-r reps] [-n ranks] [-w workgroups]
//     -x 0|1|2: the loopback exchange buffer uncached (the engine's) / plain / fine-grained
//     -m 0: one rank (x += projection), 1: no-comm debug (the local partial), 2: the granule exchange in loopback
//           (every slot of the rank's own uncached buffer, as SLI_DEBUG_OS_LOOPBACK), -n ranks (default 8)
// Prints the launch time per layer and the median per-phase spans (us) of a few workgroups.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../simplellminference_amd/csrc/tp_layers.h"

using namespace sli;

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);                  \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ void fill_half(__half* p, size_t n, unsigned seed, float scale) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        h ^= h >> 15;
        p[i] = __float2half(((float)(h & 0xffff) / 65535.0f - 0.5f) * scale);
    }
}
__global__ void fill_float(float* p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

int main(int argc, char** argv) {
    int mode = 1, L = 32, reps = 20, nranks = 8, nwg = 0, xmem = 0;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "-m")) mode = atoi(argv[i + 1]);
        if (!strcmp(argv[i], "-L")) L = atoi(argv[i + 1]);
        if (!strcmp(argv[i], "-r")) reps = atoi(argv[i + 1]);
        if (!strcmp(argv[i], "-n")) nranks = atoi(argv[i + 1]);
        if (!strcmp(argv[i], "-w")) nwg = atoi(argv[i + 1]);
        if (!strcmp(argv[i], "-x")) xmem = atoi(argv[i + 1]);
    }
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    if (!nwg) nwg = prop.multiProcessorCount;
    const int D = 4096, hq = 4, hkv = 4, Il = 1376, T = 2048, pos = 2047, HD = kTlHD;
    const int S = (T + kTlKS - 1) / kTlKS;
    auto dalloc = [](size_t n) {
        void* p;
        CK(hipMalloc(&p, n));
        CK(hipMemset(p, 0, n));
        return p;
    };
    const size_t nq = (size_t)(hq + 2 * hkv) * HD * D, no = (size_t)D * hq * HD, ng = 2ull * Il * D, nd = (size_t)D * Il;
    std::vector<const __half*> wt(4 * (size_t)L);
    for (int l = 0; l < L; ++l) {
        const size_t n[4] = {nq, no, ng, nd};
        for (int k = 0; k < 4; ++k) {
            __half* p = (__half*)dalloc(2 * n[k]);
            hipLaunchKernelGGL(fill_half, dim3(1024), dim3(256), 0, 0, p, n[k], 17u * l + k, 0.05f);
            wt[4 * l + k] = p;
        }
    }
    const __half** wd = (const __half**)dalloc(sizeof(void*) * wt.size());
    CK(hipMemcpy(wd, wt.data(), sizeof(void*) * wt.size(), hipMemcpyHostToDevice));
    float* norms = (float*)dalloc(4ull * (2 * L + 1) * D);
    hipLaunchKernelGGL(fill_float, dim3(256), dim3(256), 0, 0, norms, (size_t)(2 * L + 1) * D, 1.0f);
    const size_t nkv = (size_t)L * hkv * T * HD;
    __half* kc = (__half*)dalloc(2 * nkv);
    __half* vc = (__half*)dalloc(2 * nkv);
    hipLaunchKernelGGL(fill_half, dim3(1024), dim3(256), 0, 0, kc, nkv, 7u, 2.0f);
    hipLaunchKernelGGL(fill_half, dim3(1024), dim3(256), 0, 0, vc, nkv, 8u, 2.0f);
    float* sn = (float*)dalloc(4ull * T * HD / 2);
    float* cs = (float*)dalloc(4ull * T * HD / 2);
    hipLaunchKernelGGL(fill_float, dim3(256), dim3(256), 0, 0, sn, (size_t)T * HD / 2, 0.6f);
    hipLaunchKernelGGL(fill_float, dim3(256), dim3(256), 0, 0, cs, (size_t)T * HD / 2, 0.8f);
    DevState hs{};
    hs.pos = pos;
    DevState* st = (DevState*)dalloc(sizeof(DevState));
    CK(hipMemcpy(st, &hs, sizeof(hs), hipMemcpyHostToDevice));
    float* x = (float*)dalloc(4ull * D);
    hipLaunchKernelGGL(fill_float, dim3(16), dim3(256), 0, 0, x, (size_t)D, 0.5f);

    TlArgs a{};
    a.D = D, a.hq = hq, a.hkv = hkv, a.Il = Il, a.L = L, a.T = T, a.nwg = nwg, a.act_mode = 0;
    a.eps = 1e-5f, a.scale = 1.0f / sqrtf((float)HD);
    a.w = wd, a.norms = norms, a.kc = kc, a.vc = vc, a.sin_t = sn, a.cos_t = cs, a.st = st, a.x = x;
    a.g_x = (tl_u2*)dalloc(8ull * D);
    a.g_qkv = (tl_u2*)dalloc(8ull * (hq + 2 * hkv) * HD);
    a.g_part = (tl_u2*)dalloc(8ull * hq * S * kTlPart);
    a.g_att = (tl_u2*)dalloc(8ull * hq * HD);
    a.g_x1 = (tl_u2*)dalloc(8ull * D);
    a.g_act = (tl_u2*)dalloc(8ull * Il);
    a.epoch = (unsigned*)dalloc(16);
    a.mode = mode, a.rank = nranks - 1, a.nranks = mode == 2 ? nranks : 1, a.loopback = 1;
    if (mode == 2) {
        tl_u2* buf;
        // -x 0: uncached (what the engine maps over IPC), 1: plain device memory, 2: fine-grained
        if (xmem == 1)
            CK(hipMalloc((void**)&buf, 8ull * 2 * 8 * D));
        else
            CK(hipExtMallocWithFlags((void**)&buf, 8ull * 2 * 8 * D,
                                     xmem == 2 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
        CK(hipMemset(buf, 0, 8ull * 2 * 8 * D));
        std::vector<tl_u2*> xg(nranks, buf);
        tl_u2** xgd = (tl_u2**)dalloc(sizeof(void*) * nranks);
        CK(hipMemcpy(xgd, xg.data(), sizeof(void*) * nranks, hipMemcpyHostToDevice));
        a.xg = xgd;
    }
    a.stamps = (unsigned long long*)dalloc(8ull * nwg * L * kTlStamps);
    CK(hipDeviceSynchronize());

    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms(reps);
    for (int r = 0; r <= reps; ++r) {
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(tp_layers_kernel<1>, dim3(nwg), dim3(kTlThreads), 0, s, a);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        if (r > 0) CK(hipEventElapsedTime(&ms[r - 1], e0, e1));
    }
    CK(hipMemcpy(&hs, st, sizeof(hs), hipMemcpyDeviceToHost));
    std::sort(ms.begin(), ms.end());
    printf("tl_lab -x %d mode %d%s, %d layers, %d workgroups: median launch %.1f us = %.2f us per layer (device error %d)\n",
           xmem, mode, mode == 2 ? " (loopback exchange)" : "", L, nwg, ms[reps / 2] * 1e3, ms[reps / 2] * 1e3 / L, hs.error);
#ifdef TL_STAMPS
    std::vector<unsigned long long> h(8ull * nwg * L * kTlStamps / 8);
    CK(hipMemcpy(h.data(), a.stamps, 8ull * nwg * L * kTlStamps, hipMemcpyDeviceToHost));
    const char* names[kTlStamps] = {"E1 x", "qkv", "attn", "E3 att", "wo", "xch+E4", "gu", "E5 act", "down", "xch"};
    auto med = [&](int wg, int k0, int k1) {  // median over layers 1.. of stamp k1 - stamp k0
        std::vector<double> v;
        for (int l = 1; l < L; ++l) {
            const unsigned long long* q = &h[((size_t)wg * L + l) * kTlStamps];
            if (q[k0] && q[k1]) v.push_back((double)(q[k1] - q[k0]) / 100.0);
        }
        std::sort(v.begin(), v.end());
        return v.empty() ? -1.0 : v[v.size() / 2];
    };
    for (int wg : {0, 1, 15, 16, 100, 200, nwg - 1}) {
        if (wg >= nwg) continue;
        printf("  wg %3d: [norm %.2f gemv %.2f epi %.2f] [E2 %.2f attend %.2f (scores %.2f max %.2f pv %.2f publish %.2f) "
               "merge-gather %.2f merge %.2f]\n", wg,
               med(wg, 0, 14), med(wg, 14, 15), med(wg, 15, 1), med(wg, 1, 10), med(wg, 10, 11), med(wg, 10, 16),
               med(wg, 16, 17), med(wg, 17, 18), med(wg, 18, 11), med(wg, 11, 12), med(wg, 12, 2));
        printf("  wg %3d:", wg);
        for (int k = 0; k < 10; ++k) {
            std::vector<double> v;
            for (int l = 1; l < L; ++l) {
                const unsigned long long* q = &h[((size_t)wg * L + l) * kTlStamps];
                const unsigned long long* qp = &h[((size_t)wg * L + l - 1) * kTlStamps];
                const unsigned long long b = k == 0 ? qp[9] : q[k - 1];
                v.push_back((double)(q[k] - b) / 100.0);
            }
            std::sort(v.begin(), v.end());
            printf(" %s %.2f |", names[k], v[v.size() / 2]);
        }
        printf("\n");
    }
#endif
    return hs.error ? 2 : 0;
}
