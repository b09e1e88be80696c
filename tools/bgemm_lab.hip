// bgemm_lab.hip — diagnostic: the batched MFMA projection (csrc/bgemm.h) on the C4 shapes at chosen
// (tiles per workgroup, k-splits) and with / without the fused RMSNorm prologue, each timed over NL
// distinct weight copies inside a replayed hipGraph (no Infinity-Cache re-reads). Prints us per launch
// and GB/s of algorithmic weight bytes.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/bgemm_lab.hip -o tools/bgemm_lab
//   tools/bgemm_lab [batch]          (LAB_TILED=1: the weights in the fragment layout, BgIn::tiled)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../simplellminference_amd/csrc/bgemm.h"

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
        p[i] = __float2half(((float)(h & 0xFFFF) / 65536.0f - 0.5f) * 0.03f);
    }
}
__global__ void fill_f(float* p, size_t n, unsigned seed, float off) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2246822519u ^ seed;
        h ^= h >> 13;
        h *= 2654435761u;
        h ^= h >> 16;
        p[i] = off + (float)(h & 0xFFFF) / 65536.0f - 0.5f;
    }
}


// LAB_U=n: the kernel at a forced step width n (16-byte loads per lane per step) instead of bg_step_width's
template <bool NORM, int U>
static hipError_t launch_u(const __half* W, const BgIn& in_, const BgEpiStore& e, const BgPlan& p, hipStream_t s) {
    static const hipError_t a = hipFuncSetAttribute(reinterpret_cast<const void*>(&bgemm_kernel<BgEpiStore, NORM, U>),
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, kBgLdsMax);
    if (a != hipSuccess) return a;
    BgIn in = in_;
    in.ntiles = p.ntiles;
    in.tpw = p.tpw;
    in.splits = p.splits;
    hipLaunchKernelGGL((bgemm_kernel<BgEpiStore, NORM, U>), dim3(p.groups * p.splits), dim3(kBgThreads), p.lds, s, W, in, e);
    return hipGetLastError();
}
static hipError_t lab_launch(const __half* W, const BgIn& in, const BgEpiStore& e, const BgPlan& p, hipStream_t s) {
    const int u = getenv("LAB_U") ? atoi(getenv("LAB_U")) : 0;
    const bool nrm = in.norm_w != nullptr;
    if (u == 8) return nrm ? launch_u<true, 8>(W, in, e, p, s) : launch_u<false, 8>(W, in, e, p, s);
    if (u == 6) return nrm ? launch_u<true, 6>(W, in, e, p, s) : launch_u<false, 6>(W, in, e, p, s);
    if (u == 4) return nrm ? launch_u<true, 4>(W, in, e, p, s) : launch_u<false, 4>(W, in, e, p, s);
    if (u == 2) return nrm ? launch_u<true, 2>(W, in, e, p, s) : launch_u<false, 2>(W, in, e, p, s);
    return launch_bgemm(W, in, e, p, s);
}

static double time_cfg(const std::vector<__half*>& Ws, int rows, int K, int B, bool norm, BgPlan p, float* x,
                       float* nw, float* y, float* ws, unsigned* cnt, int reps) {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    BgIn in{x, norm ? nw : nullptr, 1e-5f, K, B, 0, 0, 0, ws, cnt};
    in.tiled = getenv("LAB_TILED") ? 1 : 0;
    BgEpiStore e{y, nullptr, nullptr, 1.0f, rows, rows};
    CK((bg_allow_lds<BgEpiStore, true>()));
    CK((bg_allow_lds<BgEpiStore, false>()));
    for (auto* W : Ws) CK(lab_launch(W, in, e, p, s));  // warm-up
    CK(hipStreamSynchronize(s));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    for (auto* W : Ws) CK(lab_launch(W, in, e, p, s));
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(s));
    return 1000.0 * ms / (reps * (double)Ws.size());
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 8;
    struct Shape { const char* name; int rows, K; bool norm; };
    const Shape shapes[] = {{"qkv", 6144, 4096, true}, {"wo", 4096, 4096, false}, {"gu", 28672, 4096, true},
                            {"down", 4096, 14336, false}, {"tp8-qkv", 768, 4096, true}, {"tp8-down", 4096, 1792, false}};
    const int NL = 8, reps = 10;
    float *x, *nw, *y, *ws;
    unsigned* cnt;
    CK(hipMalloc(&x, sizeof(float) * 8 * 16384));
    CK(hipMalloc(&nw, sizeof(float) * 16384));
    CK(hipMalloc(&y, sizeof(float) * 8 * 32768));
    CK(hipMalloc(&ws, 64 << 20));
    CK(hipMalloc(&cnt, 1 << 16));
    CK(hipMemset(cnt, 0, 1 << 16));
    fill_f<<<256, 256>>>(x, 8 * 16384, 3, 0.0f);
    fill_f<<<256, 256>>>(nw, 16384, 5, 1.0f);
    for (const Shape& sh : shapes) {
        if (getenv("LAB_SHAPE") && std::string(getenv("LAB_SHAPE")) != sh.name) continue;
        std::vector<__half*> Ws(NL);
        const size_t n = (size_t)((sh.rows + 15) / 16) * 16 * sh.K;  // whole tiles (the fragment layout's size)
        for (int l = 0; l < NL; ++l) {
            CK(hipMalloc(&Ws[l], n * 2));
            fill_h<<<1024, 256>>>(Ws[l], n, 11 + l);
        }
        CK(hipDeviceSynchronize());
        const int tiles = (sh.rows + 15) / 16;
        const double gb = n * 2.0 / 1e9;
        BgPlan auto_p = bg_plan(tiles, sh.K, B, sh.norm);
        std::vector<BgPlan> cands = {auto_p};

        const bool auto_only = getenv("LAB_AUTO_ONLY") != nullptr;
        const int tpws[] = {1, 2, 3, 4, 6, 8, 12, 16, 24, 32};
        const int sps[] = {1, 2, 4, 8};
        for (int sp : sps)
            for (int tpw : tpws) {
                if (auto_only) break;  // fused-RMS plans run on one split: their split forms are timed without the norm
                const int nkb = sh.K / 32;
                if (sp > 1 && nkb / sp < kBgWaves) continue;
                const int kbs = (nkb + sp - 1) / sp;
                if (kbs * 32 > kBgMaxStageK) continue;
                if (bg_lds_bytes(sh.K, sp, tpw) > (size_t)kBgLdsMax) continue;
                BgPlan p;
                p.ntiles = tiles;
                p.tpw = tpw;
                p.splits = sp;
                p.groups = (tiles + tpw - 1) / tpw;
                p.lds = bg_lds_bytes(sh.K, sp, tpw);
                if (p.groups * sp > 1024 || p.groups * sp < 64) continue;
                cands.push_back(p);
            }
        for (size_t c = 0; c < cands.size(); ++c) {
            const BgPlan& p = cands[c];
            const bool nrm = sh.norm && p.splits == 1;
            const double us = time_cfg(Ws, sh.rows, sh.K, B, nrm, p, x, nw, y, ws, cnt, reps);
            double us_nn = nrm ? time_cfg(Ws, sh.rows, sh.K, B, false, p, x, nw, y, ws, cnt, reps) : us;
            printf("%-8s B=%d %s tpw=%2d splits=%d wgs=%4d  %7.2f us  %6.0f GB/s   (no-norm %7.2f us)\n", sh.name, B,
                   c == 0 ? "AUTO" : "    ", p.tpw, p.splits, p.groups * p.splits, us, gb / (us * 1e-6), us_nn);
            fflush(stdout);
        }
        for (size_t ci = 0; ci < 1; ++ci) {  // per-workgroup phase stamps (s_memrealtime, 100 MHz) of the AUTO plan
            unsigned long long* st;
            const BgPlan& p = cands[ci];
            const int nwg = p.groups * p.splits;
            CK(hipMalloc(&st, sizeof(unsigned long long) * 4 * nwg));
            CK(hipMemset(st, 0, sizeof(unsigned long long) * 4 * nwg));
            BgIn in{x, sh.norm ? nw : nullptr, 1e-5f, sh.K, B, 0, 0, 0, ws, cnt, st};
            in.tiled = getenv("LAB_TILED") ? 1 : 0;
            BgEpiStore e{y, nullptr, nullptr, 1.0f, sh.rows, sh.rows};
            CK(lab_launch(Ws[0], in, e, p, 0));
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> h(4 * nwg);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull, tmax = 0;
            double st_sum = 0, str_sum = 0, ep_sum = 0, ent_max = 0;
            for (int i = 0; i < nwg; ++i) t0 = std::min(t0, h[4 * i]);
            for (int i = 0; i < nwg; ++i) {
                ent_max = std::max(ent_max, (double)(h[4 * i] - t0));
                st_sum += h[4 * i + 1] - h[4 * i];
                str_sum += h[4 * i + 2] - h[4 * i + 1];
                if (h[4 * i + 3]) ep_sum += h[4 * i + 3] - h[4 * i + 2];
                tmax = std::max(tmax, std::max(h[4 * i + 2], h[4 * i + 3]));
            }
            printf("   %s stamps: entry spread %.2f us, staging avg %.2f us, stream avg %.2f us, epilogue avg %.2f us, "
                   "first entry -> last end %.2f us\n", "AUTO", ent_max / 100.0, st_sum / nwg / 100.0, str_sum / nwg / 100.0,
                   ep_sum / nwg / 100.0, (tmax - t0) / 100.0);
            std::vector<double> send, eend;  // per workgroup: stream end, epilogue end (us after the first entry)
            for (int i = 0; i < nwg; ++i) {
                send.push_back((h[4 * i + 2] - t0) / 100.0);
                if (h[4 * i + 3]) eend.push_back((h[4 * i + 3] - t0) / 100.0);
            }
            std::sort(send.begin(), send.end());
            std::sort(eend.begin(), eend.end());
            auto pc = [](const std::vector<double>& v, double f) { return v.empty() ? 0.0 : v[(size_t)(f * (v.size() - 1))]; };
            printf("   stream end p10 %.2f p50 %.2f p90 %.2f max %.2f | epilogue end (%zu wg) p50 %.2f max %.2f us\n",
                   pc(send, .1), pc(send, .5), pc(send, .9), pc(send, 1.0), eend.size(), pc(eend, .5), pc(eend, 1.0));
            CK(hipFree(st));
        }
        for (auto* W : Ws) CK(hipFree(W));
    }
    return 0;
}
