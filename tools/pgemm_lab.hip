// pgemm_lab — tiling / ring-depth sweep of the prefill GEMM (csrc/prefill.h pgemm_kernel) on the Llama-2-7B
// projection shapes at a 256-row chunk: device time per launch (HIP events, 20 launches), issued MFMA
// TFLOP/s (hi + lo: 4 N K M), and a spot check of 64 outputs against a host fp64 sum.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I simplellminference_amd/csrc tools/pgemm_lab.hip -o tools/pgemm_lab
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "prefill.h"

using namespace sli;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

static uint32_t rng(uint64_t& s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(s >> 33);
}

struct Shape {
    const char* name;
    int N, K;
};

template <typename WT>
struct Bufs {
    WT* W;
    std::vector<WT*> Wc;  // the timing loop rotates over copies (none MALL-resident: weights stream from HBM as in
                          // the engine, where a layer's weights are read once per chunk)
    __half *hi, *lo;
    float* y;
    PfState* ps;
    std::vector<WT> hW;
    std::vector<__half> hhi, hlo;
};

static float h2f(__half h) { return __half2float(h); }

template <typename WT>
static void make(Bufs<WT>& b, int N, int K, int M) {
    uint64_t s = 12345 + N + K;
    b.hW.resize((size_t)N * K);
    for (auto& w : b.hW) {
        if constexpr (sizeof(WT) == 1)
            w = (int8_t)((int)(rng(s) % 255) - 127);
        else
            w = __float2half(((int)(rng(s) % 2001) - 1000) * 1e-3f * 0.05f);
    }
    b.hhi.resize((size_t)M * K);
    b.hlo.resize((size_t)M * K);
    for (size_t i = 0; i < b.hhi.size(); ++i) {
        const float v = ((int)(rng(s) % 200001) - 100000) * 1e-5f;
        b.hhi[i] = __float2half(v);
        b.hlo[i] = __float2half(v - __half2float(b.hhi[i]));
    }
    CK(hipMalloc(&b.W, sizeof(WT) * b.hW.size()));
    CK(hipMalloc(&b.hi, 2 * b.hhi.size()));
    CK(hipMalloc(&b.lo, 2 * b.hlo.size()));
    CK(hipMalloc(&b.y, sizeof(float) * (size_t)M * N));
    CK(hipMalloc(&b.ps, sizeof(PfState)));
    CK(hipMemcpy(b.W, b.hW.data(), sizeof(WT) * b.hW.size(), hipMemcpyHostToDevice));
    const int ncopy = getenv("LAB_HOT") ? 1 : 4;
    b.Wc.assign(1, b.W);
    for (int c = 1; c < ncopy; ++c) {
        WT* p;
        CK(hipMalloc(&p, sizeof(WT) * b.hW.size()));
        CK(hipMemcpy(p, b.W, sizeof(WT) * b.hW.size(), hipMemcpyDeviceToDevice));
        b.Wc.push_back(p);
    }
    CK(hipMemcpy(b.hi, b.hhi.data(), 2 * b.hhi.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(b.lo, b.hlo.data(), 2 * b.hlo.size(), hipMemcpyHostToDevice));
    PfState p{0, M};
    CK(hipMemcpy(b.ps, &p, sizeof p, hipMemcpyHostToDevice));
}

template <typename WT>
static void release(Bufs<WT>& b) {
    for (auto* p : b.Wc) CK(hipFree(p));
    CK(hipFree(b.hi));
    CK(hipFree(b.lo));
    CK(hipFree(b.y));
    CK(hipFree(b.ps));
}

template <class Cfg, typename WT>
static void run(const char* tag, Bufs<WT>& b, const Shape& sh, int M) {
    using Geo = PgGeo<Cfg, WT>;
    CK((pgemm_allow_lds<PgEpiResid, Cfg, WT>()));
    PgIn<WT> in{b.W, b.hi, b.lo, sh.N, sh.K, M};
    PgEpiResid e{b.y, nullptr, nullptr, sh.N, sh.N};
    CK(hipMemset(b.y, 0, sizeof(float) * (size_t)M * sh.N));
    CK((launch_pgemm<PgEpiResid, Cfg, WT>(in, e, b.ps, 0)));
    CK(hipDeviceSynchronize());
    // spot check (y[m][row] = sum_k W[row][k] (hi + lo)[m][k])
    std::vector<float> y((size_t)M * sh.N);
    CK(hipMemcpy(y.data(), b.y, sizeof(float) * y.size(), hipMemcpyDeviceToHost));
    double maxrel = 0.0;
    uint64_t s = 777;
    for (int i = 0; i < 64; ++i) {
        const int m = rng(s) % M, row = rng(s) % sh.N;
        double ref = 0.0, mag = 0.0;
        for (int k = 0; k < sh.K; ++k) {
            double w;
            if constexpr (sizeof(WT) == 1)
                w = (double)b.hW[(size_t)row * sh.K + k];
            else
                w = (double)h2f(b.hW[(size_t)row * sh.K + k]);
            const double x = (double)h2f(b.hhi[(size_t)m * sh.K + k]) + (double)h2f(b.hlo[(size_t)m * sh.K + k]);
            ref += w * x;
            mag += fabs(w * x);
        }
        maxrel = fmax(maxrel, fabs(y[(size_t)m * sh.N + row] - ref) / (mag + 1e-30));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) {
        PgIn<WT> ic = in;
        ic.W = b.Wc[i % b.Wc.size()];
        CK((launch_pgemm<PgEpiResid, Cfg, WT>(ic, e, b.ps, 0)));
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / iters;
    const double tf = 4.0 * sh.N * sh.K * (double)M / (us * 1e-6) / 1e12;
    const double wgbs = (double)sh.N * sh.K * sizeof(WT) / (us * 1e-6) / 1e9;
    const int nrb = (sh.N + Geo::BN - 1) / Geo::BN;
    printf("%-5s %-6s %-22s grid %5d lds %6zu  %8.1f us  %6.1f TF issued  W %6.0f GB/s  relerr %.1e\n", sh.name,
           sizeof(WT) == 1 ? "i8" : "f16", tag, nrb * (M / Geo::BM), Geo::LDS, us, tf, wgbs, maxrel);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

#define RUN(BM, WR, S) run<PgCfg<BM, WR, S>, WT>("BM" #BM " WR" #WR " S" #S, b, sh, M)
#define RUNP(BM, WR, S, AT) run<PgCfg<BM, WR, S, AT, true>, WT>("BM" #BM " WR" #WR " S" #S " AT" #AT " pipe", b, sh, M)
#define RUNA(BM, WR, AT, SA) \
    run<PgCfg<BM, WR, 2, AT, true, SA>, WT>("BM" #BM " WR" #WR " AT" #AT " pipe SA" #SA, b, sh, M)

template <typename WT>
static void sweep(const Shape& sh, int M) {
    Bufs<WT> b;
    make(b, sh.N, sh.K, M);
    if (getenv("LAB_QUICK")) {  // the engine's fp16 tilings at M = 256 (prefill.h pg_pick)
        if constexpr (sizeof(WT) == 2) {
            RUNA(128, 4, 2, 4);
            RUNP(64, 4, 3, 2);
            RUNP(64, 2, 3, 2);
        }
        release(b);
        return;
    }
    if constexpr (sizeof(WT) == 2) {
        RUN(128, 2, 2);
        RUN(128, 2, 3);
        RUN(128, 2, 4);
        RUN(64, 2, 3);
        RUN(64, 2, 4);
        RUN(64, 2, 6);
        RUN(64, 4, 3);
        RUN(64, 4, 4);
        RUN(128, 4, 2);
        RUN(128, 4, 3);
        RUN(256, 2, 2);
        RUN(256, 4, 2);
        RUN(32, 2, 4);
        RUN(32, 2, 8);
    } else {
        RUN(64, 2, 2);
        RUN(64, 2, 3);
        RUN(128, 2, 2);
        RUN(64, 4, 2);
        RUN(64, 4, 3);
        RUN(128, 4, 2);
        RUN(32, 2, 4);
    }
    release(b);
}

int main(int argc, char** argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 256;
    const Shape shapes[] = {{"qkv", 12288, 4096}, {"gu", 22016, 4096}, {"wo", 4096, 4096}, {"down", 4096, 11008}};
    for (const Shape& sh : shapes) sweep<__half>(sh, M);
    for (const Shape& sh : shapes) sweep<int8_t>(sh, M);
    return 0;
}
