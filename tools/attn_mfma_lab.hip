// attn_mfma_lab.hip — diagnostic: the MFMA decode attention (csrc/attn_mfma.h) against the register-staged
// kernel (csrc/attention.h) on the decode shapes: merged outputs compared (both with the in-launch last-arriver
// merge), then each timed over NL distinct K/V caches inside a replayed hipGraph in the merge placement the
// engine uses (register kernel: C1 deferred to wo = partials only, C4 partials + attn_merge_kernel; MFMA
// kernel: partials only at C1, in-launch merge elsewhere), with per-workgroup phase stamps of the MFMA kernel.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/attn_mfma_lab.hip -o tools/attn_mfma_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "../simplellminference_amd/csrc/attn_mfma.h"

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
__global__ void fill_f(float* p, size_t n, unsigned seed, float amp) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2246822519u ^ seed;
        h ^= h >> 13;
        h *= 2654435761u;
        h ^= h >> 16;
        p[i] = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * amp;
    }
}

static int cus() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    return p.multiProcessorCount;
}

template <int HD, int G>
static void launch_mfma(const AttnArgs<__half>& a, int blocks, int nbuf, hipStream_t s) {
    if (nbuf == 1)
        hipLaunchKernelGGL((attn_mfma_kernel<HD, G, 1>), dim3(blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((attn_mfma_kernel<HD, G, 2>), dim3(blocks), dim3(256), 0, s, a);
}

// nkv: kv heads over all sequences (seq_heads per sequence), positions per sequence in pos[]
template <int HD, int G>
static void run(const char* name, int nkv, int seq_heads, int T, std::vector<int> pos, int NL, int defer_ref,
                int defer_mfma, int tpw_force = 0) {
    using Geo = AttnGeom<__half, HD>;
    const int nseq = nkv / seq_heads;
    const int splits_r = (T + Geo::PPWG - 1) / Geo::PPWG;
    const int tpw = tpw_force ? tpw_force : attn_mfma_tpw(nkv, T, cus());
    const int ppwg = kAmWgKeys * tpw, splits_m = (T + ppwg - 1) / ppwg;
    const int nbuf = tpw > 1 ? 2 : 1;
    const size_t per = (size_t)nkv * T * HD;
    std::vector<__half*> K(NL), V(NL);
    for (int l = 0; l < NL; ++l) {
        CK(hipMalloc(&K[l], per * 2));
        CK(hipMalloc(&V[l], per * 2));
        fill_h<<<1024, 256>>>(K[l], per, 3 + l);
        fill_h<<<1024, 256>>>(V[l], per, 7 + l);
    }
    const int H = nkv * G;
    float *q, *out_r, *out_m, *part_r, *part_m;
    unsigned *cnt_r, *cnt_m;
    int32_t* posd;
    unsigned long long* st;
    CK(hipMalloc(&q, sizeof(float) * H * HD));
    CK(hipMalloc(&out_r, sizeof(float) * H * HD));
    CK(hipMalloc(&out_m, sizeof(float) * H * HD));
    CK(hipMalloc(&part_r, sizeof(float) * (size_t)H * splits_r * (HD + kAttnPartPad)));
    CK(hipMalloc(&part_m, sizeof(float) * (size_t)H * splits_m * (HD + kAttnPartPad)));
    CK(hipMalloc(&cnt_r, sizeof(unsigned) * nkv));
    CK(hipMalloc(&cnt_m, sizeof(unsigned) * nkv));
    CK(hipMemset(cnt_r, 0, sizeof(unsigned) * nkv));
    CK(hipMemset(cnt_m, 0, sizeof(unsigned) * nkv));
    CK(hipMalloc(&posd, sizeof(int32_t) * nseq * 16));
    std::vector<int32_t> hp(nseq * 16, 0);
    for (int b = 0; b < nseq; ++b) hp[b * 16] = pos[b % pos.size()];
    CK(hipMemcpy(posd, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    fill_f<<<64, 256>>>(q, (size_t)H * HD, 11, 2.0f);
    const int blocks_r = nkv * splits_r, blocks_m = nkv * splits_m;
    CK(hipMalloc(&st, sizeof(unsigned long long) * 4 * blocks_m));
    CK(hipDeviceSynchronize());
    auto args = [&](int l, bool mf, int defer, unsigned long long* stamps) {
        AttnArgs<__half> a{q,   K[l], V[l], HD, (long long)T * HD, mf ? part_m : part_r, mf ? out_m : out_r,
                           mf ? cnt_m : cnt_r, posd, 0, nkv, mf ? splits_m : splits_r, 1.0f / sqrtf((float)HD),
                           seq_heads, 16, stamps};
        a.defer_merge = defer;
        if (mf) a.ppwg = ppwg;
        return a;
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // correctness: both with the in-launch merge
    hipLaunchKernelGGL((attn_partial_kernel<__half, HD, G>), dim3(blocks_r), dim3(64 * attn_waves(G)), 0, s,
                       args(0, false, 0, nullptr));
    launch_mfma<HD, G>(args(0, true, 0, nullptr), blocks_m, nbuf, s);
    CK(hipStreamSynchronize(s));
    std::vector<float> hr((size_t)H * HD), hm((size_t)H * HD);
    CK(hipMemcpy(hr.data(), out_r, hr.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hm.data(), out_m, hm.size() * 4, hipMemcpyDeviceToHost));
    double md = 0, mo = 0;
    for (size_t i = 0; i < hr.size(); ++i) {
        md = std::max(md, (double)std::fabs(hr[i] - hm[i]));
        mo = std::max(mo, (double)std::fabs(hr[i]));
    }
    // timing: NL layers per graph
    auto time_it = [&](bool mf) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        for (int l = 0; l < NL; ++l) {
            if (mf) {
                launch_mfma<HD, G>(args(l, true, defer_mfma, nullptr), blocks_m, nbuf, s);
                if (defer_mfma == 2)
                    hipLaunchKernelGGL((attn_merge_kernel<__half, HD, G>), dim3(nkv * attn_merge_wgs(G * HD)),
                                       dim3(kAttnMergeThreads), 0, s, args(l, true, 2, nullptr));
            } else {
                hipLaunchKernelGGL((attn_partial_kernel<__half, HD, G>), dim3(blocks_r), dim3(64 * attn_waves(G)), 0,
                                   s, args(l, false, defer_ref, nullptr));
                if (defer_ref == 2)
                    hipLaunchKernelGGL((attn_merge_kernel<__half, HD, G>), dim3(nkv * attn_merge_wgs(G * HD)),
                                       dim3(kAttnMergeThreads), 0, s, args(l, false, 2, nullptr));
            }
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int reps = 20;
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
    const double ur = time_it(false), um = time_it(true);
    double bytes = 0;
    for (int b = 0; b < nseq; ++b) bytes += 2.0 * seq_heads * (hp[b * 16] + 1.0) * HD * 2;
    // stamps of one MFMA launch
    CK(hipMemset(st, 0, sizeof(unsigned long long) * 4 * blocks_m));
    launch_mfma<HD, G>(args(NL > 1 ? 1 : 0, true, defer_mfma == 2 ? 0 : defer_mfma, st), blocks_m, nbuf, s);
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(4 * blocks_m);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, tend = 0;
    double ent = 0, q_sum = 0, loop_sum = 0, m_sum = 0;
    int n = 0, nm = 0;
    for (int i = 0; i < blocks_m; ++i)
        if (h[4 * i]) t0 = std::min(t0, h[4 * i]);
    for (int i = 0; i < blocks_m; ++i) {
        if (!h[4 * i] || !h[4 * i + 2]) continue;
        ++n;
        ent = std::max(ent, (double)(h[4 * i] - t0));
        q_sum += h[4 * i + 1] - h[4 * i];
        loop_sum += h[4 * i + 2] - h[4 * i + 1];
        if (h[4 * i + 3]) {
            m_sum += h[4 * i + 3] - h[4 * i + 2];
            ++nm;
        }
        tend = std::max(tend, std::max(h[4 * i + 2], h[4 * i + 3]));
    }
    printf("%-8s G=%d HD=%d nkv=%3d T=%5d pos0=%5d | max|d| %.2e (max|o| %.2e) | register %7.2f us %6.0f GB/s "
           "(%d wg) | mfma tpw %2d %7.2f us %6.0f GB/s (%d wg) x%.3f | stamps: entry spread %.2f, q staged %.2f, "
           "loop %.2f, last merge %.2f (%d), span %.2f us\n",
           name, G, HD, nkv, T, pos[0], md, mo, ur, bytes / (ur * 1e3), blocks_r, tpw, um, bytes / (um * 1e3),
           blocks_m, ur / um, ent / 100, n ? q_sum / n / 100 : 0.0, n ? loop_sum / n / 100 : 0.0,
           nm ? m_sum / nm / 100 : 0.0, nm, (tend - t0) / 100.0);
    fflush(stdout);
    if (!(md <= 2e-5 * std::max(1.0, mo))) printf("MISMATCH %s\n", name);
    CK(hipStreamDestroy(s));
    for (int l = 0; l < NL; ++l) {
        CK(hipFree(K[l]));
        CK(hipFree(V[l]));
    }
    CK(hipFree(q));
    CK(hipFree(out_r));
    CK(hipFree(out_m));
    CK(hipFree(part_r));
    CK(hipFree(part_m));
    CK(hipFree(cnt_r));
    CK(hipFree(cnt_m));
    CK(hipFree(posd));
    CK(hipFree(st));
}


// K/V warm-up by plain (default-policy, Infinity-Cache allocating) loads: attention workgroup aw (kv head aw / splits,
// split aw % splits) gets its first nk keys' K and V rows read; one prefetch workgroup covers per_wg of them
template <int HD>
__global__ void __launch_bounds__(1024) kv_prefetch_kernel(const __half* K, const __half* V, int T, int splits, int ppwg,
                                                           int nk, int per_wg, int n_aw, float* sink) {
    float acc = 0.0f;
    const int chunks = nk * HD * 2 / 16;  // 16-byte chunks of one head's nk rows
    for (int a = 0; a < per_wg; ++a) {
        const int aw = blockIdx.x * per_wg + a;
        if (aw >= n_aw) break;
        const int h = aw / splits, sp = aw - h * splits;
        const size_t base = ((size_t)h * T + (size_t)sp * ppwg) * HD * 2;  // bytes
        for (int c = threadIdx.x; c < 2 * chunks; c += blockDim.x) {
            const char* src = reinterpret_cast<const char*>(c < chunks ? K : V) + base + (size_t)(c % chunks) * 16;
            const uint4 v = *reinterpret_cast<const uint4*>(src);
            acc += __uint_as_float(v.x ^ v.w);
        }
    }
    if (acc == 1.2345f) sink[threadIdx.x] = acc;
}
__global__ void __launch_bounds__(1024) nt_stream_kernel(const char* p, long long bytes, float* sink) {
    const long long per = bytes / gridDim.x;
    const char* b = p + per * blockIdx.x;
    const int nvec = (int)(per / 16);
    float acc = 0.0f;
    for (int v = threadIdx.x; v < nvec; v += 8 * 1024) {
        u32x4 w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = load16<true>(b + (size_t)min(v + j * 1024, nvec - 1) * 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += __uint_as_float(w[j].x ^ w[j].w);
    }
    if (acc == 1.2345f) sink[threadIdx.x] = acc;
}

// Does warming the first nk keys of every attention workgroup's split into the Infinity Cache (during the q/k/v
// projection: a 50 MB nt stream stands in for it) shorten the C4 attention? Graph replays of NL layers.
static void prefetch_test() {
    constexpr int HD = 128, G = 4;
    const int nkv = 64, T = 4096, NL = 3;
    const int tpw = attn_mfma_tpw(nkv, T, cus());
    const int ppwg = kAmWgKeys * tpw, splits = (T + ppwg - 1) / ppwg, blocks = nkv * splits;
    const size_t per = (size_t)nkv * T * HD;
    std::vector<__half*> K(NL), V(NL);
    std::vector<char*> Wq(NL);
    const long long wbytes = 50331648;  // the C4 q/k/v matrix
    for (int l = 0; l < NL; ++l) {
        CK(hipMalloc(&K[l], per * 2));
        CK(hipMalloc(&V[l], per * 2));
        CK(hipMalloc(&Wq[l], wbytes));
        fill_h<<<1024, 256>>>(K[l], per, 3 + l);
        fill_h<<<1024, 256>>>(V[l], per, 7 + l);
        CK(hipMemset(Wq[l], 1, wbytes));
    }
    float *q, *out, *part, *sink;
    unsigned* cnt;
    int32_t* posd;
    CK(hipMalloc(&q, sizeof(float) * nkv * G * HD));
    CK(hipMalloc(&out, sizeof(float) * nkv * G * HD));
    CK(hipMalloc(&part, sizeof(float) * (size_t)nkv * G * splits * (HD + kAttnPartPad)));
    CK(hipMalloc(&cnt, sizeof(unsigned) * nkv));
    CK(hipMemset(cnt, 0, sizeof(unsigned) * nkv));
    CK(hipMalloc(&sink, 4096 * 4));
    CK(hipMalloc(&posd, sizeof(int32_t) * 8 * 16));
    std::vector<int32_t> hp(8 * 16, 0);
    for (int b = 0; b < 8; ++b) hp[b * 16] = T - 1;
    CK(hipMemcpy(posd, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    fill_f<<<64, 256>>>(q, (size_t)nkv * G * HD, 11, 2.0f);
    CK(hipDeviceSynchronize());
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto attn = [&](int l) {
        AttnArgs<__half> a{q, K[l], V[l], HD, (long long)T * HD, part, out, cnt, posd, 0, nkv, splits,
                           1.0f / sqrtf((float)HD), 8, 16, nullptr};
        a.defer_merge = 0;
        a.ppwg = ppwg;
        launch_mfma<HD, G>(a, blocks, 2, s);
    };
    auto strm = [&](int l) { hipLaunchKernelGGL(nt_stream_kernel, dim3(192), dim3(1024), 0, s, Wq[l], wbytes, sink); };
    auto timed = [&](const std::function<void(int)>& body) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        for (int l = 0; l < NL; ++l) body(l);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int reps = 20;
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
    for (int rep = 0; rep < 2; ++rep) {
        const double a0 = timed(attn), s0 = timed(strm), sa = timed([&](int l) { strm(l); attn(l); });
        printf("attention alone %.2f us | 50 MB nt stream %.2f | stream + attention %.2f (attention ~%.2f)\n", a0, s0, sa,
               sa - s0);
        for (int nk : {64, 128, 256}) {
            for (int pwg : {64, 32}) {
                const int per_wg = (blocks + pwg - 1) / pwg;
                auto pf = [&](int l) {
                    hipLaunchKernelGGL((kv_prefetch_kernel<HD>), dim3(pwg), dim3(1024), 0, s, K[l], V[l], T, splits, ppwg, nk,
                                       per_wg, blocks, sink);
                };
                const double p0 = timed(pf), ps = timed([&](int l) { pf(l); strm(l); }),
                             psa = timed([&](int l) { pf(l); strm(l); attn(l); }),
                             pa = timed([&](int l) { pf(l); attn(l); });
                printf("  warm %3d keys/split by %2d wg: warm %.2f | warm+stream %.2f | warm+stream+attn %.2f (attention ~%.2f) | "
                       "warm+attn %.2f (attention ~%.2f)\n", nk, pwg, p0, ps, psa, psa - ps, pa, pa - p0);
                fflush(stdout);
            }
        }
    }
}

int main(int argc, char** argv) {
    const int only_tpw = argc > 1 ? atoi(argv[1]) : 0;
    if (only_tpw < 0) {  // tools/attn_mfma_lab -1: the Infinity-Cache warm-up test only
        prefetch_test();
        return 0;
    }
    // correctness sweep (positions around tile / wave / split boundaries), then the timed shapes
    for (int p : {0, 1, 31, 32, 127, 128, 129, 255, 256, 300, 1023, 1024, 2047})
        run<128, 1>("C1-pos", 32, 32, 2048, {p}, 1, 1, 1);
    for (int p : {0, 1, 5, 33, 200, 1000, 4095})
        run<128, 4>("C4-pos", 64, 8, 4096, {p}, 1, 2, 0);
    run<128, 4>("C4-rag", 64, 8, 4096, {1, 4095, 77, 2048, 3000, 5, 1024, 4000}, 1, 2, 0);
    run<128, 2>("G2", 16, 16, 2048, {2047}, 1, 0, 0);
    run<128, 8>("G8", 8, 8, 2048, {1500}, 1, 0, 0);
    run<64, 1>("hd64", 4, 4, 512, {300}, 1, 0, 0);
    run<64, 4>("hd64g4", 2, 2, 512, {511}, 1, 0, 0);
    // timed: C1 (deferred to wo), C4 (merge launch vs in-launch), B1 Llama-3-8B, TP-8 shards
    run<128, 1>("C1", 32, 32, 2048, {2047}, 8, 1, 1);
    run<128, 1>("C1-t1", 32, 32, 2048, {2047}, 8, 1, 1, 1);
    run<128, 4>("C4", 64, 8, 4096, {4095}, 3, 2, 0);
    run<128, 4>("C4-mrg", 64, 8, 4096, {4095}, 3, 2, 2);
    for (int t : {4, 6, 12, 16})
        if (!only_tpw || only_tpw == t) run<128, 4>("C4-tpw", 64, 8, 4096, {4095}, 3, 2, 0, t);
    run<128, 4>("B1-8B", 8, 8, 4096, {4095}, 16, 0, 0);
    run<128, 1>("C2-tp8", 4, 4, 2048, {2047}, 16, 0, 0);
    run<128, 4>("C4-tp8", 8, 1, 4096, {4095}, 16, 2, 0);
    for (int t : {2, 4}) {  // small grids: fewer, longer splits (a shorter last-arriver merge)
        run<128, 4>("C4-tp8-t", 8, 1, 4096, {4095}, 16, 2, 0, t);
        run<128, 4>("B1-8B-t", 8, 8, 4096, {4095}, 16, 0, 0, t);
    }
    return 0;
}
