// gemv_lab.hip — diagnostic: GEMV configurations (rows per unit R, vectors in flight U, double
// buffering) on the Llama-2-7B decode shapes (fp16 weights, fp32 x), each timed over NL distinct layers
// inside a replayed hipGraph so no launch re-reads weights from the Infinity Cache. Prints µs per launch
// and GB/s of algorithmic weight bytes, a pure streaming-read kernel as the per-shape ceiling, and the
// 4-GEMV layer chain for chosen per-shape configurations.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/gemv_lab.hip -o tools/gemv_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../simplellminference_amd/csrc/gemv.h"

using namespace sli;

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
            exit(1);                                                                        \
        }                                                                                   \
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
__global__ void fill_f(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2246822519u ^ seed;
        h ^= h >> 13;
        h *= 2654435761u;
        h ^= h >> 16;
        p[i] = (float)(h & 0xFFFF) / 65536.0f - 0.5f;
    }
}

// pure streaming read: workgroup b reads its contiguous 1/grid of the bytes, U x 16 B per lane in flight
template <int U>
__global__ void __launch_bounds__(1024) stream_kernel(const char* p, long long bytes, float* out,
                                                      unsigned long long* st = nullptr) {
    const unsigned long long t0 = st ? __builtin_amdgcn_s_memrealtime() : 0;
    const long long per = bytes / gridDim.x;
    const char* b = p + per * blockIdx.x;
    const int nvec = (int)(per / 16);
    float acc = 0.0f;
    for (int v = threadIdx.x; v < nvec; v += U * 1024) {
        u32x4 w[U];
#pragma unroll
        for (int j = 0; j < U; ++j) w[j] = load16<true>(b + (size_t)min(v + j * 1024, nvec - 1) * 16);
#pragma unroll
        for (int j = 0; j < U; ++j) acc += __uint_as_float(w[j].x ^ w[j].y ^ w[j].z ^ w[j].w);
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;
    if (st && (threadIdx.x & 63) == 0) {
        unsigned long long* q = st + ((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 4;
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        q[0] = t0;
        q[1] = t0 + 1000000000ull * (xcc & 15);  // xcc id folded into the staged slot (stream has no staging)
        q[2] = __builtin_amdgcn_s_memrealtime();
        q[3] = 1;
    }
}


// pure streaming read by LDS-DMA (global_load_lds_dwordx4, NT: nt): workgroup b reads its contiguous 1/grid of the
// bytes, each wave a ring of S 1-KiB slots in its own LDS region, S - 1 pieces in flight behind a counted vmcnt
template <int S, bool NT>
__global__ void __launch_bounds__(1024) stream_dma_kernel(const char* p, long long bytes, float* out) {
    extern __shared__ __attribute__((aligned(1024))) char sm[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
    const long long per = bytes / gridDim.x;
    const char* b = p + per * blockIdx.x;
    const long long npieces = per / 1024;  // whole KiB pieces of this workgroup
    const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)(sm + wave * S * 1024);
    long long i = wave;
    int slot = 0;
    for (; i < npieces; i += nw) {
        const char* src = b + i * 1024 + lane * 16;
        const unsigned lds = base + slot * 1024;
        unsigned keep;
        if (NT)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
        else
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
        slot = slot + 1 == S ? 0 : slot + 1;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S - 1) : "memory");  // the oldest piece landed: its slot is free
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float acc = reinterpret_cast<const float*>(sm + wave * S * 1024)[lane];
    if (acc == 1.2345f) out[blockIdx.x] = acc;
}

// streaming read with a dynamic tail (mode "dyn"): workgroup b first reads its contiguous share of the first
// static_frac of the bytes (as stream_kernel), then takes 16 x U KiB chunks of the rest from a counter (one
// agent-scope add per chunk by thread 0, the next chunk's add issued while the current chunk's loads fly), so CUs
// that finish their share early take more of the remainder. ctr: zero before the launch.
template <int U>
__global__ void __launch_bounds__(1024) stream_dyn_kernel(const char* p, long long bytes, float* out, unsigned* ctr,
                                                          float static_frac) {
    __shared__ int chunk_lds[2];
    const long long st_bytes = ((long long)(bytes * static_frac) / (gridDim.x * 16384LL)) * gridDim.x * 16384LL;
    const long long per = st_bytes / gridDim.x;
    const char* b = p + per * blockIdx.x;
    const int nvec = (int)(per / 16);
    float acc = 0.0f;
    // the first dynamic chunk's index, requested before the static share streams
    if (threadIdx.x == 0) chunk_lds[0] = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int v = threadIdx.x; v < nvec; v += U * 1024) {
        u32x4 w[U];
#pragma unroll
        for (int j = 0; j < U; ++j) w[j] = load16<true>(b + (size_t)min(v + j * 1024, nvec - 1) * 16);
#pragma unroll
        for (int j = 0; j < U; ++j) acc += __uint_as_float(w[j].x ^ w[j].y ^ w[j].z ^ w[j].w);
    }
    const long long chunk = 1024LL * U * 16;
    const long long rest = bytes - st_bytes;
    const int nchunks = (int)((rest + chunk - 1) / chunk);
    const char* d = p + st_bytes;
    __syncthreads();
    int c = chunk_lds[0];
    int par = 0;
    while (c < nchunks) {
        if (threadIdx.x == 0)
            chunk_lds[par ^ 1] = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const long long base = (long long)c * chunk;
        const int nv = (int)(min(chunk, rest - base) / 16);
        u32x4 w[U];
#pragma unroll
        for (int j = 0; j < U; ++j) w[j] = load16<true>(d + base + (size_t)min((int)threadIdx.x + j * 1024, nv - 1) * 16);
#pragma unroll
        for (int j = 0; j < U; ++j) acc += __uint_as_float(w[j].x ^ w[j].y ^ w[j].z ^ w[j].w);
        __syncthreads();
        par ^= 1;
        c = chunk_lds[par];
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;
}

// streaming read with a WAVE-level dynamic tail (round 6, mode "dyn2"): the work is cut into units of U KiB (one
// 16-byte load per lane x U); the first static_frac of the units is split evenly over the grid's waves (contiguous
// per wave), the rest into 8 per-XCD pools (pool x = units [S + x D / 8, S + (x + 1) D / 8), x = HW_REG_XCC_ID) that
// the XCD's waves drain one unit per ticket: lane 0 adds 1 to the XCD's head (agent scope) and the next ticket is
// requested with the current unit's loads, so the hand-out round trip hides under the unit. No workgroup barrier.
// ctr: 8 heads 128 B apart, zero before the launch. (Round 5's dyn took 128-KiB chunks per WORKGROUP from one
// counter behind a barrier: a chunk was ~5 us of a CU's stream, coarser than the tail it was meant to remove.)
template <int U>
__global__ void __launch_bounds__(1024) stream_dyn2_kernel(const char* p, long long bytes, float* out, unsigned* ctr,
                                                           float static_frac, unsigned long long* st = nullptr) {
    const unsigned long long t0 = st ? __builtin_amdgcn_s_memrealtime() : 0;
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 16 + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), nw = gridDim.x * 16;
    const long long ub = 1024LL * U;
    const int nu = (int)(bytes / ub);
    const int ns = (int)(nu * static_frac);
    const int u1 = (int)((long long)(gw + 1) * ns / nw);
    int u = (int)((long long)gw * ns / nw);
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const int nd = nu - ns;
    const int d0 = ns + (int)((long long)xcc * nd / 8), dn = ns + (int)((long long)(xcc + 1) * nd / 8) - d0;
    unsigned* head = ctr + xcc * 32;
    unsigned tk = 0;
    if (lane == 0) tk = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float acc = 0.0f;
    for (;;) {
        int unit;
        if (u < u1) {
            unit = u++;
        } else {
            const int t = __builtin_amdgcn_readfirstlane((int)tk);
            if (t >= dn) break;
            unit = d0 + t;
            if (lane == 0) tk = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const char* b = p + (size_t)unit * ub + lane * 16;
        u32x4 w[U];
#pragma unroll
        for (int j = 0; j < U; ++j) w[j] = load16<true>(b + j * 1024);
#pragma unroll
        for (int j = 0; j < U; ++j) acc += __uint_as_float(w[j].x ^ w[j].y ^ w[j].z ^ w[j].w);
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;
    if (st && lane == 0) {
        unsigned long long* q = st + ((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 4;
        q[0] = t0;
        q[1] = t0 + 1000000000ull * xcc;
        q[2] = __builtin_amdgcn_s_memrealtime();
        q[3] = 1;
    }
}

// dyn2 refined (mode "dyn3"): only the first DW waves of a workgroup take dynamic units (DW x 256 pullers instead of
// 4096), a wave requests its first ticket with its LAST static unit (not at entry, where 4096 adds queued ~6 us
// ahead of every first weight load), and each XCD's pool is split into NP sub-pools by workgroup (fewer pullers per
// head word; a sub-pool balances its 32 / NP CUs only).
template <int U, int DW, int NP>
__global__ void __launch_bounds__(1024) stream_dyn3_kernel(const char* p, long long bytes, float* out, unsigned* ctr,
                                                           float static_frac) {
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int gw = blockIdx.x * 16 + wv, nw = gridDim.x * 16;
    const long long ub = 1024LL * U;
    const int nu = (int)(bytes / ub);
    const int ns = (int)(nu * static_frac);
    const int u1 = (int)((long long)(gw + 1) * ns / nw);
    int u = (int)((long long)gw * ns / nw);
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const int pool = (int)xcc * NP + (int)((blockIdx.x >> 3) % NP), npool = 8 * NP;
    const int nd = nu - ns;
    const int d0 = ns + (int)((long long)pool * nd / npool), dn = ns + (int)((long long)(pool + 1) * nd / npool) - d0;
    unsigned* head = ctr + pool * 32;
    const bool dyn = wv < DW;
    unsigned tk = 0;
    if (dyn && u1 <= u && lane == 0) tk = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float acc = 0.0f;
    for (;;) {
        int unit;
        if (u < u1) {
            unit = u++;
            if (dyn && u == u1 && lane == 0) tk = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (!dyn) break;
            const int t = __builtin_amdgcn_readfirstlane((int)tk);
            if (t >= dn) break;
            unit = d0 + t;
            if (lane == 0) tk = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const char* b = p + (size_t)unit * ub + lane * 16;
        u32x4 w[U];
#pragma unroll
        for (int j = 0; j < U; ++j) w[j] = load16<true>(b + j * 1024);
#pragma unroll
        for (int j = 0; j < U; ++j) acc += __uint_as_float(w[j].x ^ w[j].y ^ w[j].z ^ w[j].w);
    }
    if (acc == 1.2345f) out[blockIdx.x] = acc;
}

// latency probe: wave 0 times one L2-hot load while the other 15 waves of the CU have `nw` 16-byte HBM
// loads per lane in flight (nw = 0: idle CU). scalar = 1: wave 0 uses a scalar (s_load) read instead.
__global__ void __launch_bounds__(1024) probe_kernel(const char* W, const float* x, int nw, int scalar,
                                                     unsigned long long* out, float* sink) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float acc = 0.0f;
    if (wave > 0) {
        const char* b = W + ((size_t)blockIdx.x * 16 + wave) * 16384;  // 16 KiB per wave: 64 MiB in all
        u32x4 w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (j < nw) w[j] = load16<true>(b + (size_t)(j * 64 + lane) * 16);
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (j < nw) acc += __uint_as_float(w[j].x);
    } else {
        __builtin_amdgcn_s_sleep(20);  // let the other waves issue first
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        float v;
        if (scalar) {
            v = __builtin_nontemporal_load(x + 7);  // uniform address
        } else {
            v = x[lane];
        }
        acc = v;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) out[blockIdx.x] = t1 - t0;
    }
    if (acc == 1.2345f) sink[threadIdx.x] = acc;
}

struct Shape {
    const char* name;
    int rows, cols;
};
static const Shape kShapes[] = {{"qkv", 12288, 4096}, {"wo", 4096, 4096}, {"gu", 22016, 4096}, {"down", 4096, 11008},
                                {"lm", 32000, 4096}};
constexpr int NL = 20;

struct Cfg {
    const char* name;
    std::function<void(const __half*, const GemvIn&, float*, int, hipStream_t)> run;
};

template <int R, int U, bool DB>
static void run_cfg(const __half* W, const GemvIn& in, float* y, int rows, hipStream_t s) {
    if (R == 0) return;
    EpiStore<R> e{y, nullptr, nullptr, 1.0f, rows};
    CK((launch_gemv<__half, R, U, true>(W, in, e, (rows + R - 1) / R, s)));
}

template <int R, int U, int NB>
static void run_cfg_nb(const __half* W, const GemvIn& in, float* y, int rows, hipStream_t s) {
    EpiStore<R> e{y, nullptr, nullptr, 1.0f, rows};
    CK((launch_gemv<__half, R, U, true, EpiStore<R>, NB>(W, in, e, (rows + R - 1) / R, s)));
}

static float time_graph(hipStream_t s, const std::function<void()>& body, int reps = 5) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    body();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, e;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&e));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e, s));
    CK(hipEventSynchronize(e));
    float ms;
    CK(hipEventElapsedTime(&ms, a, e));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return ms / reps;
}

int main(int argc, char** argv) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<__half*> w[5];
    for (int si = 0; si < 5; ++si) {
        const size_t n = (size_t)kShapes[si].rows * kShapes[si].cols;
        const int layers = si == 4 ? 4 : NL;
        for (int l = 0; l < layers; ++l) {
            __half* p;
            CK(hipMalloc(&p, n * 2));
            hipLaunchKernelGGL(fill_h, dim3(4096), dim3(256), 0, s, p, n, 77u + si * 1000 + l, 0.05f);
            w[si].push_back(p);
        }
    }
    float *x, *nw, *y, *y2;
    CK(hipMalloc(&x, 16384 * 4));
    CK(hipMalloc(&nw, 16384 * 4));
    CK(hipMalloc(&y, 32768 * 4));
    CK(hipMalloc(&y2, 32768 * 4));
    hipLaunchKernelGGL(fill_f, dim3(64), dim3(256), 0, s, x, 16384, 5u);
    hipLaunchKernelGGL(fill_f, dim3(64), dim3(256), 0, s, nw, 16384, 9u);
    CK(hipStreamSynchronize(s));

    const std::string mode = argc > 1 ? argv[1] : "all";
    auto in_for0 = [&](int si) { return GemvIn{x, si == 3 ? nullptr : nw, 1e-5f, kShapes[si].cols}; };
    if (mode == "dma") {
        // streaming-read floor: register loads (stream_kernel, 8 x 16 B per lane in flight, 1024 threads) against
        // LDS-DMA rings (S KiB per wave, nt or default policy, 256 / 512 / 1024 threads), on the gate/up and down
        // matrices (fp16 7B: 180 / 90 MB), each over NL distinct layers in a graph
        for (int si : {2, 3, 0}) {
            const long long bytes = (long long)kShapes[si].rows * kShapes[si].cols * 2;
            auto rep = [&](const char* name, const std::function<void(int)>& f) {
                for (int r = 0; r < 2; ++r) {
                    const float ms = time_graph(s, [&] { for (int l = 0; l < NL; ++l) f(l); });
                    const double us = 1000.0 * ms / NL;
                    printf("%-5s %-24s %7.2f us  %7.1f GB/s\n", kShapes[si].name, name, us, bytes / (us * 1e-6) / 1e9);
                }
                fflush(stdout);
            };
            rep("reg 8x16B 1024t", [&](int l) {
                hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2, nullptr);
            });
#define DMA_CFG(NAME, S_, NT_, THREADS)                                                                          \
            {                                                                                                \
                const size_t lds = (size_t)(THREADS / 64) * S_ * 1024;                                        \
                CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&stream_dma_kernel<S_, NT_>),             \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));              \
                rep(NAME, [&](int l) {                                                                        \
                    hipLaunchKernelGGL((stream_dma_kernel<S_, NT_>), dim3(256), dim3(THREADS), lds, s,           \
                                       (const char*)w[si][l], bytes, y2);                                      \
                });                                                                                           \
            }
            DMA_CFG("dma nt S8 1024t", 8, true, 1024)
            DMA_CFG("dma nt S9 1024t", 9, true, 1024)
            DMA_CFG("dma nt S16 512t", 16, true, 512)
            DMA_CFG("dma nt S32 256t", 32, true, 256)
            DMA_CFG("dma nt S36 256t", 36, true, 256)
            DMA_CFG("dma def S8 1024t", 8, false, 1024)
            DMA_CFG("dma def S32 256t", 32, false, 256)
#undef DMA_CFG
        }
        return 0;
    }
    if (mode == "dyn3") {
        unsigned* ctr;
        CK(hipMalloc(&ctr, NL * 32 * 128));
        for (int si : {0, 1, 2, 3}) {
            const long long bytes = (long long)kShapes[si].rows * kShapes[si].cols * 2;
            auto rep = [&](const char* name, const std::function<void(int)>& f) {
                for (int r = 0; r < 2; ++r) {
                    const float ms = time_graph(s, [&] {
                        CK(hipMemsetAsync(ctr, 0, NL * 32 * 128, s));
                        for (int l = 0; l < NL; ++l) f(l);
                    });
                    const double us = 1000.0 * ms / NL;
                    printf("%-5s %-30s %7.2f us  %7.1f GB/s\n", kShapes[si].name, name, us, bytes / (us * 1e-6) / 1e9);
                }
                fflush(stdout);
            };
            rep("static reg 8x16B", [&](int l) {
                hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2, nullptr);
            });
#define DYN3(U_, DW_, NP_, FR)                                                                                   \
            rep("dyn3 U" #U_ " DW" #DW_ " NP" #NP_ " static " #FR, [&](int l) {                                    \
                hipLaunchKernelGGL((stream_dyn3_kernel<U_, DW_, NP_>), dim3(256), dim3(1024), 0, s,                  \
                                   (const char*)w[si][l], bytes, y2, ctr + l * 32 * 32, FR##f);                      \
            });
            DYN3(8, 16, 1, 0.95) DYN3(8, 4, 1, 0.95) DYN3(8, 4, 4, 0.95) DYN3(8, 2, 1, 0.95)
            DYN3(8, 4, 1, 0.9) DYN3(8, 4, 4, 0.9) DYN3(8, 16, 4, 0.9) DYN3(8, 4, 1, 0.98)
#undef DYN3
        }
        return 0;
    }
    if (mode == "dyn2") {
        // static stream floor (stream_kernel<8>) vs the wave-level dynamic tail (stream_dyn2_kernel) at unit sizes
        // 4 / 8 KiB and static fractions 0.5-0.95; NL distinct matrices per shape in a graph, a memset zeroing the
        // per-XCD heads first (in both, so the floor pays the same node)
        unsigned* ctr;
        CK(hipMalloc(&ctr, NL * 8 * 128));
        for (int si : {0, 1, 2, 3}) {
            const long long bytes = (long long)kShapes[si].rows * kShapes[si].cols * 2;
            auto rep = [&](const char* name, const std::function<void(int)>& f) {
                for (int r = 0; r < 2; ++r) {
                    const float ms = time_graph(s, [&] {
                        CK(hipMemsetAsync(ctr, 0, NL * 8 * 128, s));
                        for (int l = 0; l < NL; ++l) f(l);
                    });
                    const double us = 1000.0 * ms / NL;
                    printf("%-5s %-26s %7.2f us  %7.1f GB/s\n", kShapes[si].name, name, us, bytes / (us * 1e-6) / 1e9);
                }
                fflush(stdout);
            };
            rep("static reg 8x16B", [&](int l) {
                hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2, nullptr);
            });
            for (float fr : {0.95f, 0.9f, 0.8f, 0.5f}) {
                char nm[64];
                snprintf(nm, sizeof nm, "dyn2 U8 static %.2f", fr);
                rep(nm, [&](int l) {
                    hipLaunchKernelGGL(stream_dyn2_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2,
                                       ctr + l * 8 * 32, fr, nullptr);
                });
                snprintf(nm, sizeof nm, "dyn2 U4 static %.2f", fr);
                rep(nm, [&](int l) {
                    hipLaunchKernelGGL(stream_dyn2_kernel<4>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2,
                                       ctr + l * 8 * 32, fr, nullptr);
                });
            }
        }
        return 0;
    }
    if (mode == "dyn") {
        // static stream floor vs a dynamic tail (stream_dyn_kernel): does taking the last part of the bytes from a
        // work counter shorten a launch's tail? NL distinct matrices per shape, in a graph (a memset zeroes the
        // counters first).
        unsigned* ctr;
        CK(hipMalloc(&ctr, NL * 128));
        for (int si : {0, 1, 2, 3}) {
            const long long bytes = (long long)kShapes[si].rows * kShapes[si].cols * 2;
            auto rep = [&](const char* name, const std::function<void(int)>& f) {
                for (int r = 0; r < 2; ++r) {
                    const float ms = time_graph(s, [&] {
                        CK(hipMemsetAsync(ctr, 0, NL * 128, s));
                        for (int l = 0; l < NL; ++l) f(l);
                    });
                    const double us = 1000.0 * ms / NL;
                    printf("%-5s %-26s %7.2f us  %7.1f GB/s\n", kShapes[si].name, name, us, bytes / (us * 1e-6) / 1e9);
                }
                fflush(stdout);
            };
            rep("static reg 8x16B", [&](int l) {
                hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2, nullptr);
            });
            for (float fr : {0.95f, 0.85f, 0.7f, 0.5f}) {
                char nm[64];
                snprintf(nm, sizeof nm, "dyn U8 static %.2f", fr);
                rep(nm, [&](int l) {
                    hipLaunchKernelGGL(stream_dyn_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2,
                                       ctr + l * 32, fr);
                });
                snprintf(nm, sizeof nm, "dyn U4 static %.2f", fr);
                rep(nm, [&](int l) {
                    hipLaunchKernelGGL(stream_dyn_kernel<4>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2,
                                       ctr + l * 32, fr);
                });
            }
        }
        return 0;
    }
    if (mode == "mall") {
        // wo GEMV (R1U2) timed cold (distinct layers) and right after a streaming read of the same matrix
        // (Infinity-Cache hot): is a prefetch in an earlier launch worth anything to the GEMV?
        const Shape& sh = kShapes[1];
        const long long bytes = (long long)sh.rows * sh.cols * 2;
        auto gemv = [&](int l) {
            EpiStore<1> e{y, nullptr, nullptr, 1.0f, sh.rows};
            CK((launch_gemv<__half, 1, 2, true>(w[1][l], in_for0(1), e, sh.rows, s)));
        };
        auto strm = [&](int l) {
            hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[1][l], bytes, y2, nullptr);
        };
        const float cold = time_graph(s, [&] { for (int l = 0; l < NL; ++l) gemv(l); });
        const float str = time_graph(s, [&] { for (int l = 0; l < NL; ++l) strm(l); });
        const float both = time_graph(s, [&] { for (int l = 0; l < NL; ++l) { strm(l); gemv(l); } });
        const float both2 = time_graph(s, [&] { for (int l = 0; l < NL; ++l) { strm(l); strm(l); } });
        printf("wo gemv cold %.2f us, stream cold %.2f us, stream+gemv(hot) %.2f us -> hot gemv ~%.2f us; stream+stream(hot) -> hot stream ~%.2f us\n",
               1000 * cold / NL, 1000 * str / NL, 1000 * both / NL, 1000 * (both - str) / NL, 1000 * (both2 - str) / NL);
        return 0;
    }
    if (mode == "i8") {
        // int8 weights (the fp16 buffers reinterpreted: half their bytes), every (R, U) on each shape, and the
        // streaming-read ceiling of the same bytes
        using I8Run = std::function<void(const int8_t*, const GemvIn&, float*, int, hipStream_t)>;
        auto mk = [](auto r_tag, auto u_tag, auto nb_tag) -> I8Run {
            constexpr int R = decltype(r_tag)::value, U = decltype(u_tag)::value, NB = decltype(nb_tag)::value;
            return [](const int8_t* W, const GemvIn& in, float* y, int rows, hipStream_t s) {
                EpiStore<R> e{y, nullptr, nullptr, 1.0f, rows};
                CK((launch_gemv<int8_t, R, U, true, EpiStore<R>, NB>(W, in, e, (rows + R - 1) / R, s)));
            };
        };
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        using I4 = std::integral_constant<int, 4>;
        std::vector<std::pair<const char*, I8Run>> cf = {
            {"R1U2", mk(I1{}, I2{}, I2{})}, {"R1U2NB3", mk(I1{}, I2{}, I3{})}, {"R1U2NB4", mk(I1{}, I2{}, I4{})},
            {"R1U4", mk(I1{}, I4{}, I2{})}, {"R1U4NB3", mk(I1{}, I4{}, I3{})},
            {"R2U2", mk(I2{}, I2{}, I2{})}, {"R2U2NB3", mk(I2{}, I2{}, I3{})}, {"R2U2NB4", mk(I2{}, I2{}, I4{})},
            {"R2U1NB4", mk(I2{}, I1{}, I4{})}};
        for (int si = 0; si < 4; ++si) {
            const Shape& sh = kShapes[si];
            const double bytes = (double)sh.rows * sh.cols;
            for (auto& c : cf) {
                const float ms = time_graph(s, [&] {
                    for (int l = 0; l < NL; ++l) c.second((const int8_t*)w[si][l], in_for0(si), y, sh.rows, s);
                });
                const double us = 1000.0 * ms / NL;
                printf("i8 %-5s %-6s %8.2f us  %7.1f GB/s\n", sh.name, c.first, us, bytes / (us * 1e-6) / 1e9);
            }
            const float ms = time_graph(s, [&] {
                for (int l = 0; l < NL; ++l)
                    hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l],
                                       (long long)bytes, y2, nullptr);
            });
            const double us = 1000.0 * ms / NL;
            printf("i8 %-5s %-6s %8.2f us  %7.1f GB/s\n", sh.name, "stream", us, bytes / (us * 1e-6) / 1e9);
        }
        return 0;
    }
    if (mode == "tail") {
        // raw per-wave stamps (entry, staged, exit, steps | xcd << 32) of the R1U4 GEMV on every shape, launches
        // 2..NL-1, written to argv[2] for offline analysis (tools/gemv_tail.py)
        const int nst = 256 * 16 * 4;
        unsigned long long* st;
        CK(hipMalloc(&st, (size_t)NL * nst * 8));
        std::vector<unsigned long long> h((size_t)NL * nst);
        FILE* f = fopen(argc > 2 ? argv[2] : "gpurun_out/gemv_tail.bin", "wb");
        for (int si : {0, 1, 2, 3}) {
            const Shape& sh = kShapes[si];
            for (int R : {1, 2}) {
                CK(hipMemset(st, 0, (size_t)NL * nst * 8));
                time_graph(s, [&] {
                    for (int l = 0; l < NL; ++l) {
                        GemvIn in = in_for0(si);
                        in.stamps = st + (size_t)l * nst;
                        if (R == 1) {
                            EpiStore<1> e{y, nullptr, nullptr, 1.0f, sh.rows};
                            CK((launch_gemv<__half, 1, 4, true>(w[si][l], in, e, sh.rows, s)));
                        } else {
                            EpiStore<2> e{y, nullptr, nullptr, 1.0f, sh.rows};
                            CK((launch_gemv<__half, 2, 4, true>(w[si][l], in, e, sh.rows / 2, s)));
                        }
                    }
                }, 1);
                CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
                const int hdr[3] = {si, R, NL};
                fwrite(hdr, 4, 3, f);
                fwrite(h.data(), 8, h.size(), f);
            }
        }
        // the int8 engine configurations (half the bytes: the fp16 buffers reinterpreted)
        for (int si : {0, 1, 2, 3}) {
            const Shape& sh = kShapes[si];
            const int R = (si == 0 || si == 2) ? 2 : 1;
            CK(hipMemset(st, 0, (size_t)NL * nst * 8));
            time_graph(s, [&] {
                for (int l = 0; l < NL; ++l) {
                    GemvIn in = in_for0(si);
                    in.stamps = st + (size_t)l * nst;
                    const int8_t* W8 = (const int8_t*)w[si][l];
                    if (R == 2) {
                        EpiStore<2> e{y, nullptr, nullptr, 1.0f, sh.rows};
                        CK((launch_gemv<int8_t, 2, 2, true>(W8, in, e, sh.rows / 2, s)));
                    } else if (si == 1) {
                        EpiStore<1> e{y, nullptr, nullptr, 1.0f, sh.rows};
                        CK((launch_gemv<int8_t, 1, 2, true>(W8, in, e, sh.rows, s)));
                    } else {
                        EpiStore<1> e{y, nullptr, nullptr, 1.0f, sh.rows};
                        CK((launch_gemv<int8_t, 1, 4, true>(W8, in, e, sh.rows, s)));
                    }
                }
            }, 1);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            const int hdr[3] = {si + 100, R, NL};  // si + 100: int8
            fwrite(hdr, 4, 3, f);
            fwrite(h.data(), 8, h.size(), f);
        }
        fclose(f);
        printf("wrote stamps\n");
        return 0;
    }
    if (mode == "probe") {
        unsigned long long* o;
        CK(hipMalloc(&o, 256 * 8));
        std::vector<unsigned long long> h(256);
        for (int sc : {0, 1})
            for (int nwl : {0, 1, 4, 8, 16}) {
                for (int rep = 0; rep < 3; ++rep) {
                    hipLaunchKernelGGL(probe_kernel, dim3(256), dim3(1024), 0, s, (const char*)w[2][rep], x, nwl, sc, o, y2);
                    CK(hipStreamSynchronize(s));
                }
                CK(hipMemcpy(h.data(), o, 256 * 8, hipMemcpyDeviceToHost));
                std::sort(h.begin(), h.end());
                printf("probe scalar=%d other waves' loads/lane=%2d: wave-0 load latency p50 %.2f us p90 %.2f max %.2f\n", sc,
                       nwl, h[128] * 0.01, h[230] * 0.01, h[255] * 0.01);
            }
        return 0;
    }
    if (mode == "stamps") {
        // per launch: first entry, staged/exit percentiles relative to it, and the gap to the next launch
        const int nst = 256 * 16 * 4;
        unsigned long long* st;
        CK(hipMalloc(&st, (size_t)NL * nst * 8));
        std::vector<unsigned long long> h((size_t)NL * nst);
        auto report = [&](const char* name) {
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            double gap_sum = 0, dur_sum = 0;
            std::vector<double> stg, ex;
            for (int l = 2; l < NL; ++l) {
                const unsigned long long* q = h.data() + (size_t)l * nst;
                unsigned long long t0 = ~0ull, tl = 0;
                for (int i = 0; i < 4096; ++i) {
                    if (q[i * 4 + 3] == 0) continue;
                    t0 = std::min(t0, q[i * 4]);
                    tl = std::max(tl, q[i * 4 + 2]);
                }
                for (int i = 0; i < 4096; ++i) {
                    if (q[i * 4 + 3] == 0) continue;
                    stg.push_back((q[i * 4 + 1] - t0) * 0.01);
                    ex.push_back((q[i * 4 + 2] - t0) * 0.01);
                }
                const unsigned long long* pq = h.data() + (size_t)(l - 1) * nst;
                unsigned long long ptl = 0;
                for (int i = 0; i < 4096; ++i)
                    if (pq[i * 4 + 3]) ptl = std::max(ptl, pq[i * 4 + 2]);
                gap_sum += (double)(t0 - ptl) * 0.01;
                dur_sum += (double)(tl - t0) * 0.01;
            }
            std::sort(stg.begin(), stg.end());
            std::sort(ex.begin(), ex.end());
            auto pc = [](std::vector<double>& v, double f) { return v[(size_t)(f * (v.size() - 1))]; };
            printf("%-16s in-kernel %6.2f us, gap before %5.2f us | staged p50 %5.2f p99 %5.2f | exit p10 %5.2f p50 %5.2f p90 %5.2f p100 %5.2f\n",
                   name, dur_sum / (NL - 2), gap_sum / (NL - 2), pc(stg, .5), pc(stg, .99), pc(ex, .1), pc(ex, .5),
                   pc(ex, .9), pc(ex, 1.0));
        };
        for (int si : {0, 1, 2, 3}) {
            const Shape& sh = kShapes[si];
            CK(hipMemset(st, 0, (size_t)NL * nst * 8));
            time_graph(s, [&] {
                for (int l = 0; l < NL; ++l)
                    hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l],
                                       (long long)sh.rows * sh.cols * 2, y2, st + (size_t)l * nst);
            }, 1);
            report((std::string(sh.name) + " stream").c_str());
            {  // exit time by XCD (launches 2..NL-1), relative to each launch's first entry
                double sum[8] = {0}, mx[8] = {0};
                int cnt[8] = {0};
                for (int l = 2; l < NL; ++l) {
                    const unsigned long long* q = h.data() + (size_t)l * nst;
                    unsigned long long t0 = ~0ull;
                    for (int i = 0; i < 4096; ++i) t0 = std::min(t0, q[i * 4]);
                    for (int i = 0; i < 4096; ++i) {
                        const int xc = (int)((q[i * 4 + 1] - q[i * 4]) / 1000000000ull) & 7;
                        const double e = (q[i * 4 + 2] - t0) * 0.01;
                        sum[xc] += e;
                        cnt[xc]++;
                        mx[xc] = std::max(mx[xc], e);
                    }
                }
                printf("   by XCD mean/max exit:");
                for (int xc = 0; xc < 8; ++xc) printf(" %d:%.1f/%.1f", xc, cnt[xc] ? sum[xc] / cnt[xc] : 0.0, mx[xc]);
                printf("\n");
            }
            for (int R : {1, 2}) {
                CK(hipMemset(st, 0, (size_t)NL * nst * 8));
                if (R == 3) {  // R=1 with the cross-wave barrier after the input loads (flag in stamps[0])
                    for (int l = 0; l < NL; ++l) {
                        const unsigned long long one = 1;
                        CK(hipMemcpy(st + (size_t)l * nst, &one, 8, hipMemcpyHostToDevice));
                    }
                }
                time_graph(s, [&] {
                    for (int l = 0; l < NL; ++l) {
                        GemvIn in = in_for0(si);
                        in.stamps = st + (size_t)l * nst;
                        if (R != 2) {
                            EpiStore<1> e{y, nullptr, nullptr, 1.0f, sh.rows};
                            CK((launch_gemv<__half, 1, 4, true>(w[si][l], in, e, sh.rows, s)));
                        } else {
                            EpiStore<2> e{y, nullptr, nullptr, 1.0f, sh.rows};
                            CK((launch_gemv<__half, 2, 4, true>(w[si][l], in, e, sh.rows / 2, s)));
                        }
                    }
                }, 1);
                report((std::string(sh.name) + (R == 1 ? " R1U4DB" : R == 2 ? " R2U4" : " R1U4DB+bar")).c_str());
            }
        }
        return 0;
    }
    if (mode == "i8s") {
        // int8 weights (the fp16 buffers reinterpreted: half their bytes) at the C3 shapes, the engine's
        // configurations and NB / U variants, with per-wave phase stamps beside the streaming-read floor
        const int nst = 256 * 16 * 4;
        unsigned long long* st;
        CK(hipMalloc(&st, (size_t)NL * nst * 8));
        std::vector<unsigned long long> h((size_t)NL * nst);
        using Run = std::function<void(int, unsigned long long*)>;
        auto report = [&](const char* name, long long bytes, int si, const Run& run) {
            const float g_ms = time_graph(s, [&] { for (int l = 0; l < NL; ++l) run(l, nullptr); });
            const float s_ms = time_graph(s, [&] {
                for (int l = 0; l < NL; ++l)
                    hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l], bytes, y2,
                                       nullptr);
            });
            CK(hipMemset(st, 0, (size_t)NL * nst * 8));
            time_graph(s, [&] { for (int l = 0; l < NL; ++l) run(l, st + (size_t)l * nst); }, 1);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> stg, ex;
            for (int l = 2; l < NL; ++l) {
                const unsigned long long* q = h.data() + (size_t)l * nst;
                unsigned long long t0 = ~0ull;
                for (int i = 0; i < 4096; ++i)
                    if (q[i * 4 + 3]) t0 = std::min(t0, q[i * 4]);
                for (int i = 0; i < 4096; ++i) {
                    if (q[i * 4 + 3] == 0) continue;
                    stg.push_back((q[i * 4 + 1] - t0) * 0.01);
                    ex.push_back((q[i * 4 + 2] - t0) * 0.01);
                }
            }
            std::sort(stg.begin(), stg.end());
            std::sort(ex.begin(), ex.end());
            auto pc = [](std::vector<double>& vv, double f) { return vv.empty() ? 0.0 : vv[(size_t)(f * (vv.size() - 1))]; };
            printf("%-22s gemv %6.2f us  stream %6.2f us | staged p50 %5.2f p99 %5.2f | exit p10 %5.2f p50 %5.2f "
                   "p90 %5.2f max %5.2f\n", name, 1000.0 * g_ms / NL, 1000.0 * s_ms / NL, pc(stg, .5), pc(stg, .99),
                   pc(ex, .1), pc(ex, .5), pc(ex, .9), pc(ex, 1.0));
        };
        auto in_of = [&](int si, bool norm, unsigned long long* stp) {
            GemvIn in{x, norm ? nw : nullptr, 1e-5f, kShapes[si].cols};
            in.stamps = stp;
            return in;
        };
#define I8_CFG(NAME, SI, NORM, R, U, NB)                                                                    \
        report(NAME, (long long)kShapes[SI].rows * kShapes[SI].cols, SI, [&](int l, unsigned long long* stp) { \
            EpiStore<R> e{y, nullptr, nullptr, 1.0f, kShapes[SI].rows};                                    \
            CK((launch_gemv<int8_t, R, U, true, EpiStore<R>, NB>((const int8_t*)w[SI][l], in_of(SI, NORM, stp), \
                                                                 e, kShapes[SI].rows / R, s)));           \
        })
        I8_CFG("i8 qkv R2U2NB2", 0, true, 2, 2, 2);
        I8_CFG("i8 qkv R2U2NB3", 0, true, 2, 2, 3);
        I8_CFG("i8 qkv R2U2NB4", 0, true, 2, 2, 4);
        I8_CFG("i8 qkv R2U1NB4", 0, true, 2, 1, 4);
        I8_CFG("i8 qkv R1U2NB4", 0, true, 1, 2, 4);
        I8_CFG("i8 qkv R1U4NB2", 0, true, 1, 4, 2);
        I8_CFG("i8 gu R2U2NB2", 2, true, 2, 2, 2);
        I8_CFG("i8 gu R2U2NB3", 2, true, 2, 2, 3);
        I8_CFG("i8 down R1U4NB2", 3, false, 1, 4, 2);
        I8_CFG("i8 down R1U4NB3", 3, false, 1, 4, 3);
        I8_CFG("i8 down R1U2NB4", 3, false, 1, 2, 4);
        I8_CFG("i8 down R2U2NB2", 3, false, 2, 2, 2);
        // round 5: whole rows per step (int8 4096 columns = 256 vectors = one U 4 chunk)
        I8_CFG("i8 qkv R2U4NB2", 0, true, 2, 4, 2);
        I8_CFG("i8 gu R2U4NB2", 2, true, 2, 4, 2);
        I8_CFG("i8 gu R1U4NB2", 2, true, 1, 4, 2);
        I8_CFG("i8 wo R1U2NB2", 1, false, 1, 2, 2);
        I8_CFG("i8 wo R1U4NB2", 1, false, 1, 4, 2);
        I8_CFG("i8 wo R2U4NB2", 1, false, 2, 4, 2);
        I8_CFG("i8 down R1U8NB2", 3, false, 1, 8, 2);

#undef I8_CFG
        return 0;
    }
    if (mode == "wo") {
        // the batch-1 wo launches at C1 (Llama-2-7B, 32 heads x 8 splits of 256 positions at position 2047):
        // plain input, merge-staged (ks 1) and the K-split merge-staged form (ks 2, the engine's default), with
        // per-wave phase stamps beside the streaming-read floor of the same bytes
        const int D = 4096, H = 32, HD = 128, MS = 8, PS = HD + 2;  // kAttnPartPad = 2
        float* part;
        int32_t* posd;
        CK(hipMalloc(&part, sizeof(float) * H * MS * PS));
        CK(hipMalloc(&posd, 64));
        hipLaunchKernelGGL(fill_f, dim3(64), dim3(256), 0, s, part, (size_t)H * MS * PS, 13u);
        const int32_t pos = 2047;
        CK(hipMemcpy(posd, &pos, 4, hipMemcpyHostToDevice));
        float* kp;
        CK(hipMalloc(&kp, sizeof(float) * 4 * D));
        const int nst = 256 * 16 * 4;
        unsigned long long* st;
        CK(hipMalloc(&st, (size_t)NL * nst * 8));
        std::vector<unsigned long long> h((size_t)NL * nst);
        const long long bytes = (long long)D * D * 2;
        auto run = [&](int variant, int l, unsigned long long* stp) {
            GemvIn in{x, nullptr, 0.0f, D};
            in.stamps = stp;
            AttnMergeIn am{part, posd, MS, 256, HD};
            if (variant == 0) {
                EpiStore<1> e{y, nullptr, nullptr, 1.0f, D};
                CK((launch_gemv_u<__half, 1, 2, true>(w[1][l], in, e, D, s)));
            } else if (variant == 1) {
                EpiStore<1> e{y, nullptr, nullptr, 1.0f, D};
                GemvIn im{nullptr, nullptr, 0.0f, D};
                im.stamps = stp;
                CK((launch_gemv_merge<__half, 1, 2, true>(w[1][l], im, e, am, D, s)));
            } else if (variant == 2) {
                const int ks = 2;
                GemvIn im{nullptr, nullptr, 0.0f, D / ks};
                im.stamps = stp;
                am.ksplit = ks;
                am.kunits = D;
                const EpiKPart e{kp, nullptr, D, ks};
                CK((launch_gemv_merge_ks<__half, 1, 2, true, EpiKPart, 8, 4>(w[1][l], im, e, am, gemv_ksplit_grid(D, ks), s)));
            } else if (variant == 3) {  // int8 (the fp16 buffer reinterpreted: half its bytes), plain input
                EpiStore<1> e{y, nullptr, nullptr, 1.0f, D};
                CK((launch_gemv_u<int8_t, 1, 2, true>((const int8_t*)w[1][l], in, e, D, s)));
            } else {  // int8 K-split merge-staged (the engine's C3 wo)
                const int ks = 2;
                GemvIn im{nullptr, nullptr, 0.0f, D / ks};
                im.stamps = stp;
                am.ksplit = ks;
                am.kunits = D;
                const EpiKPart e{kp, nullptr, D, ks};
                CK((launch_gemv_merge_ks<int8_t, 1, 1, true, EpiKPart, 8, 2>((const int8_t*)w[1][l], im, e, am,
                                                                             gemv_ksplit_grid(D, ks), s)));
            }
        };
        const float s_ms = time_graph(s, [&] {
            for (int l = 0; l < NL; ++l)
                hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[1][l], bytes, y2, nullptr);
        });
        const char* names[] = {"wo plain", "wo merge ks1", "wo merge ks2", "i8 wo plain", "i8 wo merge ks2"};
        const float s8_ms = time_graph(s, [&] {
            for (int l = 0; l < NL; ++l)
                hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[1][l], bytes / 2, y2, nullptr);
        });
        for (int v = 0; v < 5; ++v) {
            const float sv_ms = v >= 3 ? s8_ms : s_ms;
            const float g_ms = time_graph(s, [&] { for (int l = 0; l < NL; ++l) run(v, l, nullptr); });
            CK(hipMemset(st, 0, (size_t)NL * nst * 8));
            time_graph(s, [&] { for (int l = 0; l < NL; ++l) run(v, l, st + (size_t)l * nst); }, 1);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> ent, stg, ex;
            for (int l = 2; l < NL; ++l) {
                const unsigned long long* q = h.data() + (size_t)l * nst;
                unsigned long long t0 = ~0ull;
                for (int i = 0; i < 4096; ++i)
                    if (q[i * 4 + 3]) t0 = std::min(t0, q[i * 4]);
                for (int i = 0; i < 4096; ++i) {
                    if (q[i * 4 + 3] == 0) continue;
                    ent.push_back((q[i * 4] - t0) * 0.01);
                    stg.push_back((q[i * 4 + 1] - t0) * 0.01);
                    ex.push_back((q[i * 4 + 2] - t0) * 0.01);
                }
            }
            std::sort(ent.begin(), ent.end());
            std::sort(stg.begin(), stg.end());
            std::sort(ex.begin(), ex.end());
            auto pc = [](std::vector<double>& vv, double f) { return vv.empty() ? 0.0 : vv[(size_t)(f * (vv.size() - 1))]; };
            printf("%-13s gemv %6.2f us  stream %6.2f us | entry p50 %5.2f max %5.2f | staged p50 %5.2f p99 %5.2f | "
                   "exit p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f\n", names[v], 1000.0 * g_ms / NL, 1000.0 * sv_ms / NL,
                   pc(ent, .5), pc(ent, 1.0), pc(stg, .5), pc(stg, .99), pc(ex, .1), pc(ex, .5), pc(ex, .9), pc(ex, 1.0));
        }
        return 0;
    }
    if (mode == "split15") {
        // q/k/v at 1.5 two-row units per wave (6144 units, 256 workgroups x 16 waves): the engine's unsplit launch
        // (8 waves of 2 units, 8 of 1 per workgroup) against every unit cut in two column halves (SPLIT, CS 2) at the
        // same U, i.e. 3 equal half-unit items per wave; fp16 U 4 and int8 U 2 (both 2 chunks per row)
        std::vector<float> ref(32768), got(32768);
        const int rows = 12288, cols = 4096;
        for (int i8 = 0; i8 < 2; ++i8) {
            for (int cs : {1, 2}) {
                auto launch = [&](int l, float* out) {
                    GemvIn in{x, nw, 1e-5f, cols};
                    in.csplit = cs;
                    EpiStore<2> e{out, nullptr, nullptr, 1.0f, rows};
                    if (i8) {
                        const int8_t* W8 = (const int8_t*)w[0][l];
                        if (cs == 1) CK((launch_gemv<int8_t, 2, 2, true, EpiStore<2>, 2, false>(W8, in, e, rows / 2, s)));
                        else CK((launch_gemv<int8_t, 2, 2, true, EpiStore<2>, 2, true>(W8, in, e, rows / 2, s)));
                    } else {
                        if (cs == 1) CK((launch_gemv<__half, 2, 4, true, EpiStore<2>, 2, false>(w[0][l], in, e, rows / 2, s)));
                        else CK((launch_gemv<__half, 2, 4, true, EpiStore<2>, 2, true>(w[0][l], in, e, rows / 2, s)));
                    }
                };
                launch(0, cs == 1 ? y : y2);
                CK(hipStreamSynchronize(s));
                CK(hipMemcpy((cs == 1 ? ref : got).data(), cs == 1 ? y : y2, 4 * rows, hipMemcpyDeviceToHost));
                double md = 0;
                if (cs > 1)
                    for (int r = 0; r < rows; ++r) md = std::max(md, (double)std::fabs(ref[r] - got[r]));
                for (int rep = 0; rep < 3; ++rep) {
                    const float ms = time_graph(s, [&] { for (int l = 0; l < NL; ++l) launch(l, y); });
                    printf("%s qkv cs %d  %7.2f us  (max|d| vs cs 1: %.2e)\n", i8 ? "i8 " : "f16", cs, 1000.0 * ms / NL, md);
                }
                fflush(stdout);
            }
            const long long bytes = (long long)rows * cols * (i8 ? 1 : 2);
            const float sm = time_graph(s, [&] {
                for (int l = 0; l < NL; ++l)
                    hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[0][l], bytes, y2, nullptr);
            });
            printf("%s qkv stream %7.2f us\n", i8 ? "i8 " : "f16", 1000.0 * sm / NL);
        }
        return 0;
    }
    if (mode == "downcs") {
        // the 7B down GEMV (4096 rows x 11008 cols fp16, 1376 vectors per row: U 6 leaves the 4th chunk 58 % full)
        // unsplit (the engine) against each row cut in two / four column parts (SPLIT): 2 / 4 items per wave
        std::vector<float> ref(32768), got(32768);
        const int rows = 4096, cols = 11008;
        struct V { int cs, u; };
        for (V v : {V{1, 6}, V{2, 6}, V{2, 4}, V{4, 4}, V{4, 2}, V{1, 8}, V{2, 8}}) {
            auto launch = [&](int l, float* out) {
                GemvIn in{x, nullptr, 1e-5f, cols};
                in.csplit = v.cs;
                EpiStore<1> e{out, nullptr, nullptr, 1.0f, rows};
#define DCS(U_)                                                                                                 \
    do {                                                                                                        \
        if (v.cs == 1) CK((launch_gemv<__half, 1, U_, true, EpiStore<1>, 2, false>(w[3][l], in, e, rows, s)));   \
        else CK((launch_gemv<__half, 1, U_, true, EpiStore<1>, 2, true>(w[3][l], in, e, rows, s)));              \
    } while (0)
                if (v.u == 6) DCS(6);
                else if (v.u == 4) DCS(4);
                else if (v.u == 8) DCS(8);
                else DCS(2);
#undef DCS
            };
            const bool base = v.cs == 1 && v.u == 6;
            launch(0, base ? y : y2);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy((base ? ref : got).data(), base ? y : y2, 4 * rows, hipMemcpyDeviceToHost));
            double md = 0;
            if (!base)
                for (int r = 0; r < rows; ++r) md = std::max(md, (double)std::fabs(ref[r] - got[r]));
            for (int rep = 0; rep < 3; ++rep) {
                const float ms = time_graph(s, [&] { for (int l = 0; l < NL; ++l) launch(l, y); });
                printf("f16 down cs %d U %d  %7.2f us  (max|d| vs cs 1 U 6: %.2e)\n", v.cs, v.u, 1000.0 * ms / NL, md);
            }
            fflush(stdout);
        }
        const float sm = time_graph(s, [&] {
            for (int l = 0; l < NL; ++l)
                hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[3][l],
                                   (long long)rows * cols * 2, y2, nullptr);
        });
        printf("f16 down stream %7.2f us\n", 1000.0 * sm / NL);
        return 0;
    }
    if (mode == "tp8") {
        // the TP-8 shard GEMVs as the engine launches them (launch_gemv_u: the column split at these sizes), per
        // launch phase stamps, beside the streaming-read floor of the same bytes: where a small launch's time goes
        const int nst = 256 * 16 * 4;
        unsigned long long* st;
        CK(hipMalloc(&st, (size_t)NL * nst * 8));
        std::vector<unsigned long long> h((size_t)NL * nst);
        struct T8 { const char* name; int si, rows, cols, R; bool norm; };
        const T8 t8[] = {{"tp8-qkv", 0, 1536, 4096, 2, true}, {"tp8-wo", 1, 4096, 512, 1, false},
                         {"tp8-gu", 2, 2752, 4096, 2, true}, {"tp8-down", 3, 4096, 1376, 1, false},
                         {"tp4-qkv", 0, 3072, 4096, 2, true}, {"tp4-gu", 2, 5504, 4096, 2, true},
                         {"tp2-gu", 2, 11008, 4096, 2, true}, {"tp1-qkv", 0, 12288, 4096, 2, true},
                         {"tp1-down", 3, 4096, 11008, 1, false}};
        for (const T8& t : t8) {
            const long long bytes = (long long)t.rows * t.cols * 2;
            auto launch = [&](int l, unsigned long long* stp) {
                GemvIn in{x, t.norm ? nw : nullptr, 1e-5f, t.cols};
                in.stamps = stp;
                if (t.R == 2) {
                    EpiStore<2> e{y, nullptr, nullptr, 1.0f, t.rows};
                    CK((launch_gemv_u<__half, 2, 4, true>(w[t.si][l], in, e, t.rows / 2, s)));
                } else if (t.si == 1) {
                    EpiStore<1> e{y, nullptr, nullptr, 1.0f, t.rows};
                    CK((launch_gemv_u<__half, 1, 2, true>(w[t.si][l], in, e, t.rows, s)));
                } else {
                    EpiStore<1> e{y, nullptr, nullptr, 1.0f, t.rows};
                    CK((launch_gemv_u<__half, 1, 6, true>(w[t.si][l], in, e, t.rows, s)));
                }
            };
            const float g_ms = time_graph(s, [&] { for (int l = 0; l < NL; ++l) launch(l, nullptr); });
            const float s_ms = time_graph(s, [&] {
                for (int l = 0; l < NL; ++l)
                    hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[t.si][l], bytes, y2,
                                       nullptr);
            });
            CK(hipMemset(st, 0, (size_t)NL * nst * 8));
            time_graph(s, [&] { for (int l = 0; l < NL; ++l) launch(l, st + (size_t)l * nst); }, 1);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> ent, stg, ex;
            for (int l = 2; l < NL; ++l) {
                const unsigned long long* q = h.data() + (size_t)l * nst;
                unsigned long long t0 = ~0ull;
                for (int i = 0; i < 4096; ++i)
                    if (q[i * 4 + 3]) t0 = std::min(t0, q[i * 4]);
                for (int i = 0; i < 4096; ++i) {
                    if (q[i * 4 + 3] == 0) continue;
                    ent.push_back((q[i * 4] - t0) * 0.01);
                    stg.push_back((q[i * 4 + 1] - t0) * 0.01);
                    ex.push_back((q[i * 4 + 2] - t0) * 0.01);
                }
            }
            std::sort(ent.begin(), ent.end());
            std::sort(stg.begin(), stg.end());
            std::sort(ex.begin(), ex.end());
            auto pc = [](std::vector<double>& v, double f) { return v.empty() ? 0.0 : v[(size_t)(f * (v.size() - 1))]; };
            printf("%-9s %5.2f MB  gemv %6.2f us  stream %6.2f us | waves %zu: entry p50 %5.2f max %5.2f | staged p50 %5.2f "
                   "p99 %5.2f | exit p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f\n",
                   t.name, bytes / 1e6, 1000.0 * g_ms / NL, 1000.0 * s_ms / NL, ent.size() / (NL - 2), pc(ent, .5),
                   pc(ent, 1.0), pc(stg, .5), pc(stg, .99), pc(ex, .1), pc(ex, .5), pc(ex, .9), pc(ex, 1.0));
        }
        return 0;
    }
    std::vector<Cfg> cfgs = {
        {"R2U4", run_cfg<2, 4, true>}, {"R2U4NB3", run_cfg_nb<2, 4, 3>}, {"R2U2NB4", run_cfg_nb<2, 2, 4>},
        {"R1U6", run_cfg<1, 6, true>}, {"R1U6NB3", run_cfg_nb<1, 6, 3>}, {"R1U4NB3", run_cfg_nb<1, 4, 3>},
        {"R1U2", run_cfg<1, 2, true>}, {"R1U2NB3", run_cfg_nb<1, 2, 3>}, {"R1U2NB4", run_cfg_nb<1, 2, 4>},
    };
    auto in_for = [&](int si) { return GemvIn{x, si == 3 ? nullptr : nw, 1e-5f, kShapes[si].cols}; };

    // correctness against the first configuration
    std::vector<float> h1(32768), h2(32768);
    for (int si = 0; si < 5; ++si) {
        cfgs[0].run(w[si][0], in_for(si), y, kShapes[si].rows, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h1.data(), y, 4 * kShapes[si].rows, hipMemcpyDeviceToHost));
        for (size_t c = 1; c < cfgs.size(); ++c) {
            cfgs[c].run(w[si][0], in_for(si), y2, kShapes[si].rows, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h2.data(), y2, 4 * kShapes[si].rows, hipMemcpyDeviceToHost));
            double md = 0, mx = 0;
            for (int r = 0; r < kShapes[si].rows; ++r) {
                md = fmax(md, fabs((double)h1[r] - h2[r]));
                mx = fmax(mx, fabs((double)h1[r]));
            }
            if (md > 1e-4 * (mx + 1)) printf("MISMATCH %s %s max|diff| %.3e\n", kShapes[si].name, cfgs[c].name, md);
        }
    }
    std::vector<std::vector<double>> us_tab(5, std::vector<double>(cfgs.size()));
    for (int si = 0; si < 5; ++si) {
        const int layers = (int)w[si].size();
        const double bytes = (double)kShapes[si].rows * kShapes[si].cols * 2;
        for (size_t c = 0; c < cfgs.size(); ++c) {
            const float ms = time_graph(s, [&] {
                for (int l = 0; l < layers; ++l) cfgs[c].run(w[si][l], in_for(si), y, kShapes[si].rows, s);
            });
            const double us = 1000.0 * ms / layers;
            us_tab[si][c] = us;
            printf("%-5s %-9s %8.2f us  %7.1f GB/s\n", kShapes[si].name, cfgs[c].name, us, bytes / (us * 1e-6) / 1e9);
        }
        const float ms = time_graph(s, [&] {
            for (int l = 0; l < layers; ++l)
                hipLaunchKernelGGL(stream_kernel<8>, dim3(256), dim3(1024), 0, s, (const char*)w[si][l],
                                   (long long)kShapes[si].rows * kShapes[si].cols * 2, y2);
        });
        const double us = 1000.0 * ms / layers;
        printf("%-5s %-9s %8.2f us  %7.1f GB/s\n", kShapes[si].name, "stream", us, bytes / (us * 1e-6) / 1e9);
    }
    // layer chain with the best configuration per shape vs the baseline
    std::vector<int> best(4, 0);
    for (int si = 0; si < 4; ++si)
        for (size_t c = 0; c < cfgs.size(); ++c)
            if (us_tab[si][c] < us_tab[si][best[si]]) best[si] = (int)c;
    const double lbytes = 2.0 * (12288.0 * 4096 + 4096.0 * 4096 + 22016.0 * 4096 + 4096.0 * 11008);
    for (int pick = 0; pick < 2; ++pick) {
        const float ms = time_graph(s, [&] {
            for (int l = 0; l < NL; ++l)
                for (int si = 0; si < 4; ++si) {
                    const int c = pick ? best[si] : 0;
                    cfgs[c].run(w[si][l], in_for(si), y, kShapes[si].rows, s);
                }
        });
        const double us = 1000.0 * ms / NL;
        printf("layer chain %s: %8.2f us/layer  %7.1f GB/s  [", pick ? "best" : "R2U4", us, lbytes / (us * 1e-6) / 1e9);
        for (int si = 0; si < 4; ++si) printf(" %s=%s", kShapes[si].name, cfgs[pick ? best[si] : 0].name);
        printf(" ]\n");
    }
    return 0;
}

// the lab links without libsli: the persistent-grid size from the device (util.hip's device_cus)
int sli::device_cus() {
    int n = 0;
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, 0) == hipSuccess && n > 0 ? n : 256;
}
