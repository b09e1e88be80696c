// chain_lab.hip — what overlapping consecutive GEMV launches would buy (diagnostic tool).
//
// A chain of the batch-1 Llama-2-7B projections (q/k/v 12288 x 4096, wo 4096 x 4096, gate/up 22016 x 4096,
// down 4096 x 11008, fp16 weights, 32 layers = 128 launches, 13.2 GB of distinct weights), each launch's input the
// previous launch's output. Modes:
//   graph      : the launches captured in a hipGraph (the engine today): a full kernel boundary per edge
//   direct     : the same launches from the host, no graph
//   graph+wait : captured, with the hand-off protocol below (its cost without any overlap: the graph drops the flag)
//   anyorder   : hipExtLaunchKernel(..., hipExtAnyOrderLaunch): the AQL barrier bit clear, so launch i+1's
//                workgroups become resident while launch i drains; each issues its first weight loads, then waits
//                for launch i's arrival counter (sc1 poll), loads its input with sc1 loads and runs; every launch
//                stores its output sc1, drains, and adds once per workgroup to its own counter (MI355X_MICROARCH.md
//                hand-off table, row 1)
// Prints the chain's time per launch and its weight stream rate, and checks that every mode's final output equals
// the graph mode's bit for bit (the arithmetic is identical; a stale input would show).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hip/hip_fp16.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include <cmath>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kT = 1024, kWaves = 16;
#ifndef LAB_D
#define LAB_D 8  // 16-byte weight loads in flight per lane
#endif
constexpr int kD = LAB_D;
constexpr unsigned kSpin = 1u << 22;

struct Link {
    const __half* W;
    const float* x;
    float* y;
    int rows, K;
    unsigned* wait_ctr;   // nullptr: no wait (kernel boundary ordering)
    unsigned wait_target;
    unsigned* sig_ctr;    // nullptr: no signal
    int* err;
    int steps;            // per wave, a multiple of kD (padded; host-computed)
};

__device__ __forceinline__ float wave_sum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <int NC>
__global__ void __launch_bounds__(kT) chain_gemv(Link L) {
    extern __shared__ __attribute__((aligned(16))) float xs[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int nc = NC;  // 512-k chunks per row (64 lanes x 8 halves)
    const int r0 = (int)(((long long)blockIdx.x * L.rows) / gridDim.x);
    const int r1 = (int)(((long long)(blockIdx.x + 1) * L.rows) / gridDim.x);
    const int my_rows = r1 - r0 > wave ? (r1 - r0 - wave + kWaves - 1) / kWaves : 0;
    const int n_real = my_rows * nc;
    const int n = L.steps;

    auto addr = [&](int s) -> const u32x4* {
        if (s >= n_real) s = 0;
        const unsigned ri = (unsigned)s / nc, c = (unsigned)s - ri * nc;
        const int row = min(r0 + wave + ri * kWaves, L.rows - 1);
        int k = (int)c * 512 + lane * 8;
        if (k >= L.K) k = 0;
        return reinterpret_cast<const u32x4*>(L.W + (size_t)row * L.K + k);
    };

    u32x4 ring[kD];
#pragma unroll
    for (int j = 0; j < kD; ++j) ring[j] = __builtin_nontemporal_load(addr(j));

    if (L.wait_ctr) {
        if (tid == 0) {
            for (unsigned spins = 0;; ++spins) {
                if (__hip_atomic_load(L.wait_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= L.wait_target) break;
                if (spins >= kSpin) { __hip_atomic_fetch_or(L.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
    }
    // input vector -> LDS (zero-padded to nc * 512)
    const int kp = nc * 512;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(L.x), 0, L.K * 4, 0x00020000);
    for (int k = tid * 4; k < kp; k += kT * 4) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (k < L.K) {
            if (L.wait_ctr) v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, 4u * k, 0, 16 /* sc1 */));
            else v = *reinterpret_cast<const f32x4*>(L.x + k);
        }
        *reinterpret_cast<f32x4*>(xs + k) = v;
    }
    __syncthreads();

    float acc = 0.f;
    for (int s0 = 0; s0 < n; s0 += kD) {
#pragma unroll
        for (int j = 0; j < kD; ++j) {
            const int s = s0 + j;
            const u32x4 w = ring[j];
            if (s + kD < n) ring[j] = __builtin_nontemporal_load(addr(s + kD));
            if (s < n_real) {
                const unsigned ri = (unsigned)s / nc, c = (unsigned)s - ri * nc;
                const f32x4 xa = *reinterpret_cast<const f32x4*>(xs + c * 512 + lane * 8);
                const f32x4 xb = *reinterpret_cast<const f32x4*>(xs + c * 512 + lane * 8 + 4);
                const __half2* h = reinterpret_cast<const __half2*>(&w);
                float2 f0 = __half22float2(h[0]), f1 = __half22float2(h[1]), f2 = __half22float2(h[2]),
                       f3 = __half22float2(h[3]);
                acc += f0.x * xa[0] + f0.y * xa[1] + f1.x * xa[2] + f1.y * xa[3] + f2.x * xb[0] + f2.y * xb[1] +
                       f3.x * xb[2] + f3.y * xb[3];
                if (c == nc - 1) {
                    const float v = wave_sum(acc);
                    acc = 0.f;
                    const int row = r0 + wave + (int)ri * kWaves;
                    if (lane == 0) {
                        if (L.sig_ctr) __hip_atomic_store(L.y + row, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        else L.y[row] = v;
                    }
                }
            }
        }
    }
    if (L.sig_ctr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(L.sig_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void fill_half(__half* w, size_t n, unsigned seed, float scale) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        w[i] = __float2half(((h & 0xffff) / 32768.0f - 1.0f) * scale);
    }
}

int main(int argc, char** argv) {
    const int layers = argc > 1 ? atoi(argv[1]) : 32;
    const int grid = 256;
    struct Shape { const char* name; int rows, K; };
    const Shape shapes[4] = {{"qkv", 12288, 4096}, {"wo", 4096, 4096}, {"gate_up", 22016, 4096}, {"down", 4096, 11008}};
    const int n = layers * 4;
    std::vector<Link> links(n);
    std::vector<__half*> ws(n);
    std::vector<float*> ys(n);
    float* x0; CK(hipMalloc(&x0, 16384 * 4));
    std::vector<float> hx(16384);
    for (int i = 0; i < 16384; ++i) hx[i] = ((i * 37) % 101) / 50.0f - 1.0f;
    CK(hipMemcpy(x0, hx.data(), 16384 * 4, hipMemcpyHostToDevice));
    unsigned* ctr; CK(hipMalloc(&ctr, (n + 1) * 128));
    int* err; CK(hipMalloc(&err, 4)); CK(hipMemset(err, 0, 4));
    double bytes = 0;
    for (int i = 0; i < n; ++i) {
        const Shape& s = shapes[i % 4];
        const size_t nw = (size_t)s.rows * s.K;
        CK(hipMalloc(&ws[i], nw * 2));
        hipLaunchKernelGGL(fill_half, dim3(2048), dim3(256), 0, 0, ws[i], nw, 1234u + i, 1.7f / sqrtf((float)s.K));
        CK(hipMalloc(&ys[i], (size_t)s.rows * 4));
        CK(hipMemset(ys[i], 0, (size_t)s.rows * 4));
        bytes += nw * 2.0;
        Link& L = links[i];
        L.W = ws[i]; L.x = i ? ys[i - 1] : x0; L.y = ys[i]; L.rows = s.rows; L.K = s.K; L.err = err;
        const int nc = (s.K + 511) / 512;
        const int rpw = ((s.rows + grid - 1) / grid + kWaves - 1) / kWaves;  // max rows per wave
        L.steps = ((rpw * nc + kD - 1) / kD) * kD;
    }
    CK(hipDeviceSynchronize());
    size_t lds_max = 0;
    for (auto& s : shapes) lds_max = std::max(lds_max, (size_t)((s.K + 511) / 512) * 512 * 4);
    CK(hipFuncSetAttribute((const void*)chain_gemv<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
    CK(hipFuncSetAttribute((const void*)chain_gemv<22>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
    hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

    auto kfn = [](const Link& L) -> const void* { return L.K == 4096 ? (const void*)chain_gemv<8> : (const void*)chain_gemv<22>; };
    auto lds_of = [&](const Link& L) { return (size_t)((L.K + 511) / 512) * 512 * 4; };
    // mode: 0 graph, 1 direct, 2 graph+wait, 3 anyorder
    auto enqueue = [&](int mode) {
        for (int i = 0; i < n; ++i) {
            Link L = links[i];
            const bool wait = mode >= 2;
            L.wait_ctr = (wait && i) ? ctr + (i - 1) * 32 : nullptr;
            L.wait_target = grid;
            L.sig_ctr = wait ? ctr + i * 32 : nullptr;
            void* args[] = {&L};
            CK(hipExtLaunchKernel(kfn(L), dim3(grid), dim3(kT), args, lds_of(L), st, nullptr, nullptr,
                                  (mode == 3 && i) ? hipExtAnyOrderLaunch : 0));
        }
    };
    std::vector<float> ref(4096), out(4096);
    const char* names[4] = {"graph", "direct", "graph+wait", "anyorder"};
    for (int mode : {0, 1, 2, 3}) {
        hipGraphExec_t ge = nullptr;
        if (mode == 0 || mode == 2) {
            hipGraph_t g;
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
            enqueue(mode);
            CK(hipStreamEndCapture(st, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        }
        hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        float best = 1e30f, sum = 0.f;
        const int reps = 6;
        for (int r = 0; r < reps + 1; ++r) {
            CK(hipMemsetAsync(ctr, 0, (n + 1) * 128, st));
            CK(hipEventRecord(a, st));
            if (ge) CK(hipGraphLaunch(ge, st)); else enqueue(mode);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            if (r) { best = std::min(best, ms); sum += ms; }
        }
        int herr; CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(out.data(), ys[n - 1], 4096 * 4, hipMemcpyDeviceToHost));
        if (mode == 0) ref = out;
        const bool same = memcmp(ref.data(), out.data(), 4096 * 4) == 0;
        printf("%-11s %3d launches: mean %8.1f us (best %8.1f) = %6.2f us per launch, %5.2f TB/s | err %d | final "
               "output %s the graph mode's (y[0] %.6g)\n", names[mode], n, 1000.0 * sum / reps, 1000.0 * best,
               1000.0 * sum / reps / n, bytes / (sum / reps * 1e-3) / 1e12, herr, same ? "==" : "!=", out[0]);
        if (ge) CK(hipGraphExecDestroy(ge));
    }
    // one launch of each shape alone (graph of 50 back-to-back copies of layer 0's launch of that shape)
    for (int k = 0; k < 4; ++k) {
        Link L = links[k];
        L.wait_ctr = nullptr; L.sig_ctr = nullptr;
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        void* args[] = {&L};
        for (int r = 0; r < 20; ++r)
            CK(hipExtLaunchKernel(kfn(L), dim3(grid), dim3(kT), args, lds_of(L), st, nullptr, nullptr, 0));
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        CK(hipEventRecord(a, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        const double wb = (double)L.rows * L.K * 2;
        printf("  %-8s alone (L2/MALL-warm repeats): %6.2f us, %5.2f TB/s\n", shapes[k].name, 1000.0 * ms / 20,
               wb / (ms / 20 * 1e-3) / 1e12);
    }
    return 0;
}
