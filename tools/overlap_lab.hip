// overlap_lab.hip — does a kernel launched with hipExtAnyOrderLaunch (AQL barrier bit clear) start before the
// previous kernel on the same stream has finished, on this GPU, directly and inside a captured hipGraph?
// (diagnostic tool: the answer decides whether a GEMV can prefetch its first weight steps during the previous
// launch's tail instead of after the kernel boundary.)
//
// A: 256 workgroups that each spin `spin_us` (s_memrealtime, 100 MHz) and record their end time.
// B: 256 workgroups that record their start time.
// Prints max(A end) -> min(B start): negative = B started while A still ran.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void __launch_bounds__(256) spin_kernel(unsigned long long* end, int spin_ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long t = t0;
    // workgroup b spins spin_ticks * (1 + b % 4) / 4: a ragged tail like a real launch's
    const unsigned long long lim = (unsigned long long)spin_ticks * (1 + blockIdx.x % 4) / 4;
    while (t - t0 < lim) { __builtin_amdgcn_s_sleep(1); t = __builtin_amdgcn_s_memrealtime(); }
    if (threadIdx.x == 0) end[blockIdx.x] = t;
}

__global__ void __launch_bounds__(256) stamp_kernel(unsigned long long* start) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) start[blockIdx.x] = t;
}

static void report(const char* name, const unsigned long long* h, int n) {
    const unsigned long long* a_end = h;
    const unsigned long long* b_start = h + n;
    unsigned long long amax = 0, amin = ~0ull, bmin = ~0ull, bmax = 0;
    for (int i = 0; i < n; ++i) {
        amax = std::max(amax, a_end[i]); amin = std::min(amin, a_end[i]);
        bmin = std::min(bmin, b_start[i]); bmax = std::max(bmax, b_start[i]);
    }
    int early = 0;
    for (int i = 0; i < n; ++i) early += b_start[i] < amax;
    printf("%-28s A end spread %6.2f us | last A end -> first B start %+7.2f us, -> last B start %+7.2f us | "
           "B workgroups started before A ended: %d/%d\n", name, (amax - amin) / 100.0,
           ((double)bmin - (double)amax) / 100.0, ((double)bmax - (double)amax) / 100.0, early, n);
}

int main() {
    const int n = 256, spin_ticks = 2000;  // 20 us
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long* d; CK(hipMalloc(&d, 2 * n * sizeof(unsigned long long)));
    std::vector<unsigned long long> h(2 * n);
    unsigned long long* a_end = d;
    unsigned long long* b_start = d + n;
    int ticks = spin_ticks;
    void* a_args[] = {&a_end, &ticks};
    void* b_args[] = {&b_start};

    for (int flag : {0, 1}) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemsetAsync(d, 0, 2 * n * sizeof(unsigned long long), s));
            CK(hipExtLaunchKernel((const void*)spin_kernel, dim3(n), dim3(256), a_args, 0, s, nullptr, nullptr, 0));
            CK(hipExtLaunchKernel((const void*)stamp_kernel, dim3(n), dim3(256), b_args, 0, s, nullptr, nullptr, flag));
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
            char name[64]; snprintf(name, sizeof name, "direct flag=%d rep %d", flag, rep);
            report(name, h.data(), n);
        }
        // the same pair captured into a graph and replayed
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        CK(hipExtLaunchKernel((const void*)spin_kernel, dim3(n), dim3(256), a_args, 0, s, nullptr, nullptr, 0));
        CK(hipExtLaunchKernel((const void*)stamp_kernel, dim3(n), dim3(256), b_args, 0, s, nullptr, nullptr, flag));
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemsetAsync(d, 0, 2 * n * sizeof(unsigned long long), s));
            CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
            char name[64]; snprintf(name, sizeof name, "graph  flag=%d rep %d", flag, rep);
            report(name, h.data(), n);
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
