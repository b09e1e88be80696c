// launch_overhead.hip — per-kernel cost inside a replayed hipGraph on this GPU (diagnostic tool).
// Chains N dependent launches of (a) a 1-thread kernel and (b) a 256-workgroup x 1024-thread kernel
// that touches one word per workgroup; prints mean microseconds per launch.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void tiny(int* p) { if (threadIdx.x == 0) p[0] += 1; }
__global__ void __launch_bounds__(1024) wide(int* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int run(const char* name, bool use_wide, int n, hipStream_t s, int* buf) {
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < n; ++i) {
        if (use_wide) hipLaunchKernelGGL(wide, dim3(256), dim3(1024), 0, s, buf);
        else hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, buf);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int reps = 20;
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    printf("%-6s graph of %4d launches: %.3f us per launch\n", name, n, 1000.0 * ms / (reps * n));
    return 0;
}

int main() {
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int* buf; CK(hipMalloc(&buf, 4096)); CK(hipMemset(buf, 0, 4096));
    for (int n : {50, 200}) { run("tiny", false, n, s, buf); run("wide", true, n, s, buf); }
    return 0;
}
