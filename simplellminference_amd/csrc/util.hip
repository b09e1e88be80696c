// util.hip — C-ABI error plumbing and device-memory helpers (include/sli.h "device helpers").
#include <atomic>
#include <cstdio>
#include <string>

#include "common.h"

namespace sli {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? SLI_ERR_NOMEM : SLI_ERR_HIP;
}

int device_cus() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    int n = cache[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
    return n;
}

}  // namespace sli

using namespace sli;

extern "C" {

int sli_version(void) { return 1; }

const char* sli_status_str(int status) {
    switch (status) {
        case SLI_OK: return "ok";
        case SLI_ERR_ARG: return "invalid argument";
        case SLI_ERR_SHAPE: return "shape mismatch";
        case SLI_ERR_RANGE: return "index out of range";
        case SLI_ERR_HIP: return "HIP runtime error";
        case SLI_ERR_NOMEM: return "out of device memory";
        case SLI_ERR_COMM: return "RCCL error";
        case SLI_ERR_STATE: return "invalid state";
        case SLI_ERR_TIMEOUT: return "communicator wait timed out";
        default: return "unknown status";
    }
}

const char* sli_last_error(void) { return g_last_error.c_str(); }

int sli_device_count(int* n) {
    SLI_CHECK(n, SLI_ERR_ARG, "sli_device_count: null");
    SLI_HIP(hipGetDeviceCount(n));
    return SLI_OK;
}

int sli_set_device(int device) {
    SLI_HIP(hipSetDevice(device));
    return SLI_OK;
}

int sli_malloc(void** ptr, size_t bytes) {
    SLI_CHECK(ptr, SLI_ERR_ARG, "sli_malloc: null");
    SLI_HIP(hipMalloc(ptr, bytes ? bytes : 16));
    return SLI_OK;
}

int sli_free(void* ptr) {
    if (ptr) SLI_HIP(hipFree(ptr));
    return SLI_OK;
}

int sli_memset(void* ptr, int value, size_t bytes, sli_stream_t stream) {
    SLI_HIP(hipMemsetAsync(ptr, value, bytes, as_stream(stream)));
    return SLI_OK;
}

int sli_memcpy_h2d(void* dst, const void* src, size_t bytes, sli_stream_t stream) {
    SLI_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, as_stream(stream)));
    return SLI_OK;
}

int sli_memcpy_d2h(void* dst, const void* src, size_t bytes, sli_stream_t stream) {
    SLI_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, as_stream(stream)));
    SLI_HIP(hipStreamSynchronize(as_stream(stream)));
    return SLI_OK;
}

int sli_memcpy_d2d(void* dst, const void* src, size_t bytes, sli_stream_t stream) {
    SLI_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, as_stream(stream)));
    return SLI_OK;
}

int sli_stream_create(sli_stream_t* out) {
    SLI_CHECK(out, SLI_ERR_ARG, "sli_stream_create: null");
    hipStream_t s;
    SLI_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *out = s;
    return SLI_OK;
}

int sli_stream_destroy(sli_stream_t stream) {
    if (stream) SLI_HIP(hipStreamDestroy(as_stream(stream)));
    return SLI_OK;
}

int sli_stream_sync(sli_stream_t stream) {
    SLI_HIP(hipStreamSynchronize(as_stream(stream)));
    return SLI_OK;
}

}  // extern "C"
