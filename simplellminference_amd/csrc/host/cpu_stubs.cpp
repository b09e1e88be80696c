// cpu_stubs.cpp — weak definitions of the reference's CPU kernel symbols (include/kernel/cpu_kernels.h).
// The product has no CPU backend (a CPU path would be a silent fallback): a layer run on
// DeviceType::kDeviceCPU stops here with the reference's LOG, unless the integrating build keeps the
// reference's own source/kernel/cpu/*.cpp, whose strong definitions replace these.
#include "cpu_kernels.h"

#define SLI_NO_CPU(name) LOG(name ": libsli.so has no CPU backend (run the layer on kDeviceCUDA, or link the reference's CPU kernels)")

namespace kernel {

__attribute__((weak)) void add_kernel_cpu(const mem::Tensor&, const mem::Tensor&, const mem::Tensor&, int32_t) {
    SLI_NO_CPU("add_kernel_cpu");
}
__attribute__((weak)) void emb_kernel_cpu(const mem::Tensor&, const mem::Tensor&, const mem::Tensor&, int32_t, int32_t) {
    SLI_NO_CPU("emb_kernel_cpu");
}
__attribute__((weak)) void matmul_kernel_cpu(const mem::Tensor&, const mem::Tensor&, const mem::Tensor&, int32_t, int32_t,
                                             float) {
    SLI_NO_CPU("matmul_kernel_cpu");
}
__attribute__((weak)) void mha_kernel_cpu(const mem::Tensor&, const mem::Tensor&, const mem::Tensor&, const mem::Tensor&,
                                          const mem::Tensor&, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t,
                                          int32_t, int32_t, base::DeviceType) {
    SLI_NO_CPU("mha_kernel_cpu");
}
__attribute__((weak)) void rmsnorm_kernel_cpu(const mem::Tensor&, const mem::Tensor&, const mem::Tensor&, int32_t, float) {
    SLI_NO_CPU("rmsnorm_kernel_cpu");
}
__attribute__((weak)) void rope_cache_cal(int, int, const mem::Tensor, const mem::Tensor, float) {
    SLI_NO_CPU("rope_cache_cal");
}
__attribute__((weak)) void rope_kernel_cpu(const mem::Tensor&, const mem::Tensor&, const mem::Tensor&, const mem::Tensor&,
                                           const mem::Tensor&, int32_t, int32_t) {
    SLI_NO_CPU("rope_kernel_cpu");
}
__attribute__((weak)) void swiglu_kernel_cpu(const mem::Tensor&, const mem::Tensor&, const mem::Tensor&, int32_t) {
    SLI_NO_CPU("swiglu_kernel_cpu");
}

}  // namespace kernel
