// persistent.hip — instantiations and host launcher of the persistent step kernel (persistent.h).
#include "persistent.h"

#include "persistent_launch.h"

namespace sli {

namespace {
template <typename WT, typename KT, int HD, int G>
int launch(const StepParams* P, int grid, size_t lds, unsigned* bar, int pb, int pe, int fin, hipStream_t s) {
    auto kern = step_kernel<WT, KT, HD, G>;
    static bool attr_done = false;
    if (!attr_done && lds > 65536)
        SLI_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_done = true;
    SLI_HIP(hipMemsetAsync(bar, 0, sizeof(unsigned) * kBarWords, s));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), lds, s, P, pb, pe, fin);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

template <typename WT, typename KT>
int by_shape(int hd, int g, const StepParams* P, int grid, size_t lds, unsigned* bar, int pb, int pe, int fin,
             hipStream_t s) {
    if (hd == 128 && g == 1) return launch<WT, KT, 128, 1>(P, grid, lds, bar, pb, pe, fin, s);
    if (hd == 128 && g == 4) return launch<WT, KT, 128, 4>(P, grid, lds, bar, pb, pe, fin, s);
    if (hd == 64 && g == 1) return launch<WT, KT, 64, 1>(P, grid, lds, bar, pb, pe, fin, s);
    if (hd == 64 && g == 2) return launch<WT, KT, 64, 2>(P, grid, lds, bar, pb, pe, fin, s);
    return fail(SLI_ERR_STATE, "persistent step: unsupported head shape");
}
}  // namespace

bool persistent_supported(int wd, int kd, int hd, int g) {
    const bool pair = (wd == SLI_DT_F16 && kd == SLI_DT_F16) || wd == SLI_DT_F32 || (wd == SLI_DT_I8 && kd == SLI_DT_F16);
    return pair && ((hd == 128 && (g == 1 || g == 4)) || (hd == 64 && (g == 1 || g == 2)));
}

int persistent_launch(int wd, int kd, int hd, int g, const StepParams* P, int grid, size_t lds, unsigned* bar, int pb,
                      int pe, int fin, hipStream_t s) {
    if (wd == SLI_DT_F16 && kd == SLI_DT_F16) return by_shape<__half, __half>(hd, g, P, grid, lds, bar, pb, pe, fin, s);
    if (wd == SLI_DT_F32 && kd == SLI_DT_F16) return by_shape<float, __half>(hd, g, P, grid, lds, bar, pb, pe, fin, s);
    if (wd == SLI_DT_F32 && kd == SLI_DT_F32) return by_shape<float, float>(hd, g, P, grid, lds, bar, pb, pe, fin, s);
    if (wd == SLI_DT_I8 && kd == SLI_DT_F16) return by_shape<int8_t, __half>(hd, g, P, grid, lds, bar, pb, pe, fin, s);
    return fail(SLI_ERR_STATE, "persistent step not instantiated for this dtype pair");
}

}  // namespace sli
