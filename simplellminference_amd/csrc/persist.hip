// persist.hip — launcher of the persistent batch-1 decode step (persist.h) for the engine (engine.hip):
// one instantiation per (weight type, KV type, head_dim, heads per kv head).
#include "ops_internal.h"
#include "persist.h"

namespace sli {

int ps_max_splits(int kv_dtype, int hd, int T) {
    int ppwg = 0;
    if (kv_dtype == SLI_DT_F16)
        ppwg = hd == 128 ? PsAttnGeom<__half, 128>::PPWG : PsAttnGeom<__half, 64>::PPWG;
    else
        ppwg = hd == 128 ? PsAttnGeom<float, 128>::PPWG : PsAttnGeom<float, 64>::PPWG;
    return (T + ppwg - 1) / ppwg;
}

template <typename WT, typename KT, int HD, int G>
static int launch_t(const PsArgs& a, const PsArgs* a_dev, int grid, size_t lds, hipStream_t s, bool prepare) {
    auto k = ps_step_kernel<WT, KT, HD, G>;
    if (prepare) {
        SLI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
        return SLI_OK;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(kPsThreads), lds, s, a_dev);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

template <typename WT, typename KT, int HD>
static int launch_g(const PsArgs& a, const PsArgs* a_dev, int g, int grid, size_t lds, hipStream_t s, bool prepare) {
    if (g == 1) return launch_t<WT, KT, HD, 1>(a, a_dev, grid, lds, s, prepare);
    if (g == 2) return launch_t<WT, KT, HD, 2>(a, a_dev, grid, lds, s, prepare);
    return fail(SLI_ERR_SHAPE, "persistent step: heads per kv head must be 1 or 2");
}

template <typename WT, typename KT>
static int launch_h(const PsArgs& a, const PsArgs* a_dev, int g, int grid, size_t lds, hipStream_t s, bool prepare) {
    if (a.hd == 128) return launch_g<WT, KT, 128>(a, a_dev, g, grid, lds, s, prepare);
    if (a.hd == 64) return launch_g<WT, KT, 64>(a, a_dev, g, grid, lds, s, prepare);
    return fail(SLI_ERR_SHAPE, "persistent step: head_dim must be 64 or 128");
}

template <typename WT>
static int launch_k(const PsArgs& a, const PsArgs* a_dev, int kv_dtype, int g, int grid, size_t lds, hipStream_t s, bool prepare) {
    if (kv_dtype == SLI_DT_F16) return launch_h<WT, __half>(a, a_dev, g, grid, lds, s, prepare);
    return launch_h<WT, float>(a, a_dev, g, grid, lds, s, prepare);
}

int ps_launch(const PsArgs& a, const PsArgs* a_dev, int w_dtype, int kv_dtype, int grid, size_t lds, hipStream_t s, bool prepare) {
    const int g = a.hq / a.hkv;
    switch (w_dtype) {
        case SLI_DT_F16: return launch_k<__half>(a, a_dev, kv_dtype, g, grid, lds, s, prepare);
        case SLI_DT_F32: return launch_k<float>(a, a_dev, kv_dtype, g, grid, lds, s, prepare);
        case SLI_DT_I8: return launch_k<int8_t>(a, a_dev, kv_dtype, g, grid, lds, s, prepare);
        default: return fail(SLI_ERR_ARG, "persistent step: bad weight dtype");
    }
}

}  // namespace sli
