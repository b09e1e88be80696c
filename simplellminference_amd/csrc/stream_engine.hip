// stream_engine.hip — host side of the stream engine (stream_engine.h): the geometry the host chooses (ring
// slots, attention job size, LDS layout) and one kernel instantiation per (weight type, KV type, head_dim,
// heads per kv head).
#include <algorithm>

#include "ops_internal.h"
#include "stream_engine.h"

namespace sli {

int es_positions_per_slot(int kv_dtype, int hd) { return kEsSlot / (hd * (kv_dtype == SLI_DT_F16 ? 2 : 4)); }

// Attention jobs: (kv head, split of ppj positions); ppj = PPS x spj with spj the smallest count of slot pairs
// that keeps every job of a full context on its own CU (hkv x ceil(T / ppj) <= grid).
int es_job_positions(int kv_dtype, int hd, int hkv, int T, int grid) {
    const int pps = es_positions_per_slot(kv_dtype, hd);
    const int slots = (T + pps - 1) / pps;
    int spj = 1;
    while ((long long)hkv * ((slots + spj - 1) / spj) > grid) ++spj;
    return pps * spj;
}


// LDS layout: ring [slots][16 KiB] at 0, then xs (the staged input; the attention scratch aliases it), res (the
// row sums of this CU's rows of one op), xres (this CU's rows of the residual stream), ctl.
int es_layout(int D, int Il, int hq, int hd, int hkv, int v_n, int grid, EsLds* out) {
    const int g = hq / hkv;
    auto up16 = [](int b) { return (b + 15) & ~15; };
    const int xs = up16(4 * std::max({D, Il, hq * hd, kEsNC * g * (hd + 2)}));
    auto res_rows = [&](int nu, int R) {
        const int units = (nu + grid - 1) / grid;
        return ((units * R + kEsNC - 1) / kEsNC) * kEsNC;
    };
    const int res = up16(4 * std::max({res_rows((hq + 2 * hkv) * hd / 2, 2), res_rows(D, 1), res_rows(Il, 2),
                                       res_rows(v_n, 1)}));
    const int xres = up16(4 * ((D + grid - 1) / grid));
    const int ctl = 4 * kEsCtlWords;
    const int rest = xs + res + xres + ctl;
    const int budget = 160 * 1024;
    const int slots = std::min(kEsMaxSlots, (budget - rest) / kEsSlot);
    if (slots < 3) return fail(SLI_ERR_SHAPE, "stream engine: LDS cannot hold 3 ring slots beside the staged input");
    out->slots = slots;
    out->xs = slots * kEsSlot;
    out->res = out->xs + xs;
    out->xres = out->res + res;
    out->ctl = out->xres + xres;
    out->total = out->ctl + ctl;
    return SLI_OK;
}

template <typename WT, typename KT, int HD, int G>
static int launch_t(const EsArgs* a_dev, int grid, size_t lds, hipStream_t s, int mode) {
    auto k = es_step_kernel<WT, KT, HD, G>;
    if (mode == 1) {
        SLI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
        int per_cu = 0;
        SLI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kEsThreads, lds));
        // every workgroup must be resident at once (they wait on each other's arrivals)
        SLI_CHECK(per_cu >= 1 && (long long)per_cu * device_cus() >= grid, SLI_ERR_STATE,
                  "stream engine: the grid cannot be co-resident (LDS / registers)");
        return SLI_OK;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(kEsThreads), lds, s, a_dev);
    SLI_HIP(hipGetLastError());
    return SLI_OK;
}

template <typename WT, typename KT, int HD>
static int launch_g(const EsArgs* a_dev, int g, int grid, size_t lds, hipStream_t s, int mode) {
    if (g == 1) return launch_t<WT, KT, HD, 1>(a_dev, grid, lds, s, mode);
    if (g == 2) return launch_t<WT, KT, HD, 2>(a_dev, grid, lds, s, mode);
    if (g == 4) return launch_t<WT, KT, HD, 4>(a_dev, grid, lds, s, mode);
    return fail(SLI_ERR_SHAPE, "stream engine: heads per kv head must be 1, 2 or 4");
}

template <typename WT, typename KT>
static int launch_h(const EsArgs* a_dev, int hd, int g, int grid, size_t lds, hipStream_t s, int mode) {
    if (hd == 128) return launch_g<WT, KT, 128>(a_dev, g, grid, lds, s, mode);
    if (hd == 64) return launch_g<WT, KT, 64>(a_dev, g, grid, lds, s, mode);
    return fail(SLI_ERR_SHAPE, "stream engine: head_dim must be 64 or 128");
}

template <typename WT>
static int launch_k(const EsArgs* a_dev, int kv_dtype, int hd, int g, int grid, size_t lds, hipStream_t s, int mode) {
    if (kv_dtype == SLI_DT_F16) return launch_h<WT, __half>(a_dev, hd, g, grid, lds, s, mode);
    return launch_h<WT, float>(a_dev, hd, g, grid, lds, s, mode);
}

// mode 0: launch; 1: prepare (raise the dynamic-LDS limit, check co-residency)
int es_launch(const EsArgs* a_dev, int w_dtype, int kv_dtype, int hd, int g, int grid, size_t lds, hipStream_t s,
              int mode) {
    switch (w_dtype) {
        case SLI_DT_F16: return launch_k<__half>(a_dev, kv_dtype, hd, g, grid, lds, s, mode);
        case SLI_DT_F32: return launch_k<float>(a_dev, kv_dtype, hd, g, grid, lds, s, mode);
        case SLI_DT_I8: return launch_k<int8_t>(a_dev, kv_dtype, hd, g, grid, lds, s, mode);
        default: return fail(SLI_ERR_ARG, "stream engine: bad weight dtype");
    }
}

}  // namespace sli
