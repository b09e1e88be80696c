// rope_table.h — the RoPE sin/cos table (source/kernel/cpu/rope_kernel.cpp:4-19).
// Computed on the host in float with libm powf/sinf/cosf, so the table is bit-identical to the
// reference CPU table; the device only ever reads it (on-device sinf/powf would differ by ulps and
// turn a memory-bound op VALU-bound: cdna_hip_programming.md Appendix B, Element-wise).
#pragma once
#include <math.h>

#include <vector>

namespace sli {

inline void rope_table_host(int head_dim, int max_seq_len, float theta, std::vector<float>& sin_t,
                            std::vector<float>& cos_t) {
    const int half = head_dim / 2;
    sin_t.resize((size_t)max_seq_len * half);
    cos_t.resize((size_t)max_seq_len * half);
    for (int i = 0; i < max_seq_len; i++) {
        for (int d = 0; d < half; d++) {
            const int tmp = 2 * d;
            const float freq = 1.0f / powf(theta, (float)tmp / (float)head_dim);
            const float val = freq * (float)i;
            sin_t[(size_t)i * half + d] = sinf(val);
            cos_t[(size_t)i * half + d] = cosf(val);
        }
    }
}

}  // namespace sli
