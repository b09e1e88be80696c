// common.h — shared HIP helpers for the gfx950 decode path (wave64 reductions, 16-byte vector loads,
// error plumbing for the C ABI).
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/sli.h"

namespace sli {

constexpr int kWave = 64;  // CDNA wavefront; never 32 (MI355X_MICROARCH.md "wave = 64 not 32")
// Split-context attention partial row: o[hd], m, l, 2 pad floats (16-B aligned rows for float4 merges).
constexpr int kAttnPartPad = 4;

// ---------------------------------------------------------------- error plumbing (host)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);
// Compute units of the current device (hipDeviceProp_t::multiProcessorCount, cached per device): every
// persistent grid is sized from it, never from a hard-coded chip geometry.
int device_cus();

#define SLI_HIP(expr)                                         \
    do {                                                      \
        hipError_t e_ = (expr);                               \
        if (e_ != hipSuccess) return ::sli::hip_fail(e_, #expr); \
    } while (0)

#define SLI_CHECK(cond, code, msg)                        \
    do {                                                  \
        if (!(cond)) return ::sli::fail((code), (msg));   \
    } while (0)

inline hipStream_t as_stream(sli_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- device helpers
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Lane exchanges inside a 16-lane DPP row as VALU operand modifiers (no LDS round trip, unlike the
// ds_bpermute that __shfl_xor becomes): xor 1 and xor 2 as quad permutations, then the half-row mirror
// (lane i <-> 7 - i: pairs each quad with the other quad of its 8) and the row mirror (i <-> 15 - i: pairs
// the two halves). A butterfly over these four reaches every lane of the row; beyond 16 lanes the
// exchange is a ds_bpermute (xor 16, xor 32).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1, 0, 3, 2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2, 3, 0, 1]
constexpr int kDppHalfMirror = 0x141;  // row_half_mirror
constexpr int kDppMirror = 0x140;      // row_mirror

constexpr int kDppRor8 = 0x128;        // row_ror:8 (lane i <- i + 8 mod 16: xor 8 inside a row)

// Across rows: the gfx950 permlane swaps (VALU). With both operands the same value, permlane16_swap
// returns {v with its odd rows replaced by the even rows, v with its even rows replaced by the odd
// rows} and permlane32_swap the same for the two 32-lane halves, so the two results always hold a lane's
// own value and its xor-16 (xor-32) partner's — in the same order on both partners.
struct LanePair {
    float a, b;
};
__device__ __forceinline__ LanePair lanes_xor16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return {__uint_as_float(r[0]), __uint_as_float(r[1])};
}
__device__ __forceinline__ LanePair lanes_xor32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return {__uint_as_float(r[0]), __uint_as_float(r[1])};
}
__device__ __forceinline__ float sum_xor16(float v) {
    const LanePair p = lanes_xor16(v);
    return p.a + p.b;
}
__device__ __forceinline__ float sum_xor32(float v) {
    const LanePair p = lanes_xor32(v);
    return p.a + p.b;
}
__device__ __forceinline__ float max_xor16(float v) {
    const LanePair p = lanes_xor16(v);
    return fmaxf(p.a, p.b);
}
__device__ __forceinline__ float max_xor32(float v) {
    const LanePair p = lanes_xor32(v);
    return fmaxf(p.a, p.b);
}

// sum over groups of `width` consecutive lanes (width a power of two <= 64); every lane of a group
// gets the same value (each step adds the same two operands on both partners)
template <int WIDTH>
__device__ __forceinline__ float group_sum(float v) {
    static_assert(WIDTH >= 1 && WIDTH <= 64 && (WIDTH & (WIDTH - 1)) == 0, "group width");
    if constexpr (WIDTH >= 2) v += dpp_f<kDppXor1>(v);
    if constexpr (WIDTH >= 4) v += dpp_f<kDppXor2>(v);
    if constexpr (WIDTH >= 8) v += dpp_f<kDppHalfMirror>(v);
    if constexpr (WIDTH >= 16) v += dpp_f<kDppMirror>(v);
    if constexpr (WIDTH >= 32) v = sum_xor16(v);
    if constexpr (WIDTH >= 64) v = sum_xor32(v);
    return v;
}

template <int WIDTH>
__device__ __forceinline__ float group_max(float v) {
    static_assert(WIDTH >= 1 && WIDTH <= 64 && (WIDTH & (WIDTH - 1)) == 0, "group width");
    if constexpr (WIDTH >= 2) v = fmaxf(v, dpp_f<kDppXor1>(v));
    if constexpr (WIDTH >= 4) v = fmaxf(v, dpp_f<kDppXor2>(v));
    if constexpr (WIDTH >= 8) v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
    if constexpr (WIDTH >= 16) v = fmaxf(v, dpp_f<kDppMirror>(v));
    if constexpr (WIDTH >= 32) v = max_xor16(v);
    if constexpr (WIDTH >= 64) v = max_xor32(v);
    return v;
}

// sum / max over the lanes congruent modulo STRIDE (the row groups of a wave that hold the same
// columns: lanes STRIDE, 2·STRIDE, … apart); STRIDE in {4, 8, 16, 32, 64}. The xor-16/32 steps stay on
// ds_bpermute here: in the attention tails (many independent values) the permlane swaps measured slower
// (C4 GQA-4 attention 38.2 -> 43.8 us), the LDS pipe overlapping its round trips better.
template <int STRIDE>
__device__ __forceinline__ float stride_sum(float v) {
    static_assert(STRIDE == 4 || STRIDE == 8 || STRIDE == 16 || STRIDE == 32 || STRIDE == 64, "stride");
    if constexpr (STRIDE <= 4) v += __shfl_xor(v, 4, kWave);
    if constexpr (STRIDE <= 8) v += dpp_f<kDppRor8>(v);
    if constexpr (STRIDE <= 16) v += __shfl_xor(v, 16, kWave);
    if constexpr (STRIDE <= 32) v += __shfl_xor(v, 32, kWave);
    return v;
}
template <int STRIDE>
__device__ __forceinline__ float stride_max(float v) {
    static_assert(STRIDE == 4 || STRIDE == 8 || STRIDE == 16 || STRIDE == 32 || STRIDE == 64, "stride");
    if constexpr (STRIDE <= 4) v = fmaxf(v, __shfl_xor(v, 4, kWave));
    if constexpr (STRIDE <= 8) v = fmaxf(v, dpp_f<kDppRor8>(v));
    if constexpr (STRIDE <= 16) v = fmaxf(v, __shfl_xor(v, 16, kWave));
    if constexpr (STRIDE <= 32) v = fmaxf(v, __shfl_xor(v, 32, kWave));
    return v;
}

__device__ __forceinline__ float wave_sum(float v) { return group_sum<64>(v); }
__device__ __forceinline__ float wave_max(float v) { return group_max<64>(v); }

// 16-byte loads. NT = non-temporal (streamed-once weights: MI355X_MICROARCH.md "nt-weights").
template <bool NT>
__device__ __forceinline__ u32x4 load16(const void* p) {
    if constexpr (NT) {
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    } else {
        return *reinterpret_cast<const u32x4*>(p);
    }
}

// element types of a 16-byte vector
template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
    static constexpr int N = 4;
    __device__ __forceinline__ static void unpack(const u32x4& v, float* o) {
        o[0] = __uint_as_float(v.x);
        o[1] = __uint_as_float(v.y);
        o[2] = __uint_as_float(v.z);
        o[3] = __uint_as_float(v.w);
    }
    __device__ __forceinline__ static u32x4 pack(const float* f) {
        return u32x4{__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3])};
    }
};
template <>
struct Vec16<__half> {
    static constexpr int N = 8;
    __device__ __forceinline__ static void unpack(const u32x4& v, float* o) {
        unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            __half2 h = *reinterpret_cast<const __half2*>(&w[i]);
            float2 f = __half22float2(h);
            o[2 * i] = f.x;
            o[2 * i + 1] = f.y;
        }
    }
    // inverse of unpack for values already representable in fp16 (exact)
    __device__ __forceinline__ static u32x4 pack(const float* f) {
        unsigned w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const __half2 h = __floats2half2_rn(f[2 * i], f[2 * i + 1]);
            w[i] = *reinterpret_cast<const unsigned*>(&h);
        }
        return u32x4{w[0], w[1], w[2], w[3]};
    }
};
template <>
struct Vec16<int8_t> {
    static constexpr int N = 16;
    __device__ __forceinline__ static void unpack(const u32x4& v, float* o) {
        unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int b = 0; b < 4; ++b) o[4 * i + b] = (float)(int)(int8_t)((w[i] >> (8 * b)) & 0xFFu);
        }
    }
};

template <typename T>
__device__ __forceinline__ float to_f32(T v);
template <>
__device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f32<__half>(__half v) { return __half2float(v); }
template <>
__device__ __forceinline__ float to_f32<int8_t>(int8_t v) { return (float)(int)v; }

template <typename T>
__device__ __forceinline__ T from_f32(float v);
template <>
__device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ __half from_f32<__half>(float v) { return __float2half_rn(v); }

// Orderable 64-bit argmax key: larger value wins; equal values -> lower index wins (std::max_element's
// first-max rule, source/op/argmax.cpp:11, whose scan is `if (*best < *it) best = it`). Key 0 is below
// every real key. Exactly that scan's result, including the values `<` does not order:
//   * -0.0 and +0.0 compare equal, so -0.0 is keyed as +0.0 (the earlier of the two wins);
//   * a NaN never displaces the current best (`best < NaN` is false): key 0, below every number;
//   * a NaN at index 0 is never displaced either (`NaN < x` is false): the all-ones key, above all.
__device__ __forceinline__ unsigned long long argmax_key(float v, unsigned idx) {
    if (v != v) return idx == 0 ? ~0ull : 0ull;
    unsigned u = __float_as_uint(v);
    u = u == 0x80000000u ? 0u : u;
    unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)ord << 32) | (unsigned long long)(0xFFFFFFFFu - idx);
}
__device__ __forceinline__ unsigned argmax_key_index(unsigned long long k) {
    return 0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull);
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        unsigned long long w = __shfl_xor(v, o, kWave);
        v = w > v ? w : v;
    }
    return v;
}

}  // namespace sli
