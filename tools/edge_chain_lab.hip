// edge_chain_lab.hip — the dependency edges of a C2 TP-8 rank layer inside ONE persistent launch, with no GEMV
// arithmetic (a feasibility probe for VERDICT r5 item 1: a whole TP-8 rank layer as one launch).
//
// Llama-2-7B at TP 8, one rank (source/model/model.cpp:50-129 sharded as DESIGN.md §6): per layer
//   E1  x (4096)  -> every CU          (RMSNorm + q/k/v input; after the previous layer's down + exchange)
//   E2  q, k, v (1536, 6 values per CU) -> the 64 attention CUs (head h = cu / 16 reads its 3 x 128 values)
//   E3a attention partials (m, l, o[128]) of 16 splits per head -> one merging CU per head
//   E3b merged attention output (512, from 4 CUs) -> every CU (wo input)
//   E4  x1 (4096)  -> every CU          (gate/up input; after wo + exchange)
//   E5  act (1376) -> every CU          (down input)
// Every edge: producers store their values as 8-byte {value, tag} granules with one sc1 store each (no drain, no
// flag: MI355X_MICROARCH.md granule rows), consumers sweep the granules with sc1 loads (all 512 threads of the CU,
// flat), re-read the ones whose tag is not yet this edge's, and write the values into LDS. Tags are unique per
// (launch, layer, edge), so one granule array per edge is reused layer after layer: every edge is all-to-all, so a
// CU cannot overwrite a granule before every reader of its previous value has moved past it.
//
// Optional weight traffic beside the edges (-w): each CU streams its real per-op byte share (q/k/v 48 KB, K/V 16 KB,
// wo 16 KB, gate/up 88 KB, down 44 KB) into registers right after the previous op, as the persistent layer would,
// and consumes it (a checksum) before publishing the op's output.
//
//   edge_chain_lab [-w] [-L layers] [-r reps]
// prints µs per layer (launch time / layers) and the per-edge stamps of one CU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            printf("%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);                  \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int kWG = 256, kT = 512;
constexpr int kD = 4096, kQKV = 1536, kHD = 128, kH = 4, kSplits = 16, kIl = 1376, kPart = kHD + 2;
constexpr unsigned kSpinMax = 1u << 16;  // sweep passes before a wait gives up (error flag; later waits then skip)

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Args {
    u32x2 *g_x, *g_qkv, *g_part, *g_att, *g_x1, *g_act;
    const u32x4* w;      // weight pool (streamed, -w)
    size_t w_per_cu;     // 16-byte vectors per CU per layer
    int layers, weights;
    unsigned epoch;
    unsigned* err;
    unsigned long long* stamps;  // [kWG][layers][8]
    float* sink;
};

__device__ __forceinline__ void put(u32x2* g, int i, float v, unsigned tag) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(v), tag}, rs, 8u * i, 0, 16 /* sc1 */);
}

// gather n granules g[i0 .. i0+n) with tag into dst[0 .. n) (LDS); all threads of the workgroup
__shared__ int g_dead;  // a wait of this workgroup gave up: every later one returns at once (the grid drains)

__device__ __forceinline__ void gather(const u32x2* g, int i0, int n, unsigned tag, float* dst, unsigned* err) {
    if (g_dead) return;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x2*>(g), 0, 0x7fffffff, 0x00020000);
    constexpr int kPer = 8;  // granules per thread per pass (n <= kT * kPer)
    unsigned todo = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j)
        if ((int)threadIdx.x + j * kT < n) todo |= 1u << j;
    for (unsigned pass = 0;; ++pass) {
        u32x2 v[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j)
            if (todo & (1u << j)) v[j] = __builtin_amdgcn_raw_buffer_load_b64(rs, 8u * (i0 + threadIdx.x + j * kT), 0, 16);
#pragma unroll
        for (int j = 0; j < kPer; ++j)
            if ((todo & (1u << j)) && v[j].y == tag) {
                dst[threadIdx.x + j * kT] = __uint_as_float(v[j].x);
                todo &= ~(1u << j);
            }
        if (__syncthreads_or(todo != 0) == 0) break;
        if (pass > kSpinMax) {
            if (threadIdx.x == 0) {
                atomicOr(err, 1u);
                g_dead = 1;
            }
            __syncthreads();
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// this CU's share of an op's weights, issued into registers (nt) before the op's input edge and consumed (a checksum)
// after it, as the persistent layer would hold them: n <= 12 * kT 16-byte vectors
struct WRegs {
    u32x4 a[12];
    int n;
};
__device__ __forceinline__ void issue(WRegs& r, const u32x4* w, int n) {
    r.n = n;
#pragma unroll
    for (int j = 0; j < 12; ++j)
        if ((int)threadIdx.x + j * kT < n) r.a[j] = __builtin_nontemporal_load(w + threadIdx.x + j * kT);
}
__device__ __forceinline__ float consume(const WRegs& r) {
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < 12; ++j)
        if ((int)threadIdx.x + j * kT < r.n) acc += __uint_as_float(r.a[j].x & 0x3fffffffu);
    return acc;
}

__global__ void __launch_bounds__(kT) chain(Args a) {
    __shared__ float xs[kD];
    __shared__ float att[kH * kHD];
    const int cu = blockIdx.x, t = threadIdx.x;
    if (t == 0) g_dead = 0;
    __syncthreads();
    float chk = 0.0f;
    // byte shares per op (16-byte vectors per CU): q/k/v 48 KB, K/V 16 KB, wo 16 KB, gate/up 88 KB, down 44 KB
    const int n_qkv = 3072, n_kv = 1024, n_wo = 1024, n_gu = 5632, n_dn = 2816;
    for (int l = 0; l < a.layers; ++l) {
        const u32x4* wb = a.w + ((size_t)l * kWG + cu) * a.w_per_cu;  // every layer's bytes distinct: HBM, not MALL
        const unsigned tb = (a.epoch * 64u + (unsigned)l) * 8u;
        unsigned long long* st = a.stamps + ((size_t)cu * a.layers + l) * 8;
        // E1: x
        WRegs wr;
        if (a.weights) issue(wr, wb, n_qkv);
        gather(a.g_x, 0, kD, tb + 1, xs, a.err);
        if (a.weights) chk += consume(wr);
        if (t == 0) st[0] = __builtin_amdgcn_s_memrealtime();
        // q/k/v: 6 values per CU
        if (t < 6) put(a.g_qkv, cu * 6 + t, xs[(cu * 6 + t) % kD] + chk * 0.0f, tb + 2);
        // attention CUs: head h = cu / 16, split s = cu % 16; read q, k, v of the head (3 x 128)
        if (cu < kH * kSplits) {
            const int h = cu / kSplits, s = cu % kSplits;
            if (a.weights) issue(wr, wb + n_qkv, n_kv);
            gather(a.g_qkv, 0 * 512 + h * kHD, kHD, tb + 2, xs, a.err);
            gather(a.g_qkv, 1 * 512 + h * kHD, kHD, tb + 2, xs + kHD, a.err);
            gather(a.g_qkv, 2 * 512 + h * kHD, kHD, tb + 2, xs + 2 * kHD, a.err);
            if (a.weights) chk += consume(wr);
            if (t == 0) st[1] = __builtin_amdgcn_s_memrealtime();
            if (t < kPart) put(a.g_part, (h * kSplits + s) * kPart + t, xs[t % (3 * kHD)], tb + 3);
            if (s == 0) {  // the head's merging CU
                gather(a.g_part, h * kSplits * kPart, kSplits * kPart, tb + 3, xs, a.err);
                if (t < kHD) {
                    float o = 0.0f;
                    for (int j = 0; j < kSplits; ++j) o += xs[j * kPart + t];
                    put(a.g_att, h * kHD + t, o, tb + 4);
                }
            }
        }
        if (a.weights) issue(wr, wb + n_qkv + n_kv, n_wo);
        gather(a.g_att, 0, kH * kHD, tb + 4, att, a.err);
        if (a.weights) chk += consume(wr);
        if (t == 0) st[2] = __builtin_amdgcn_s_memrealtime();
        // wo -> x1: 16 rows per CU
        if (t < 16) put(a.g_x1, cu * 16 + t, att[(cu * 16 + t) % (kH * kHD)], tb + 5);
        if (a.weights) issue(wr, wb + n_qkv + n_kv + n_wo, n_gu);
        gather(a.g_x1, 0, kD, tb + 5, xs, a.err);
        if (a.weights) chk += consume(wr);
        if (t == 0) st[3] = __builtin_amdgcn_s_memrealtime();
        // gate/up -> act: 5.375 values per CU
        {
            const int a0 = cu * kIl / kWG, a1 = (cu + 1) * kIl / kWG;
            if (t < a1 - a0) put(a.g_act, a0 + t, xs[a0 + t], tb + 6);
        }
        if (a.weights) issue(wr, wb + n_qkv + n_kv + n_wo + n_gu, n_dn);
        gather(a.g_act, 0, kIl, tb + 6, xs, a.err);
        if (a.weights) chk += consume(wr);
        if (t == 0) st[4] = __builtin_amdgcn_s_memrealtime();
        // down -> x (next layer's E1): 16 rows per CU
        if (t < 16) put(a.g_x, cu * 16 + t, xs[(cu * 16 + t) % kIl], tb + 8 + 1);
    }
    if (chk == 12345.0f) a.sink[cu] = chk;
}

// the epoch's first x (tag of layer 0's E1), written before the launch
__global__ void seed_x(u32x2* g, unsigned tag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < kD) g[i] = u32x2{__float_as_uint(1.0f), tag};
}

int main(int argc, char** argv) {
    int layers = 32, reps = 20, weights = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-w")) weights = 1;
        if (!strcmp(argv[i], "-L") && i + 1 < argc) layers = atoi(argv[++i]);
        if (!strcmp(argv[i], "-r") && i + 1 < argc) reps = atoi(argv[++i]);
    }
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    if (p.multiProcessorCount < kWG) {
        printf("needs %d CUs (one persistent workgroup each), device has %d\n", kWG, p.multiProcessorCount);
        return 1;
    }
    Args a{};
    auto alloc = [](size_t n) {
        void* q;
        CK(hipMalloc(&q, n));
        CK(hipMemset(q, 0, n));
        return q;
    };
    a.g_x = (u32x2*)alloc(8 * kD);
    a.g_qkv = (u32x2*)alloc(8 * kQKV);
    a.g_part = (u32x2*)alloc(8 * kH * kSplits * kPart);
    a.g_att = (u32x2*)alloc(8 * kH * kHD);
    a.g_x1 = (u32x2*)alloc(8 * kD);
    a.g_act = (u32x2*)alloc(8 * kIl);
    a.w_per_cu = 3072 + 1024 + 1024 + 5632 + 2816;
    a.w = (const u32x4*)alloc(16 * a.w_per_cu * kWG * (size_t)layers);
    a.err = (unsigned*)alloc(4);
    a.stamps = (unsigned long long*)alloc(8 * 8 * (size_t)kWG * layers);
    a.sink = (float*)alloc(4 * kWG);
    a.layers = layers;
    a.weights = weights;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms(reps);
    for (int r = 0; r <= reps; ++r) {
        a.epoch = (unsigned)(r + 1);
        hipLaunchKernelGGL(seed_x, dim3(kD / 256), dim3(256), 0, s, a.g_x, (a.epoch * 64u) * 8u + 1);
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(chain, dim3(kWG), dim3(kT), 0, s, a);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        if (r > 0) CK(hipEventElapsedTime(&ms[r - 1], e0, e1));
    }
    unsigned err = 0;
    CK(hipMemcpy(&err, a.err, 4, hipMemcpyDeviceToHost));
    std::sort(ms.begin(), ms.end());
    const double med = ms[reps / 2] * 1e3 / layers;
    std::vector<unsigned long long> st(8 * (size_t)kWG * layers);
    CK(hipMemcpy(st.data(), a.stamps, st.size() * 8, hipMemcpyDeviceToHost));
    // per-edge spans of CU 0 (an attention and merging CU) and CU 200, median over layers 1..L-1, in us (100 MHz clock)
    auto span = [&](int cu, int e0_, int e1_) {
        std::vector<double> v;
        for (int l = 1; l < layers; ++l) {
            const unsigned long long* q = &st[((size_t)cu * layers + l) * 8];
            const unsigned long long* qp = &st[((size_t)cu * layers + l - 1) * 8];
            const unsigned long long a0 = e0_ < 0 ? qp[4] : q[e0_];
            if (q[e1_] && a0) v.push_back((double)(q[e1_] - a0) / 100.0);
        }
        std::sort(v.begin(), v.end());
        return v.empty() ? -1.0 : v[v.size() / 2];
    };
    printf("edge chain%s: %d layers, median launch %.1f us = %.2f us per layer (err %u)\n", weights ? " + weights" : "",
           layers, ms[reps / 2] * 1e3, med, err);
    for (int cu : {0, 200}) {
        printf("  CU %3d: E1 x %.2f | E2 qkv %.2f | E3 attn %.2f | E4 x1 %.2f | E5 act %.2f us\n", cu, span(cu, -1, 0),
               cu < kH * kSplits ? span(cu, 0, 1) : -1.0, cu < kH * kSplits ? span(cu, 1, 2) : span(cu, 0, 2),
               span(cu, 2, 3), span(cu, 3, 4));
    }
    return err ? 2 : 0;
}
