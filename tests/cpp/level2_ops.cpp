// level2_ops.cpp — INTEGRATION.md Level 2: an operator-level client written the way the reference's
// source/op/*.cpp are (builder's own code, not reference source): it includes the kernel headers by the
// names those files include ("matmul_kernel.h" + "matmul_kernel.cuh", ...; -I include/kernel/cpu and
// -I include/kernel/cuda as the reference's build adds them), builds mem::Tensor operands, moves them
// to the device with to_cuda(), and calls each kernel::*_kernel_cuda launcher with the reference's
// signature. Inputs and outputs go to a file that tests/test_dropin_cpp.py checks against the oracle.
//
// usage: level2_ops <out.bin>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "add_kernel.cuh"
#include "add_kernel.h"
#include "emb_kernel.cuh"
#include "emb_kernel.h"
#include "matmul_kernel.cuh"
#include "matmul_kernel.h"
#include "mha_kernel.cuh"
#include "mha_kernel.h"
#include "rms_kernel.cuh"
#include "rms_kernel.h"
#include "rope_kernel.cuh"
#include "rope_kernel.h"
#include "swiglu_kernel.cuh"
#include "swiglu_kernel.h"

static std::ofstream g_out;

static void put(const std::string& name, const std::vector<float>& v) {
    const int32_t n = (int32_t)name.size(), m = (int32_t)v.size();
    g_out.write((const char*)&n, 4);
    g_out.write(name.data(), n);
    g_out.write((const char*)&m, 4);
    g_out.write((const char*)v.data(), 4 * v.size());
}

static unsigned g_seed = 12345u;
static float rnd() {  // deterministic, sign-symmetric, O(1)
    g_seed = g_seed * 1664525u + 1013904223u;
    return ((float)(g_seed >> 8) / 16777216.0f - 0.5f) * 2.0f;
}

// a device tensor filled from host values (the reference pattern: host tensor, then to_cuda)
static mem::Tensor dev(const std::vector<int32_t>& dims, const std::string& name, float scale = 1.0f) {
    mem::Tensor t(dims, true, mem::CPUDeviceAllocatorFactory::get_instance());
    std::vector<float> v(t.size());
    for (auto& f : v) f = rnd() * scale;
    for (size_t i = 0; i < v.size(); ++i) t.index<float>(i) = v[i];
    put(name, v);
    t.to_cuda();
    return t;
}

static mem::Tensor dev_out(const std::vector<int32_t>& dims) {
    return mem::Tensor(dims, true, mem::CUDADeviceAllocatorFactory::get_instance());
}

static void get(const std::string& name, const mem::Tensor& t) {
    std::vector<float> v(t.size());
    if (hipMemcpy(v.data(), t.ptr<float>(), 4 * v.size(), hipMemcpyDeviceToHost) != hipSuccess) LOG("hipMemcpy");
    put(name, v);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s out.bin\n", argv[0]);
        return 2;
    }
    g_out.open(argv[1], std::ios::binary);
    // matmul (matmul.cpp: kernel::matmul_kernel_cuda(input, weight, output, dim0, dim1))
    {
        auto x = dev({256}, "mm_x");
        auto w = dev({64, 256}, "mm_w", 0.0625f);
        auto y = dev_out({64});
        kernel::matmul_kernel_cuda(x, w, y, 64, 256);
        get("mm_y", y);
    }
    // rmsnorm (rmsnorm.cpp)
    {
        auto x = dev({256}, "rms_x");
        auto w = dev({256}, "rms_w");
        auto y = dev_out({256});
        kernel::rmsnorm_kernel_cuda(x, w, y, 256, 1e-5f);
        get("rms_y", y);
    }
    // RoPE table + apply (model.cpp:312-316, rope.cpp; the position is a host tensor, model.cpp:258-262)
    {
        auto sin_c = dev_out({16, 32}), cos_c = dev_out({16, 32});
        kernel::rope_cache_cal_cuda(64, 16, sin_c, cos_c, 10000.0f);
        get("rope_sin", sin_c);
        get("rope_cos", cos_c);
        auto q = dev({256}, "rope_q");
        auto k = dev({128}, "rope_k");
        mem::Tensor pos({1}, true, mem::CPUDeviceAllocatorFactory::get_instance());
        pos.index<int32_t>(0) = 5;
        kernel::rope_kernel_cuda(q, k, pos, sin_c, cos_c, 256, 64);
        get("rope_q_out", q);
        get("rope_k_out", k);
    }
    // decode attention (mha.cpp: score {head_dim, max_seq_len} scratch, model.cpp:279), GQA 4 / 2
    {
        const int L = 2, T = 16, H = 4, KVH = 2, hd = 64;
        auto q = dev({H * hd}, "mha_q");
        auto kc = dev({L, T, KVH * hd}, "mha_k");
        auto vc = dev({L, T, KVH * hd}, "mha_v");
        auto score = dev_out({hd, T});
        auto out = dev_out({H * hd});
        kernel::mha_kernel_cuda(q, score, kc, vc, out, 1, 9, T, hd, H * hd, KVH * hd, H / KVH, H,
                                base::DeviceType::kDeviceCUDA);
        get("mha_out", out);
    }
    // swiglu (swiglu.cpp: inputs (up, gate))
    {
        auto up = dev({768}, "sw_up");
        auto gate = dev({768}, "sw_gate", 4.0f);
        auto out = dev_out({768});
        kernel::swiglu_kernel_cuda(up, gate, out, 768);
        get("sw_out", out);
    }
    // residual add (add.cpp)
    {
        auto a = dev({256}, "add_a");
        auto b = dev({256}, "add_b");
        auto out = dev_out({256});
        kernel::add_kernel_cuda(a, b, out, 256);
        get("add_out", out);
    }
    // embedding (embedding.cpp: the token is a host tensor, emb_kernel.cu:15)
    {
        auto table = dev({512, 256}, "emb_table");
        mem::Tensor tok({1}, true, mem::CPUDeviceAllocatorFactory::get_instance());
        tok.index<int32_t>(0) = 17;
        auto out = dev_out({256});
        kernel::emb_kernel_cuda(tok, table, out, 512, 256);
        get("emb_out", out);
    }
    g_out.close();
    std::printf("level2 ok\n");
    return 0;
}
