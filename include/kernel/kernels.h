// kernels.h — the reference's kernel launcher signatures (include/kernel/cuda/*.cuh), implemented over
// the libsli.so C ABI (csrc/host/kernels.cpp). A reference maintainer replaces source/kernel/cuda/*.cu
// with these.
#pragma once
#include "tensor.h"

namespace kernel {

void matmul_kernel_cuda(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output, int32_t dim0,
                        int32_t dim1, float scale = 1.0f);                          // matmul_kernel.cuh:6-7
void rmsnorm_kernel_cuda(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output,
                         int32_t hidden_dim_size, float eps);                       // rms_kernel.cuh:6-7
void rope_cache_cal_cuda(int head_size, int max_seq_len, const mem::Tensor sin_cache, const mem::Tensor cos_cache,
                         float rope_theta);                                         // rope_kernel.cuh:5-6
void rope_kernel_cuda(const mem::Tensor& input_q, const mem::Tensor& input_k, const mem::Tensor& pos_now,
                      const mem::Tensor& sin_cache, const mem::Tensor& cos_cache, int32_t hidden_dim_size,
                      int32_t head_dim);                                            // rope_kernel.cuh:7-8
void mha_kernel_cuda(const mem::Tensor& query, const mem::Tensor& score, const mem::Tensor& key_cache,
                     const mem::Tensor& value_cache, const mem::Tensor& mha_out, int32_t layer_index, int32_t pos,
                     int32_t max_seq_len, int32_t head_dim, int32_t hidden_dim, int32_t kv_hidden_dim,
                     int32_t att_kv_head_group, int32_t num_attention_heads,
                     base::DeviceType device_type);                                 // mha_kernel.cuh:6-21
void swiglu_kernel_cuda(const mem::Tensor& up, const mem::Tensor& gate, const mem::Tensor& output,
                        int32_t intermediate_size);                                 // swiglu_kernel.cuh:5
void add_kernel_cuda(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& output,
                     int32_t dim_size);                                             // add_kernel.cuh:6
void emb_kernel_cuda(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output,
                     int32_t vocab_size, int32_t hidden_dim_size);                  // emb_kernel.cuh:6-7

// The mha launcher needs split-context scratch; this variant takes it explicitly (the op layer owns it).
void mha_kernel_cuda_ws(const mem::Tensor& query, const mem::Tensor& key_cache, const mem::Tensor& value_cache,
                        const mem::Tensor& mha_out, int32_t layer_index, int32_t pos, int32_t max_seq_len,
                        int32_t head_dim, int32_t num_attention_heads, int32_t num_kv_heads, const mem::Tensor& workspace);
size_t mha_workspace_floats(int32_t max_seq_len, int32_t num_attention_heads, int32_t head_dim);

}  // namespace kernel
