// cpu_kernels.h — the reference's CPU kernel signatures (include/kernel/cpu/*.h), declared so the
// reference's unchanged source/op/*.cpp compile against this tree (Level 2). libsli.so has
// no CPU backend: it defines these as WEAK symbols that stop with LOG (the reference's error path) when a
// layer is run on DeviceType::kDeviceCPU; a maintainer who keeps the reference's source/kernel/cpu/*.cpp
// links those, and their strong definitions take precedence.
#pragma once
#include "tensor.h"

namespace kernel {

void add_kernel_cpu(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& output,
                    int32_t dim_size);                                              // add_kernel.h
void emb_kernel_cpu(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output,
                    int32_t vocab_size, int32_t hidden_dim_size);                   // emb_kernel.h
void matmul_kernel_cpu(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output, int32_t dim0,
                       int32_t dim1, float scale = 1.0f);                           // matmul_kernel.h
void mha_kernel_cpu(const mem::Tensor& query, const mem::Tensor& score, const mem::Tensor& key_cache,
                    const mem::Tensor& value_cache, const mem::Tensor& mha_out, int32_t layer_index, int32_t pos,
                    int32_t max_seq_len, int32_t head_dim, int32_t hidden_dim, int32_t kv_hidden_dim,
                    int32_t att_kv_head_group, int32_t num_attention_heads,
                    base::DeviceType device_type);                                  // mha_kernel.h
void rmsnorm_kernel_cpu(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output,
                        int32_t hidden_dim_size, float eps);                        // rms_kernel.h
void rope_cache_cal(int head_size, int max_seq_len, const mem::Tensor sin_cache, const mem::Tensor cos_cache,
                    float rope_theta);                                              // rope_kernel.h
void rope_kernel_cpu(const mem::Tensor& input_q, const mem::Tensor& input_k, const mem::Tensor& pos_now,
                     const mem::Tensor& sin_cache, const mem::Tensor& cos_cache, int32_t hidden_dim_size,
                     int32_t head_dim);                                             // rope_kernel.h
void swiglu_kernel_cpu(const mem::Tensor& up, const mem::Tensor& gate, const mem::Tensor& output,
                       int32_t intermediate_size);                                  // swiglu_kernel.h

}  // namespace kernel
