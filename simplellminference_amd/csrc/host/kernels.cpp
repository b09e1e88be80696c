// kernels.cpp — the reference's kernel launchers (include/kernel/cuda/*.cuh signatures) over the
// libsli.so C ABI: unpack mem::Tensor (pointer, dims, element type) and call sli_*; a non-zero status
// becomes LOG(...) exactly where the reference would LOG (e.g. matmul_kernel.cu:44-46).
#include <hip/hip_runtime.h>

#include <string>

#include "kernels.h"
#include "sli.h"

namespace kernel {

namespace {
void check(int rc, const char* what) {
    if (rc != SLI_OK) LOG(std::string(what) + ": " + sli_status_str(rc) + " (" + sli_last_error() + ")");
}
int sli_dtype(const mem::Tensor& t) {
    switch (t.data_type()) {
        case base::DataType::kFp16: return SLI_DT_F16;
        case base::DataType::kInt8: return SLI_DT_I8;
        default: return SLI_DT_F32;
    }
}
float* f32(const mem::Tensor& t) { return const_cast<float*>(t.ptr<float>()); }
}  // namespace

void matmul_kernel_cuda(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output, int32_t dim0,
                        int32_t dim1, float scale) {
    if (input.get_dim(0) != dim1) LOG("Tensor with Wrong Dim!");
    if (weight.data_type() == base::DataType::kInt8) LOG("int8 weights need row scales: use the model-level API");
    check(sli_matmul(f32(input), weight.ptr<void>(), sli_dtype(weight), nullptr, f32(output), dim0, dim1, scale, nullptr),
          "matmul_kernel_cuda");
}

void rmsnorm_kernel_cuda(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output,
                         int32_t hidden_dim_size, float eps) {
    check(sli_rmsnorm(f32(input), weight.ptr<float>(), f32(output), hidden_dim_size, eps, nullptr), "rmsnorm_kernel_cuda");
}

void rope_cache_cal_cuda(int head_size, int max_seq_len, const mem::Tensor sin_cache, const mem::Tensor cos_cache,
                         float rope_theta) {
    check(sli_rope_cache(head_size, max_seq_len, f32(sin_cache), f32(cos_cache), rope_theta, nullptr),
          "rope_cache_cal_cuda");
}

// pos_now is a host tensor in the reference (model.cpp:258-262); a device tensor is read on the device.
void rope_kernel_cuda(const mem::Tensor& input_q, const mem::Tensor& input_k, const mem::Tensor& pos_now,
                      const mem::Tensor& sin_cache, const mem::Tensor& cos_cache, int32_t hidden_dim_size,
                      int32_t head_dim) {
    const bool dev_pos = pos_now.device_type() == base::DeviceType::kDeviceCUDA;
    const int32_t pos = dev_pos ? 0 : *pos_now.ptr<int32_t>();
    check(sli_rope(f32(input_q), f32(input_k), pos, dev_pos ? pos_now.ptr<int32_t>() : nullptr, sin_cache.ptr<float>(),
                   cos_cache.ptr<float>(), hidden_dim_size, (int32_t)input_k.size(), head_dim, nullptr),
          "rope_kernel_cuda");
}

size_t mha_workspace_floats(int32_t max_seq_len, int32_t num_attention_heads, int32_t head_dim) {
    return (sli_mha_workspace_bytes(max_seq_len, num_attention_heads, head_dim) + 3) / 4;
}

void mha_kernel_cuda_ws(const mem::Tensor& query, const mem::Tensor& key_cache, const mem::Tensor& value_cache,
                        const mem::Tensor& mha_out, int32_t layer_index, int32_t pos, int32_t max_seq_len,
                        int32_t head_dim, int32_t num_attention_heads, int32_t num_kv_heads, const mem::Tensor& ws) {
    check(sli_mha(query.ptr<float>(), key_cache.ptr<void>(), value_cache.ptr<void>(), sli_dtype(key_cache), f32(mha_out),
                  layer_index, pos, max_seq_len, head_dim, num_attention_heads, num_kv_heads,
                  const_cast<float*>(ws.ptr<float>()), ws.byte_size(), nullptr),
          "mha_kernel_cuda");
}

// Reference signature: `score` ({head_dim, max_seq_len} scratch, model.cpp:279) doubles as the
// split-context workspace when large enough; otherwise a per-call allocator scratch is used.
void mha_kernel_cuda(const mem::Tensor& query, const mem::Tensor& score, const mem::Tensor& key_cache,
                     const mem::Tensor& value_cache, const mem::Tensor& mha_out, int32_t layer_index, int32_t pos,
                     int32_t max_seq_len, int32_t head_dim, int32_t hidden_dim, int32_t kv_hidden_dim,
                     int32_t att_kv_head_group, int32_t num_attention_heads, base::DeviceType device_type) {
    (void)hidden_dim;
    (void)att_kv_head_group;
    (void)device_type;
    const int32_t kvh = kv_hidden_dim / head_dim;
    const size_t need = sli_mha_workspace_bytes(max_seq_len, num_attention_heads, head_dim);
    if (score.byte_size() >= need && score.device_type() == base::DeviceType::kDeviceCUDA) {
        mha_kernel_cuda_ws(query, key_cache, value_cache, mha_out, layer_index, pos, max_seq_len, head_dim,
                           num_attention_heads, kvh, score);
        return;
    }
    // A score buffer too small for the split partials (more than ~16384/(hd+4) heads): a per-call scratch
    // from the device allocator, returned to its pool when this call returns. Every kernel-level op runs on
    // the default stream, so a later reuse of the block is ordered behind this launch (the reference's own
    // per-call RMSNorm scratch follows the same pattern, rms_kernel.cu:48-51).
    mem::Tensor ws({(int32_t)((need + 3) / 4)}, true, mem::CUDADeviceAllocatorFactory::get_instance());
    mha_kernel_cuda_ws(query, key_cache, value_cache, mha_out, layer_index, pos, max_seq_len, head_dim,
                       num_attention_heads, kvh, ws);
}

void swiglu_kernel_cuda(const mem::Tensor& up, const mem::Tensor& gate, const mem::Tensor& output,
                        int32_t intermediate_size) {
    check(sli_swiglu(up.ptr<float>(), gate.ptr<float>(), f32(output), intermediate_size, nullptr), "swiglu_kernel_cuda");
}

void add_kernel_cuda(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& output, int32_t dim_size) {
    check(sli_add(input1.ptr<float>(), input2.ptr<float>(), f32(output), dim_size, nullptr), "add_kernel_cuda");
}

// The token is a host tensor in the reference (emb_kernel.cu:15); a device token is read on the device.
void emb_kernel_cuda(const mem::Tensor& input, const mem::Tensor& weight, const mem::Tensor& output, int32_t vocab_size,
                     int32_t hidden_dim_size) {
    const bool dev_tok = input.device_type() == base::DeviceType::kDeviceCUDA;
    const int32_t token = dev_tok ? 0 : *input.ptr<int32_t>();
    if (!dev_tok && (token < 0 || token >= vocab_size)) LOG("Token index is greater than vocab size.");
    check(sli_embedding(token, dev_tok ? input.ptr<int32_t>() : nullptr, weight.ptr<void>(), sli_dtype(weight), nullptr,
                        f32(output), vocab_size, hidden_dim_size, nullptr),
          "emb_kernel_cuda");
}

}  // namespace kernel
