// ops.h — the reference's concrete operators (include/op/{matmul,rmsnorm,rope,mha,swiglu,add,
// embedding,argmax}.h), same constructors and slots. Device dispatch: kDeviceCUDA (== HIP here) runs
// the libsli.so kernels; any other device LOG-exits with "Device Type ERROR!" as the reference's
// forward() does (e.g. source/op/matmul.cpp:19-25). The CPU backend is not part of the product.
#pragma once
#include "layer.h"

namespace op {

class MatmulLayer : public LayerParam {  // matmul.h:7-16; inputs {x}, weight {W [dim0][dim1]}, output {y}
public:
    explicit MatmulLayer(base::DeviceType device_type, int32_t dim0, int32_t dim1);
    using Layer::forward;  // keep the 1-5 input overloads visible on the concrete type
    void forward() override;

private:
    int32_t dim0_ = 0;
    int32_t dim1_ = 0;
};

class RmsNormLayer : public LayerParam {  // rmsnorm.h:7-16
public:
    explicit RmsNormLayer(base::DeviceType device_type, int32_t hidden_dim_size, float eps);
    using Layer::forward;  // keep the 1-5 input overloads visible on the concrete type
    void forward() override;

private:
    int32_t hidden_dim_size_ = 0;
    float eps_ = 0.0f;
};

// rope.h:7-15: forward(q, k, pos, sin_cache, cos_cache) — cos arrives in output slot 0 (rope.cpp:12-16).
class RoPELayer : public Layer {
public:
    explicit RoPELayer(base::DeviceType device_type, int32_t hidden_dim_size, int32_t head_dim);
    using Layer::forward;  // keep the 1-5 input overloads visible on the concrete type
    void forward() override;

private:
    int32_t hidden_dim_size_ = 0;
    int32_t head_dim_ = 0;
};

// mha.h:7-32: forward(q, score, key_cache, value_cache, out) at (layer, pos) set by the setters.
class MultiHeadAttention : public Layer {
public:
    explicit MultiHeadAttention(base::DeviceType device_type, int32_t max_seq_len, int32_t head_dim,
                                int32_t num_attention_heads, int32_t num_key_value_heads);
    void set_pos(int32_t pos);
    void set_layer_index(int32_t index);
    using Layer::forward;  // keep the 1-5 input overloads visible on the concrete type
    void forward() override;

private:
    int32_t layer_index_ = 0;
    int32_t pos_ = 0;
    int32_t max_seq_len_ = 0;
    int32_t head_dim_ = 0;
    int32_t hidden_dim_ = 0;         // num_attention_heads * head_dim (mha.cpp:21, the reference's members)
    int32_t kv_hidden_dim_ = 0;      // num_key_value_heads * head_dim (mha.cpp:22)
    int32_t num_attention_heads_ = 0;
    int32_t num_key_value_heads_ = 0;
    int32_t att_kv_head_group_ = 0;  // num_attention_heads / num_key_value_heads (mha.cpp:23)
    mem::Tensor workspace_;  // split-context partials (replaces the reference's score scratch)
};

class SwigluLayer : public Layer {  // swiglu.h:6-13: forward(up, gate, out) = sigmoid(gate) * up
public:
    explicit SwigluLayer(base::DeviceType device_type, int32_t intermediate_size);
    using Layer::forward;  // keep the 1-5 input overloads visible on the concrete type
    void forward() override;

private:
    int32_t intermediate_size_ = 0;
};

class VecAddLayer : public Layer {  // add.h:7-14
public:
    explicit VecAddLayer(base::DeviceType device_type, int32_t dim_size);
    using Layer::forward;  // keep the 1-5 input overloads visible on the concrete type
    void forward() override;

private:
    int32_t dim_size_ = 0;
};

class EmbeddingLayer : public LayerParam {  // embedding.h:7-15; input {token}, weight {table [V][D]}
public:
    explicit EmbeddingLayer(base::DeviceType device_type, int32_t vocab_size, int32_t hidden_dim_size);
    using Layer::forward;  // keep the 1-5 input overloads visible on the concrete type
    void forward() override;

private:
    int32_t vocab_size_ = 0;
    int32_t hidden_dim_size_ = 0;
};

// argmax.h:7-13: first index of the maximum. The reference runs it on the host only (argmax.cpp:13-14);
// here a device logits tensor is reduced on the device and the index lands in `input_idx`.
class argmaxLayer {
public:
    explicit argmaxLayer(base::DeviceType device_type, int32_t hidden_dim_size);
    void forward(const mem::Tensor& logits, const mem::Tensor& input_idx);

private:
    base::DeviceType device_type_ = base::DeviceType::kDeviceUnknown;
    int32_t hidden_dim_size_ = 0;
};

}  // namespace op
