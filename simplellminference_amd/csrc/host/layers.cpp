// layers.cpp — the drop-in operator framework and concrete operators (reference: source/op/*.cpp).
// kDeviceCUDA (== HIP) dispatches to kernel::*_cuda (kernels.cpp -> libsli.so C ABI); any other device
// LOG-exits with the reference's message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>

#include "kernels.h"
#include "ops.h"
#include "sli.h"

namespace op {

namespace {
bool on_hip(base::DeviceType t) { return t == base::DeviceType::kDeviceCUDA; }
}  // namespace

// ---------------------------------------------------------------- BaseLayer / Layer / LayerParam
BaseLayer::BaseLayer(base::DeviceType device_type, LayerType layer_type, std::string layer_name)
    : layer_name_(std::move(layer_name)), layer_type_(layer_type), device_type_(device_type) {}
LayerType BaseLayer::layer_type() const { return layer_type_; }
const std::string& BaseLayer::get_layer_name() const { return layer_name_; }
void BaseLayer::set_layer_name(const std::string& n) { layer_name_ = n; }
base::DeviceType BaseLayer::device_type() const { return device_type_; }
void BaseLayer::set_device_type(base::DeviceType t) { device_type_ = t; }

Layer::Layer(base::DeviceType device_type, LayerType layer_type, std::string layer_name)
    : BaseLayer(device_type, layer_type, std::move(layer_name)) {}

void Layer::set_input(int32_t idx, const mem::Tensor& t) { inputs_.at(idx) = t; }
void Layer::set_output(int32_t idx, const mem::Tensor& t) { outputs_.at(idx) = t; }
const mem::Tensor& Layer::get_input(int32_t idx) const { return inputs_.at(idx); }
const mem::Tensor& Layer::get_output(int32_t idx) const { return outputs_.at(idx); }
mem::Tensor& Layer::get_input(int32_t idx) { return inputs_.at(idx); }
mem::Tensor& Layer::get_output(int32_t idx) { return outputs_.at(idx); }
size_t Layer::input_size() const { return inputs_.size(); }
size_t Layer::output_size() const { return outputs_.size(); }
void Layer::reset_input_size(size_t n) { inputs_.resize(n); }
void Layer::reset_output_size(size_t n) { outputs_.resize(n); }
void Layer::set_weight(int32_t, const mem::Tensor&) { LOG("Function not Implementation!"); }
void Layer::set_weight(int32_t, const std::vector<int32_t>&, const void*, base::DeviceType) {
    LOG("Function not Implementation!");
}
void Layer::forward() { LOG("Function not Implementation!"); }

void Layer::to_cuda() {
    for (auto& t : inputs_)
        if (!t.is_empty()) t.to_cuda();
    for (auto& t : outputs_)
        if (!t.is_empty()) t.to_cuda();
}

void Layer::forward(const mem::Tensor& i1, const mem::Tensor& o1) {
    set_input(0, i1);
    set_output(0, o1);
    forward();
}
void Layer::forward(const mem::Tensor& i1, const mem::Tensor& i2, const mem::Tensor& o1) {
    set_input(0, i1);
    set_input(1, i2);
    set_output(0, o1);
    forward();
}
void Layer::forward(const mem::Tensor& i1, const mem::Tensor& i2, const mem::Tensor& i3, const mem::Tensor& o1) {
    set_input(0, i1);
    set_input(1, i2);
    set_input(2, i3);
    set_output(0, o1);
    forward();
}
void Layer::forward(const mem::Tensor& i1, const mem::Tensor& i2, const mem::Tensor& i3, const mem::Tensor& i4,
                    const mem::Tensor& o1) {
    set_input(0, i1);
    set_input(1, i2);
    set_input(2, i3);
    set_input(3, i4);
    set_output(0, o1);
    forward();
}
void Layer::forward(const mem::Tensor& i1, const mem::Tensor& i2, const mem::Tensor& i3, const mem::Tensor& i4,
                    const mem::Tensor& i5, const mem::Tensor& o1) {
    set_input(0, i1);
    set_input(1, i2);
    set_input(2, i3);
    set_input(3, i4);
    set_input(4, i5);
    set_output(0, o1);
    forward();
}

LayerParam::LayerParam(base::DeviceType device_type, LayerType layer_type, std::string layer_name)
    : Layer(device_type, layer_type, std::move(layer_name)) {}
size_t LayerParam::weight_size() const { return weights_.size(); }
void LayerParam::reset_weight_size(size_t n) { weights_.resize(n); }
mem::Tensor& LayerParam::get_weight(int32_t idx) { return weights_.at(idx); }
const mem::Tensor& LayerParam::get_weight(int32_t idx) const { return weights_.at(idx); }

void LayerParam::to_cuda() {
    Layer::to_cuda();
    for (auto& w : weights_)
        if (!w.is_empty()) w.to_cuda();
}

void LayerParam::set_weight(int32_t idx, const mem::Tensor& weight) {
    if (weight.is_empty()) return;
    if (weight.device_type() != device_type_) LOG("Device not the same!");
    weights_.at(idx) = weight;
}

// Non-owning fp32 view of caller memory (layer.cpp:183-196); to_cuda() later copies it to the device.
void LayerParam::set_weight(int32_t idx, const std::vector<int32_t>& dims, const void* weight_ptr,
                            base::DeviceType device_type) {
    if (weight_ptr == nullptr) LOG("Ptr is empty!");
    const size_t bytes = std::accumulate(dims.begin(), dims.end(), sizeof(float),
                                         [](size_t a, int32_t b) { return a * (size_t)b; });
    auto buf = std::make_shared<mem::Buffer>(bytes, nullptr, const_cast<void*>(weight_ptr), true);
    if (device_type != base::DeviceType::kDeviceUnknown) buf->set_device_type(device_type);
    mem::Tensor w(dims);
    w.set_device_type(device_type);  // the placeholder buffer must carry the same tag for assign()
    w.assign(buf);
    weights_.at(idx) = w;
}

// ---------------------------------------------------------------- concrete operators
MatmulLayer::MatmulLayer(base::DeviceType d, int32_t dim0, int32_t dim1)
    : LayerParam(d, LayerType::kLayerMatmul, "Matmul"), dim0_(dim0), dim1_(dim1) {
    reset_input_size(1);
    reset_weight_size(1);
    reset_output_size(1);
}
void MatmulLayer::forward() {
    if (!on_hip(device_type_)) LOG("Device Type ERROR!");
    kernel::matmul_kernel_cuda(get_input(0), get_weight(0), get_output(0), dim0_, dim1_);
}

RmsNormLayer::RmsNormLayer(base::DeviceType d, int32_t hidden_dim_size, float eps)
    : LayerParam(d, LayerType::kLayerRMSNorm, "RMSNorm"), hidden_dim_size_(hidden_dim_size), eps_(eps) {
    reset_input_size(1);
    reset_output_size(1);
    reset_weight_size(1);
}
void RmsNormLayer::forward() {
    if (!on_hip(device_type_)) LOG("Device Type ERROR!");
    kernel::rmsnorm_kernel_cuda(get_input(0), get_weight(0), get_output(0), hidden_dim_size_, eps_);
}

RoPELayer::RoPELayer(base::DeviceType d, int32_t hidden_dim_size, int32_t head_dim)
    : Layer(d, LayerType::kLayerRoPe, "RoPE"), hidden_dim_size_(hidden_dim_size), head_dim_(head_dim) {
    reset_input_size(4);
    reset_output_size(1);
}
void RoPELayer::forward() {
    if (!on_hip(device_type_)) LOG("Device Type ERROR!");
    kernel::rope_kernel_cuda(get_input(0), get_input(1), get_input(2), get_input(3), get_output(0), hidden_dim_size_,
                             head_dim_);
}

MultiHeadAttention::MultiHeadAttention(base::DeviceType d, int32_t max_seq_len, int32_t head_dim,
                                       int32_t num_attention_heads, int32_t num_key_value_heads)
    : Layer(d, LayerType::kLayerMHA, "MultiHeadAttention"),
      max_seq_len_(max_seq_len),
      head_dim_(head_dim),
      num_attention_heads_(num_attention_heads),
      num_key_value_heads_(num_key_value_heads) {
    reset_input_size(4);
    reset_output_size(1);
    hidden_dim_ = num_attention_heads * head_dim;
    kv_hidden_dim_ = num_key_value_heads * head_dim;
    att_kv_head_group_ = num_key_value_heads > 0 ? num_attention_heads / num_key_value_heads : 0;
}
void MultiHeadAttention::set_pos(int32_t pos) { pos_ = pos; }
void MultiHeadAttention::set_layer_index(int32_t index) { layer_index_ = index; }
void MultiHeadAttention::forward() {
    if (!on_hip(device_type_)) LOG("Device Type ERROR!");
    if (workspace_.is_empty()) {
        const size_t n = kernel::mha_workspace_floats(max_seq_len_, num_attention_heads_, head_dim_);
        workspace_ = mem::Tensor({(int32_t)n}, true, mem::CUDADeviceAllocatorFactory::get_instance());
    }
    kernel::mha_kernel_cuda_ws(get_input(0), get_input(2), get_input(3), get_output(0), layer_index_, pos_,
                               max_seq_len_, head_dim_, num_attention_heads_, num_key_value_heads_, workspace_);
}

SwigluLayer::SwigluLayer(base::DeviceType d, int32_t intermediate_size)
    : Layer(d, LayerType::kLayerSwiGLU, "SwiGLU"), intermediate_size_(intermediate_size) {
    reset_input_size(2);
    reset_output_size(1);
}
void SwigluLayer::forward() {
    if (!on_hip(device_type_)) LOG("Device Type ERROR!");
    kernel::swiglu_kernel_cuda(get_input(0), get_input(1), get_output(0), intermediate_size_);
}

VecAddLayer::VecAddLayer(base::DeviceType d, int32_t dim_size) : Layer(d, LayerType::kLayerAdd, "Add"), dim_size_(dim_size) {
    reset_input_size(2);
    reset_output_size(1);
}
void VecAddLayer::forward() {
    if (!on_hip(device_type_)) LOG("Device Type ERROR!");
    kernel::add_kernel_cuda(get_input(0), get_input(1), get_output(0), dim_size_);
}

EmbeddingLayer::EmbeddingLayer(base::DeviceType d, int32_t vocab_size, int32_t hidden_dim_size)
    : LayerParam(d, LayerType::kLayerEmbedding, "Embedding"), vocab_size_(vocab_size), hidden_dim_size_(hidden_dim_size) {
    reset_weight_size(1);
    reset_input_size(1);
    reset_output_size(1);
}
void EmbeddingLayer::forward() {
    if (!on_hip(device_type_)) LOG("Device Type ERROR!");
    kernel::emb_kernel_cuda(get_input(0), get_weight(0), get_output(0), vocab_size_, hidden_dim_size_);
}

argmaxLayer::argmaxLayer(base::DeviceType d, int32_t hidden_dim_size) : device_type_(d), hidden_dim_size_(hidden_dim_size) {}

void argmaxLayer::forward(const mem::Tensor& logits, const mem::Tensor& input_idx) {
    int32_t* dst = const_cast<int32_t*>(input_idx.ptr<int32_t>());
    if (logits.device_type() == base::DeviceType::kDeviceCUDA) {
        // per-call device scratch from the allocator pool (the copy below synchronises before it returns)
        mem::Tensor scratch({1}, base::DataType::kFp32, true, mem::CUDADeviceAllocatorFactory::get_instance());
        int32_t* d = scratch.ptr<int32_t>();
        if (sli_argmax(logits.ptr<float>(), hidden_dim_size_, d, nullptr) != SLI_OK) LOG(sli_last_error());
        if (input_idx.device_type() == base::DeviceType::kDeviceCUDA) {
            if (hipMemcpy(dst, d, 4, hipMemcpyDeviceToDevice) != hipSuccess) LOG("hipMemcpy");
        } else if (hipMemcpy(dst, d, 4, hipMemcpyDeviceToHost) != hipSuccess) {
            LOG("hipMemcpy");
        }
        return;
    }
    if (device_type_ != base::DeviceType::kDeviceCPU && device_type_ != base::DeviceType::kDeviceCUDA)
        LOG("wrong device!\n");
    const float* p = logits.ptr<float>();  // host logits: first max (std::max_element, argmax.cpp:11)
    *dst = (int32_t)std::distance(p, std::max_element(p, p + hidden_dim_size_));
}

}  // namespace op
