// layer.h — drop-in for the reference's operator framework (include/op/layer.h:8-150): LayerType,
// BaseLayer (pure virtual), Layer (input/output slots + 1-5 input forward overloads) and LayerParam
// (weights; set_weight wraps a non-owning view; to_cuda uploads through the HIP allocator).
#pragma once
#include <string>
#include <vector>

#include "tensor.h"

namespace op {

enum class LayerType : uint8_t {
    kLayerUnknown = 0,
    kLayerLinear = 1,
    kLayerEncode = 2,
    kLayerEmbedding = 3,
    kLayerRMSNorm = 4,
    kLayerMatmul = 5,
    kLayerRoPe = 6,
    kLayerMHA = 7,
    kLayerSoftmax = 8,
    kLayerAdd = 9,
    kLayerSwiGLU = 10,
};

class BaseLayer {
public:
    explicit BaseLayer(base::DeviceType device_type, LayerType layer_type, std::string layer_name = "");
    virtual ~BaseLayer() = default;

    LayerType layer_type() const;
    const std::string& get_layer_name() const;
    void set_layer_name(const std::string& layer_name);
    base::DeviceType device_type() const;
    void set_device_type(base::DeviceType device_type);

    virtual void forward() = 0;
    virtual void forward(const mem::Tensor& input1, const mem::Tensor& output1) = 0;
    virtual void forward(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& output1) = 0;
    virtual void forward(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& input3,
                         const mem::Tensor& output1) = 0;
    virtual void forward(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& input3,
                         const mem::Tensor& input4, const mem::Tensor& output1) = 0;
    virtual void forward(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& input3,
                         const mem::Tensor& input4, const mem::Tensor& input5, const mem::Tensor& output1) = 0;

    virtual void set_input(int32_t idx, const mem::Tensor& input) = 0;
    virtual void set_output(int32_t idx, const mem::Tensor& output) = 0;
    virtual size_t input_size() const = 0;
    virtual size_t output_size() const = 0;
    virtual mem::Tensor& get_input(int32_t idx) = 0;
    virtual mem::Tensor& get_output(int32_t idx) = 0;
    virtual const mem::Tensor& get_input(int32_t idx) const = 0;
    virtual const mem::Tensor& get_output(int32_t idx) const = 0;
    virtual void set_weight(int32_t idx, const mem::Tensor& weight) = 0;
    virtual void set_weight(int32_t idx, const std::vector<int32_t>& dims, const void* weight_ptr,
                            base::DeviceType device_type = base::DeviceType::kDeviceUnknown) = 0;

protected:
    std::string layer_name_;
    LayerType layer_type_ = LayerType::kLayerUnknown;
    base::DeviceType device_type_ = base::DeviceType::kDeviceUnknown;
};

class Layer : public BaseLayer {
public:
    explicit Layer(base::DeviceType device_type, LayerType layer_type, std::string layer_name = "");

    void set_input(int32_t idx, const mem::Tensor& input) override;
    void set_output(int32_t idx, const mem::Tensor& output) override;
    const mem::Tensor& get_input(int32_t idx) const override;
    const mem::Tensor& get_output(int32_t idx) const override;
    mem::Tensor& get_input(int32_t idx) override;
    mem::Tensor& get_output(int32_t idx) override;
    size_t input_size() const override;
    size_t output_size() const override;
    void reset_input_size(size_t size);
    void reset_output_size(size_t size);
    void set_weight(int32_t idx, const mem::Tensor& weight) override;
    void set_weight(int32_t idx, const std::vector<int32_t>& dims, const void* weight_ptr,
                    base::DeviceType device_type = base::DeviceType::kDeviceUnknown) override;
    virtual void to_cuda();

    void forward() override;
    void forward(const mem::Tensor& input1, const mem::Tensor& output1) override;
    void forward(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& output1) override;
    void forward(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& input3,
                 const mem::Tensor& output1) override;
    void forward(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& input3,
                 const mem::Tensor& input4, const mem::Tensor& output1) override;
    void forward(const mem::Tensor& input1, const mem::Tensor& input2, const mem::Tensor& input3,
                 const mem::Tensor& input4, const mem::Tensor& input5, const mem::Tensor& output1) override;

protected:
    std::vector<mem::Tensor> inputs_;
    std::vector<mem::Tensor> outputs_;
};

class LayerParam : public Layer {
public:
    explicit LayerParam(base::DeviceType device_type, LayerType layer_type, std::string layer_name = "");

    size_t weight_size() const;
    void reset_weight_size(size_t size);
    mem::Tensor& get_weight(int32_t idx);
    const mem::Tensor& get_weight(int32_t idx) const;
    void to_cuda() override;
    void set_weight(int32_t idx, const mem::Tensor& weight) override;
    void set_weight(int32_t idx, const std::vector<int32_t>& dims, const void* weight_ptr,
                    base::DeviceType device_type = base::DeviceType::kDeviceUnknown) override;

protected:
    std::vector<mem::Tensor> weights_;
};

}  // namespace op
