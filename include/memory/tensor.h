// tensor.h — drop-in for the reference's include/memory/tensor.h: int32 dims over a shared Buffer,
// fp32 by default (reference semantics), with an element-type extension for fp16 / int8 weights.
#pragma once
#include <memory>
#include <numeric>  // std::accumulate, which the reference's source/op/layer.cpp:187 gets from here (tensor.h:7)
#include <utility>
#include <vector>

#include "buffer.h"

namespace mem {

// ABI tag: this Tensor carries an element type (dtype_) after the reference's fields, so it is 56 bytes where
// the reference's include/memory/tensor.h Tensor is 48. The tag is part of every mangled name that takes a
// Tensor (mem::Tensor[abi:sli_dtype]), so an object compiled against the REFERENCE's memory headers cannot
// link against libsli.so's kernel::*_cuda launchers (an undefined-symbol error) instead of silently passing a
// 48-byte object to code that reads 56. INTEGRATION.md Level 2: compile against this include/.
class [[gnu::abi_tag("sli_dtype")]] Tensor {
public:
    Tensor() = default;
    explicit Tensor(std::vector<int32_t> dims, bool need_alloc = false, std::shared_ptr<DeviceAllocator> alloc = nullptr,
                    void* ptr = nullptr);
    Tensor(std::vector<int32_t> dims, base::DataType dtype, bool need_alloc, std::shared_ptr<DeviceAllocator> alloc,
           void* ptr = nullptr);

    void to_cpu();
    void to_cuda();
    bool is_empty() const;
    void init_buffer(std::shared_ptr<DeviceAllocator> alloc, bool need_alloc, void* ptr);
    bool allocate(std::shared_ptr<DeviceAllocator> allocator, bool need_realloc = false);
    bool assign(std::shared_ptr<Buffer> buffer);
    void reset(const std::vector<int32_t>& dims);
    void reshape(const std::vector<int32_t>& dims);
    Tensor clone() const;

    template <typename T> T* ptr();
    template <typename T> const T* ptr() const;
    template <typename T> T* ptr(int64_t index);
    template <typename T> const T* ptr(int64_t index) const;
    template <typename T> T& index(int64_t offset);
    template <typename T> const T& index(int64_t offset) const;

    std::shared_ptr<Buffer> get_buffer() const;
    size_t size() const;
    size_t byte_size() const;
    int32_t dims_size() const;
    int32_t get_dim(int32_t idx) const;
    const std::vector<int32_t>& dims() const;
    std::vector<size_t> strides() const;
    void set_device_type(base::DeviceType device_type) const;
    base::DeviceType device_type() const;
    base::DataType data_type() const { return dtype_; }

private:
    size_t size_ = 0;
    std::vector<int32_t> dims_;
    std::shared_ptr<Buffer> buffer_;
    base::DataType dtype_ = base::DataType::kFp32;
};

template <typename T>
T* Tensor::ptr() {
    return buffer_ ? reinterpret_cast<T*>(buffer_->ptr()) : nullptr;
}
template <typename T>
const T* Tensor::ptr() const {
    return buffer_ ? reinterpret_cast<const T*>(buffer_->ptr()) : nullptr;
}
template <typename T>
T* Tensor::ptr(int64_t index) {
    if (!buffer_ || !buffer_->ptr()) LOG("ERROR Get Ptr!");
    return reinterpret_cast<T*>(buffer_->ptr()) + index;
}
template <typename T>
const T* Tensor::ptr(int64_t index) const {
    if (!buffer_ || !buffer_->ptr()) LOG("ERROR Get Ptr!");
    return reinterpret_cast<const T*>(buffer_->ptr()) + index;
}
template <typename T>
T& Tensor::index(int64_t offset) {
    if (offset < 0 || offset >= (int64_t)size_) LOG("ERROR Index!");
    return reinterpret_cast<T*>(buffer_->ptr())[offset];
}
template <typename T>
const T& Tensor::index(int64_t offset) const {
    if (offset < 0 || offset >= (int64_t)size_) LOG("ERROR Index!");
    return reinterpret_cast<const T*>(buffer_->ptr())[offset];
}

// {dim}-element views of the K and V cache rows [layer][pos] (reference tensor.cpp:199-212).
std::pair<Tensor, Tensor> slice_KV_cache(int32_t layer_idx, int32_t pos, int32_t max_seq_len, int32_t dim,
                                         const Tensor& key_cache, const Tensor& value_cache);

}  // namespace mem
