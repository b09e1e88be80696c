// memory.cpp — base::fatal, the CPU / HIP allocators, Buffer and Tensor of the drop-in C++ layer
// (reference: source/memory/{alloc,buffer,tensor}.cpp, include/base/base.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <new>
#include <numeric>

#include "tensor.h"

namespace base {
void fatal(const std::string& message, const char* file, int line) {
    std::cout << "file: " << file << " line: " << line << " - " << message << std::endl;
    std::exit(EXIT_FAILURE);
}
}  // namespace base

namespace mem {

namespace {
hipMemcpyKind to_hip(base::MemcpyKind k) {
    switch (k) {
        case base::MemcpyKind::kMemcpyCPU2CUDA: return hipMemcpyHostToDevice;
        case base::MemcpyKind::kMemcpyCUDA2CPU: return hipMemcpyDeviceToHost;
        case base::MemcpyKind::kMemcpyCUDA2CUDA: return hipMemcpyDeviceToDevice;
        default: return hipMemcpyHostToHost;
    }
}
}  // namespace

base::DeviceType DeviceAllocator::device_type() { return device_type_; }

void DeviceAllocator::memcpy(const void* src_ptr, void* dst_ptr, size_t byte_size, base::MemcpyKind kind) const {
    if (!src_ptr || !dst_ptr) LOG(" ERROR! Ptr is empty! ");
    if (byte_size == 0) return;
    if (kind == base::MemcpyKind::kMemcpyCPU2CPU) {
        std::memcpy(dst_ptr, src_ptr, byte_size);
        return;
    }
    if (hipMemcpy(dst_ptr, src_ptr, byte_size, to_hip(kind)) != hipSuccess) LOG(" ERROR! hipMemcpy failed ");
}

void DeviceAllocator::memset_zero(void* ptr, size_t byte_size) {
    if (!ptr) LOG(" ERROR! Ptr is Empty! ");
    if (device_type_ == base::DeviceType::kDeviceUnknown) LOG(" ERROR! Device Type Unknown! ");
    if (device_type_ == base::DeviceType::kDeviceCPU) {
        std::memset(ptr, 0, byte_size);
    } else if (hipMemset(ptr, 0, byte_size) != hipSuccess) {
        LOG(" ERROR! hipMemset failed ");
    }
}

CPUDeviceAllocator::CPUDeviceAllocator() : DeviceAllocator(base::DeviceType::kDeviceCPU) {}

void* CPUDeviceAllocator::allocate(size_t byte_size) const {
    if (!byte_size) return nullptr;
    return std::aligned_alloc(64, (byte_size + 63) / 64 * 64);
}

void CPUDeviceAllocator::release(void* ptr) const { std::free(ptr); }

// ---- HIP caching allocator: 512-byte granules below 1 MiB, 2 MiB granules above; a freed block is
// reused by any later request it covers with less than 2x waste (best fit), so model-lifetime tensors
// allocate once and per-call scratch recycles.
CUDADeviceAllocator::CUDADeviceAllocator() : DeviceAllocator(base::DeviceType::kDeviceCUDA) {}

CUDADeviceAllocator::~CUDADeviceAllocator() { release_cached_memory(); }

size_t CUDADeviceAllocator::round_up(size_t n) {
    const size_t g = n < (1u << 20) ? 512 : (2u << 20);
    return (n + g - 1) / g * g;
}

void* CUDADeviceAllocator::allocate(size_t byte_size) const {
    if (!byte_size) return nullptr;
    const size_t want = round_up(byte_size);
    std::lock_guard<std::mutex> lk(mu_);
    auto it = free_.lower_bound(want);
    if (it != free_.end() && it->first < 2 * want) {
        void* p = it->second;
        live_[p] = it->first;
        free_.erase(it);
        return p;
    }
    void* p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) {
        for (auto& kv : free_) (void)hipFree(kv.second);  // flush the cache and retry (alloc.cpp:118-131)
        free_.clear();
        (void)hipGetLastError();
        if (hipMalloc(&p, want) != hipSuccess) throw std::bad_alloc();
    }
    live_[p] = want;
    return p;
}

void CUDADeviceAllocator::release(void* ptr) const {
    if (!ptr) return;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = live_.find(ptr);
    if (it == live_.end()) return;  // not ours
    free_.emplace(it->second, ptr);
    live_.erase(it);
}

size_t CUDADeviceAllocator::cached_bytes() const {
    std::lock_guard<std::mutex> lk(mu_);
    size_t n = 0;
    for (auto& kv : free_) n += kv.first;
    return n;
}

void CUDADeviceAllocator::release_cached_memory() const {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : free_) (void)hipFree(kv.second);
    free_.clear();
}

std::shared_ptr<CPUDeviceAllocator> CPUDeviceAllocatorFactory::get_instance() {
    static std::shared_ptr<CPUDeviceAllocator> inst = std::make_shared<CPUDeviceAllocator>();
    return inst;
}

std::shared_ptr<CUDADeviceAllocator> CUDADeviceAllocatorFactory::get_instance() {
    static std::shared_ptr<CUDADeviceAllocator> inst = std::make_shared<CUDADeviceAllocator>();
    return inst;
}

// ---------------------------------------------------------------- Buffer (buffer.cpp)
Buffer::Buffer(size_t byte_size, std::shared_ptr<DeviceAllocator> allocator, void* ptr, bool use_external)
    : byte_size_(byte_size), ptr_(ptr), use_external_(use_external), allocator_(std::move(allocator)) {
    if (!ptr_ && allocator_) {
        device_type_ = allocator_->device_type();
        use_external_ = false;
        ptr_ = allocator_->allocate(byte_size_);
    }
}

Buffer::~Buffer() {
    if (!use_external_ && ptr_ && allocator_) allocator_->release(ptr_);
}

bool Buffer::allocate() {
    if (!allocator_ || byte_size_ == 0) return false;
    use_external_ = false;
    ptr_ = allocator_->allocate(byte_size_);
    return ptr_ != nullptr;
}

void Buffer::copy_from(const Buffer& other) const {
    if (!allocator_) LOG("Buffer::copy_from: no allocator");
    const size_t n = std::min(byte_size_, other.byte_size_);
    const bool src_dev = other.device_type_ == base::DeviceType::kDeviceCUDA;
    const bool dst_dev = device_type_ == base::DeviceType::kDeviceCUDA;
    const base::MemcpyKind k = src_dev ? (dst_dev ? base::MemcpyKind::kMemcpyCUDA2CUDA : base::MemcpyKind::kMemcpyCUDA2CPU)
                                       : (dst_dev ? base::MemcpyKind::kMemcpyCPU2CUDA : base::MemcpyKind::kMemcpyCPU2CPU);
    allocator_->memcpy(other.ptr_, ptr_, n, k);
}

void Buffer::copy_from(const Buffer* other) const { copy_from(*other); }
void* Buffer::ptr() { return ptr_; }
const void* Buffer::ptr() const { return ptr_; }
size_t Buffer::byte_size() const { return byte_size_; }
std::shared_ptr<DeviceAllocator> Buffer::allocator() const { return allocator_; }
base::DeviceType Buffer::device_type() const { return device_type_; }
void Buffer::set_device_type(base::DeviceType t) { device_type_ = t; }
bool Buffer::is_external() const { return use_external_; }

// ---------------------------------------------------------------- Tensor (tensor.cpp)
static size_t numel(const std::vector<int32_t>& d) {
    if (d.empty()) return 0;
    return std::accumulate(d.begin(), d.end(), (size_t)1, [](size_t a, int32_t b) { return a * (size_t)b; });
}

Tensor::Tensor(std::vector<int32_t> dims, bool need_alloc, std::shared_ptr<DeviceAllocator> alloc, void* ptr)
    : Tensor(std::move(dims), base::DataType::kFp32, need_alloc, std::move(alloc), ptr) {}

Tensor::Tensor(std::vector<int32_t> dims, base::DataType dtype, bool need_alloc, std::shared_ptr<DeviceAllocator> alloc,
               void* ptr)
    : dims_(std::move(dims)), dtype_(dtype) {
    size_ = numel(dims_);
    if (need_alloc && alloc)
        allocate(alloc);
    else
        init_buffer(alloc, need_alloc, ptr);
}

void Tensor::init_buffer(std::shared_ptr<DeviceAllocator> alloc, bool need_alloc, void* ptr) {
    if (!alloc && !need_alloc)
        buffer_ = std::make_shared<Buffer>(byte_size(), nullptr, ptr, true);
    else
        allocate(alloc, true);
}

bool Tensor::allocate(std::shared_ptr<DeviceAllocator> allocator, bool need_realloc) {
    if (!allocator) return false;
    if (buffer_ && byte_size() <= buffer_->byte_size() && !need_realloc) return true;
    buffer_ = std::make_shared<Buffer>(byte_size(), allocator, nullptr);
    if (!buffer_->ptr()) LOG("The memory allocated is a null pointer!");
    return true;
}

size_t Tensor::byte_size() const { return base::data_type_size(dtype_) * size_; }

base::DeviceType Tensor::device_type() const {
    return buffer_ ? buffer_->device_type() : base::DeviceType::kDeviceUnknown;
}

void Tensor::to_cpu() {
    if (!buffer_) LOG(" No buffer in Tensor! ");
    const auto t = device_type();
    if (t == base::DeviceType::kDeviceUnknown) LOG(" The device type of the tensor is unknown. ");
    if (t == base::DeviceType::kDeviceCPU) return;
    auto cpu = CPUDeviceAllocatorFactory::get_instance();
    auto nb = std::make_shared<Buffer>(byte_size(), cpu);
    cpu->memcpy(buffer_->ptr(), nb->ptr(), byte_size(), base::MemcpyKind::kMemcpyCUDA2CPU);
    buffer_ = nb;
}

void Tensor::to_cuda() {
    if (!buffer_) LOG(" No buffer in Tensor! ");
    const auto t = device_type();
    if (t == base::DeviceType::kDeviceUnknown) LOG(" The device type of the tensor is unknown. ");
    if (t == base::DeviceType::kDeviceCUDA) return;
    auto dev = CUDADeviceAllocatorFactory::get_instance();
    auto nb = std::make_shared<Buffer>(byte_size(), dev);
    dev->memcpy(buffer_->ptr(), nb->ptr(), byte_size(), base::MemcpyKind::kMemcpyCPU2CUDA);
    buffer_ = nb;
}

bool Tensor::is_empty() const { return size_ == 0 || !buffer_ || !buffer_->ptr(); }

void Tensor::reshape(const std::vector<int32_t>& dims) {
    const size_t n = numel(dims);
    if (buffer_ && n > size_) {
        auto nb = std::make_shared<Buffer>(n * base::data_type_size(dtype_), buffer_->allocator());
        nb->copy_from(buffer_.get());
        buffer_ = nb;
    }
    dims_ = dims;
    size_ = n;
}

std::shared_ptr<Buffer> Tensor::get_buffer() const { return buffer_; }
size_t Tensor::size() const { return size_; }
int32_t Tensor::dims_size() const { return (int32_t)dims_.size(); }

int32_t Tensor::get_dim(int32_t idx) const {
    if (idx < 0 || idx >= dims_size()) LOG("idx is wrong!");
    return dims_[idx];
}

const std::vector<int32_t>& Tensor::dims() const { return dims_; }

bool Tensor::assign(std::shared_ptr<Buffer> buffer) {
    if (!buffer) return false;
    if (buffer_ && buffer_->device_type() != buffer->device_type()) return false;
    if (byte_size() > buffer->byte_size()) return false;
    buffer_ = std::move(buffer);
    return true;
}

void Tensor::reset(const std::vector<int32_t>& dims) {
    dims_ = dims;
    size_ = numel(dims);
    buffer_ = nullptr;
}

std::vector<size_t> Tensor::strides() const {
    std::vector<size_t> s(dims_.size(), 1);
    for (int i = (int)dims_.size() - 2; i >= 0; --i) s[i] = s[i + 1] * (size_t)dims_[i + 1];
    return s;
}

void Tensor::set_device_type(base::DeviceType t) const {
    if (buffer_) buffer_->set_device_type(t);
}

Tensor Tensor::clone() const {
    Tensor t = *this;
    t.buffer_ = std::make_shared<Buffer>(byte_size(), buffer_->allocator());
    t.buffer_->copy_from(buffer_.get());
    return t;
}

std::pair<Tensor, Tensor> slice_KV_cache(int32_t layer_idx, int32_t pos, int32_t max_seq_len, int32_t dim,
                                         const Tensor& key_cache, const Tensor& value_cache) {
    const size_t off = ((size_t)layer_idx * max_seq_len + pos) * dim;
    Tensor k({dim}, false, nullptr, const_cast<float*>(key_cache.ptr<float>()) + off);
    Tensor v({dim}, false, nullptr, const_cast<float*>(value_cache.ptr<float>()) + off);
    k.set_device_type(key_cache.device_type());
    v.set_device_type(value_cache.device_type());
    return {k, v};
}

}  // namespace mem
