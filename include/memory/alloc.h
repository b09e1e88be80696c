// alloc.h — drop-in for the reference's include/memory/alloc.h: CPU and device allocators behind the
// same DeviceAllocator interface and singleton factories. The device allocator is a HIP caching
// allocator (best-fit over freed blocks, split on reuse, cache flushed and retried on OOM), guarded by
// a mutex; the factories are thread-safe (the reference's are not, alloc.h:113-137).
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>

#include "base.h"

#define DataTypeSize 4  // bytes of the reference's only element type (alloc.h:12)

namespace mem {

class DeviceAllocator {
public:
    explicit DeviceAllocator(base::DeviceType device_type) : device_type_(device_type) {}
    virtual ~DeviceAllocator() = default;

    virtual base::DeviceType device_type();
    virtual void* allocate(size_t byte_size) const = 0;
    virtual void release(void* ptr) const = 0;

    void memcpy(const void* src_ptr, void* dst_ptr, size_t byte_size, base::MemcpyKind memcpy_kind) const;
    virtual void memset_zero(void* ptr, size_t byte_size);

private:
    base::DeviceType device_type_ = base::DeviceType::kDeviceUnknown;
};

class CPUDeviceAllocator : public DeviceAllocator {
public:
    CPUDeviceAllocator();
    void* allocate(size_t byte_size) const override;
    void release(void* ptr) const override;
};

// HIP device allocator (named for source compatibility with callers that use the CUDA name).
class CUDADeviceAllocator : public DeviceAllocator {
public:
    CUDADeviceAllocator();
    ~CUDADeviceAllocator() override;
    void* allocate(size_t byte_size) const override;
    void release(void* ptr) const override;
    size_t cached_bytes() const;
    void release_cached_memory() const;

private:
    static size_t round_up(size_t n);
    mutable std::mutex mu_;
    mutable std::multimap<size_t, void*> free_;        // size -> block (best fit)
    mutable std::unordered_map<void*, size_t> live_;  // block -> size
};

class CPUDeviceAllocatorFactory {
public:
    static std::shared_ptr<CPUDeviceAllocator> get_instance();
};

class CUDADeviceAllocatorFactory {
public:
    static std::shared_ptr<CUDADeviceAllocator> get_instance();
};

}  // namespace mem
