// buffer.h — drop-in for the reference's include/memory/buffer.h: an owning or external byte range
// with its allocator and device tag (external buffers are never freed, buffer.cpp:14-21).
#pragma once
#include <memory>

#include "alloc.h"

namespace mem {

class Buffer {
public:
    Buffer() = default;
    explicit Buffer(size_t byte_size, std::shared_ptr<DeviceAllocator> allocator = nullptr, void* ptr = nullptr,
                    bool use_external = false);
    Buffer(const Buffer&) = delete;
    Buffer& operator=(const Buffer&) = delete;
    virtual ~Buffer();

    bool allocate();
    void copy_from(const Buffer& buffer) const;
    void copy_from(const Buffer* buffer) const;
    void* ptr();
    const void* ptr() const;
    size_t byte_size() const;
    std::shared_ptr<DeviceAllocator> allocator() const;
    base::DeviceType device_type() const;
    void set_device_type(base::DeviceType device_type);
    bool is_external() const;

private:
    size_t byte_size_ = 0;
    void* ptr_ = nullptr;
    bool use_external_ = false;
    base::DeviceType device_type_ = base::DeviceType::kDeviceUnknown;
    std::shared_ptr<DeviceAllocator> allocator_;
};

}  // namespace mem
