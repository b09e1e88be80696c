// weight_loader.h — drop-in for the reference's include/model/weight_loader.h: a read-only mmap of the
// headerless flat fp32 weight file (model.cpp:204-245), released on destruction.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace model {

struct RawModelData {
    virtual ~RawModelData();
    int32_t fd = -1;
    size_t file_size = 0;
    void* data = nullptr;
    void* weight_data = nullptr;
    virtual const void* weight(size_t offset) const = 0;
    bool open_file(const std::string& path);  // returns false on any failure (the caller LOGs)
};

struct RawModelDataFp32 : RawModelData {
    const void* weight(size_t offset) const override;  // offset in floats
};

}  // namespace model
