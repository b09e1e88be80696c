// base.h — drop-in for the reference's include/base/base.h (LOG macro, MemcpyKind, DeviceType).
// kDeviceCUDA keeps its value 2 so unchanged callers select this library's HIP backend; kDeviceHIP is
// an alias. DataType is an extension (the reference is fp32-only, include/memory/alloc.h:12).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace base {

// Prints "file: F line: L - msg" and exits with EXIT_FAILURE, as the reference's log_message
// (base.h:6-10) does.
[[noreturn]] void fatal(const std::string& message, const char* file, int line);

enum class MemcpyKind { kMemcpyCPU2CPU = 0, kMemcpyCPU2CUDA = 1, kMemcpyCUDA2CPU = 2, kMemcpyCUDA2CUDA = 3 };

enum class DeviceType { kDeviceUnknown = 0, kDeviceCPU = 1, kDeviceCUDA = 2, kDeviceHIP = 2 };

enum class DataType { kFp32 = 0, kFp16 = 1, kInt8 = 2 };

inline size_t data_type_size(DataType t) { return t == DataType::kFp32 ? 4 : t == DataType::kFp16 ? 2 : 1; }

}  // namespace base

#define LOG(message) ::base::fatal((message), __FILE__, __LINE__)
