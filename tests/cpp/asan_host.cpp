// asan_host.cpp — the CPU-only parts of the C++ drop-in layer (csrc/host/*.cpp) under AddressSanitizer +
// UBSan (oracle/Makefile `asan`, tools/asan_check.sh). No device call is made: every path here is the reference's
// CPU device (source/memory/{alloc,buffer,tensor}.cpp semantics), the flat-file reader (source/model/
// weight_loader.cpp + model.cpp:204-245) and the CPU kernel stubs (their LOG-exit, run in mode "stub").
//
//   asan_host            run every check, print "asan_host: ok"
//   asan_host stub       call one CPU kernel stub (exits 1 through the reference's LOG, as a layer on kDeviceCPU)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unistd.h>
#include <vector>

#include "cpu_kernels.h"
#include "tensor.h"
#include "weight_loader.h"

#define EXPECT(c)                                                                   \
    do {                                                                            \
        if (!(c)) {                                                                 \
            std::fprintf(stderr, "asan_host: %s:%d: %s failed\n", __FILE__, __LINE__, #c); \
            std::exit(2);                                                           \
        }                                                                           \
    } while (0)

static void allocator_and_buffer() {
    auto cpu = mem::CPUDeviceAllocatorFactory::get_instance();
    EXPECT(cpu->device_type() == base::DeviceType::kDeviceCPU);
    for (size_t n : {1ul, 3ul, 63ul, 64ul, 65ul, 4097ul}) {  // rounded to 64-byte multiples by the allocator
        void* p = cpu->allocate(n);
        EXPECT(p != nullptr);
        std::memset(p, 0x5a, n);
        cpu->memset_zero(p, n);
        EXPECT(static_cast<unsigned char*>(p)[n - 1] == 0);
        cpu->release(p);
    }
    EXPECT(cpu->allocate(0) == nullptr);
    mem::Buffer a(256, cpu), b(256, cpu);
    EXPECT(a.ptr() && b.ptr() && !a.is_external());
    std::memset(a.ptr(), 7, 256);
    b.copy_from(a);
    b.copy_from(&a);
    EXPECT(static_cast<unsigned char*>(b.ptr())[255] == 7);
    std::vector<float> host(16, 1.5f);
    mem::Buffer ext(sizeof(float) * host.size(), nullptr, host.data(), true);  // never freed (buffer.cpp:14-21)
    EXPECT(ext.is_external() && ext.ptr() == host.data());
}

static void tensors() {
    auto cpu = mem::CPUDeviceAllocatorFactory::get_instance();
    mem::Tensor t({3, 5, 7}, true, cpu);
    EXPECT(t.size() == 105 && t.byte_size() == 420 && t.dims_size() == 3 && t.get_dim(2) == 7);
    const auto st = t.strides();
    EXPECT(st.size() == 3 && st[0] == 35 && st[1] == 7 && st[2] == 1);
    for (int i = 0; i < 105; ++i) t.index<float>(i) = (float)i;
    EXPECT(*t.ptr<float>(104) == 104.0f);
    mem::Tensor c = t.clone();
    EXPECT(c.ptr<float>() != t.ptr<float>() && c.index<float>(50) == 50.0f);
    t.reshape({105});
    EXPECT(t.dims_size() == 1 && t.index<float>(104) == 104.0f);
    t.reshape({210});  // grows: reallocates (tensor.cpp reshape semantics)
    EXPECT(t.size() == 210);
    t.index<float>(209) = 1.0f;
    mem::Tensor h({8}, base::DataType::kFp16, true, cpu);
    EXPECT(h.byte_size() == 16);
    mem::Tensor q({9}, base::DataType::kInt8, true, cpu);
    EXPECT(q.byte_size() == 9);
    q.ptr<int8_t>()[8] = -3;
    auto buf = std::make_shared<mem::Buffer>(4 * 105, cpu);
    mem::Tensor v({105});
    EXPECT(v.is_empty() && !v.assign(buf));  // an external (device-unknown) buffer refuses a CPU one (tensor.cpp:150-154)
    v.reset({105});                          // no buffer: any large-enough buffer is taken
    EXPECT(v.assign(buf) && !v.is_empty() && v.index<float>(104) == v.index<float>(104));
    v.reset({4, 4});
    EXPECT(v.size() == 16);
    std::vector<float> ext(12, 2.0f);
    mem::Tensor e({3, 4}, false, nullptr, ext.data());  // a view on caller memory
    EXPECT(e.index<float>(11) == 2.0f);
}

static void flat_file() {
    char path[] = "/tmp/asan_host_flat_XXXXXX";
    const int fd = mkstemp(path);
    EXPECT(fd >= 0);
    std::vector<float> w(1000);
    for (size_t i = 0; i < w.size(); ++i) w[i] = 0.25f * (float)i;
    EXPECT(write(fd, w.data(), w.size() * 4) == (ssize_t)(w.size() * 4));
    close(fd);
    {
        model::RawModelDataFp32 raw;
        EXPECT(raw.open_file(path));
        EXPECT(raw.file_size == 4000);
        EXPECT(*static_cast<const float*>(raw.weight(999)) == 0.25f * 999.0f);
    }  // unmapped and closed here
    model::RawModelDataFp32 missing;
    EXPECT(!missing.open_file("/nonexistent/asan_host_weights.bin"));
    unlink(path);
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "stub") {
        auto cpu = mem::CPUDeviceAllocatorFactory::get_instance();
        mem::Tensor a({4}, true, cpu), b({4}, true, cpu), o({4}, true, cpu);
        kernel::add_kernel_cpu(a, b, o, 4);  // weak stub: LOG -> exit(1)
        return 0;
    }
    allocator_and_buffer();
    tensors();
    flat_file();
    std::printf("asan_host: ok\n");
    return 0;
}
