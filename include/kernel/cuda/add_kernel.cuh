// add_kernel.cuh — the name source/op/*.cpp includes for kernel::add_kernel_cuda; the HIP launchers live in
// libsli.so (kernels.h, csrc/host/kernels.cpp). INTEGRATION.md, Level 2.
#pragma once
#include "../kernels.h"
