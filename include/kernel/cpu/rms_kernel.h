// rms_kernel.h — the name source/op/*.cpp includes for the CPU kernel declarations (cpu_kernels.h).
// INTEGRATION.md, Level 2.
#pragma once
#include "../cpu_kernels.h"
