// persistent_launch.h — host entry to the persistent step kernel (persistent.hip), kept in its own
// translation unit: its instantiations dominate compile time and it is opt-in (SLI_STEP_MODE=persistent).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace sli {
struct StepParams;
bool persistent_supported(int w_dtype, int kv_dtype, int head_dim, int group);
int persistent_launch(int w_dtype, int kv_dtype, int head_dim, int group, const StepParams* dparams, int grid,
                      size_t lds_bytes, unsigned* bar, int p_begin, int p_end, int finalize, hipStream_t s);
}  // namespace sli
