"""simplellminference_amd — MI355X-native (gfx950) decode path of Boundwhd/SimpleLLMInference.

The compute lives in libsli.so (hand-written HIP kernels behind the C ABI in include/sli.h). This
package holds the thin Python mirror of the reference's operator and model interfaces:

    simplellminference_amd.ops    kernel::*_cuda launchers (matmul, rmsnorm, rope, mha, softmax, ...)
    simplellminference_amd.model  model::LlamaModel (init / forward / predict) over the fused step
    simplellminference_amd.build  in-tree hipcc build of libsli.so for gfx950

Importing the package does not load the HIP library; the first call does, and fails loudly if it
is missing — there is no CPU fallback.
"""
from ._lib import DT_F16, DT_F32, DT_I8, LIB_PATH, SliError, load  # noqa: F401

__all__ = ["load", "SliError", "LIB_PATH", "DT_F32", "DT_F16", "DT_I8"]
