// pt_flat_fast.hip — the flat path's kernel-argument-table kernel with a scene's flags baked
// in (FastTableMask, pt_trace.h): what a cold first frame runs while the scene's hipRTC kernel
// compiles ("cold start"). Its own translation unit because it is compiled like
// the hipRTC scene kernel (Makefile: 8 waves, the AMDGPU pressure trackers, camera fields in
// argument registers, plain threadIdx.x) rather than like the offline walks of pt_kernel.hip.
#include <hip/hip_runtime.h>

#define PT_WAVES 8
#define PT_CAM_KERNARG 0
#define PT_FRESH_TID 0
#include "pt_internal.h"
#include "pt_trace.h"

namespace pt {

template <bool kSpecular, bool kMask32>
__global__ __launch_bounds__(kBlock, PT_WAVES) void pt_flat_fast_kernel(TraceArgs A) {
    trace_body_flat<FastTableMask<kSpecular, kMask32>>(A);
}

void* flat_fast_kernel(bool specular, bool mask32) {
    if (specular)
        return mask32 ? (void*)&pt_flat_fast_kernel<true, true> : (void*)&pt_flat_fast_kernel<true, false>;
    return mask32 ? (void*)&pt_flat_fast_kernel<false, true> : (void*)&pt_flat_fast_kernel<false, false>;
}

}  // namespace pt
