// kfec_count.hpp -- the completion count of a counted launch (device code; included by the .hip files only).
//
// The queues' small sealed flushes and opener flushes (kfec_pipeline.cpp, at most kSealCountRows packets) wait for
// this count in coherent pinned host memory instead of the stream: every wave waits for its own stores, the
// workgroup meets at a barrier, and one lane makes a system-scope release and adds the workgroup in (the producer
// form of MI355X_MICROARCH.md's hand-off recipe, with the host as the consumer).  The host sees the rows once the
// last workgroup has counted itself, without the runtime's completion signal and stream wait.  Every thread of the
// workgroup must reach it (the kernels that call it have no early return).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kfec {

__device__ __forceinline__ void count_workgroup_done(uint32_t *done)
{
    if (!done) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace kfec
