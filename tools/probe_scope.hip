// Which cache-policy bits the HIP scoped atomics get on gfx950 (hand-off
// granule loads / stores).  Compile only:
//   hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only tools/probe_scope.hip -o /tmp/probe_scope.s
#include <hip/hip_runtime.h>

#include <cstdint>

extern "C" __global__ void probe_scope(uint64_t* p, uint64_t* q, uint64_t v) {
    const uint64_t a = __hip_atomic_load(p + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t b = __hip_atomic_load(p + 64 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t c = __hip_atomic_load(p + 128 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + threadIdx.x, a + b + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 64 + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(q + 128 + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
