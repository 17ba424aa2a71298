// Compile-only probe: does a K-deep rotation of granule polls keep K loads in
// flight (s_waitcnt vmcnt(K-1) before each check) or does the compiler drain
// them (vmcnt(0))?
//   hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only -DVAR=n tools/probe_poll.hip -o /tmp/pp.s
#include <hip/hip_runtime.h>

#include <cstdint>

#ifndef VAR
#define VAR 0
#endif
constexpr int K = 4;

__device__ __forceinline__ uint64_t ld(const uint64_t* p) {
#if VAR == 0
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    uint64_t v;
    asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
#endif
}

extern "C" __global__ void probe_poll(const uint64_t* g, uint64_t* out, uint32_t want, int64_t ngr) {
    const int lane = threadIdx.x & 63;
    const int64_t x = lane < ngr ? lane : ngr - 1;        // branch-free window index
    uint64_t q[K];
    uint64_t pf = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        if (i > 0) __builtin_amdgcn_s_sleep(8);
        q[i] = ld(g + x);
    }
    bool fin = false;
    while (!fin) {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            if (fin) continue;
#if VAR == 1
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K - 1) : "memory");
#endif
            if ((uint32_t)(pf >> 32) != want) pf = q[i];
            if (__all((uint32_t)(pf >> 32) == want)) {
                fin = true;
                continue;
            }
            __builtin_amdgcn_s_sleep(1);
            q[i] = ld(g + x);
        }
    }
    out[threadIdx.x] = pf;
}
