// ubench_handoff.hip -- latency of one WG-stripe hand-off granule, in
// isolation and beside a store stream like the fill's.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_handoff tools/ubench_handoff.hip
//   tools/ubench_handoff            (run on the GPU box)
//
// Workgroup 0 wave 0 publishes granule n = {tag n+1, value} every ~2 us with
// one 8-byte store; workgroup 1 wave 0 polls it (one 8-byte load per poll)
// and records when it sees each tag.  s_memrealtime (100 MHz, one clock for
// the whole chip) stamps both sides.  Variants:
//   store  : sc1 (agent atomic store, the fill's form) | plain + release fence
//   poll   : s_sleep(1) between polls | back to back
//   stream : 16-byte nt stores into a 4 GB buffer (the fill's table stream)
//            from the other waves of both workgroups (3 each, like a fill
//            workgroup's compute waves) and every other CU (1), or from a
//            subset (2 producer's CU, 3 consumer's CU, 4 all but those two,
//            5 all but the producer's CU, 6 all but the consumer's CU)
//   throttle: streaming waves keep at most 4 / 8 / 16 stores in flight
// Reported: median / p90 of (seen - stored) over 2000 hand-offs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int NH = 2000;
typedef int v4i __attribute__((ext_vector_type(4)));

struct Args {
    uint64_t* gran;        // one granule
    uint64_t* t_store;     // [NH]
    uint64_t* t_seen;      // [NH]
    v4i* sink;             // stream target
    int64_t sink_n;        // int4 elements per streaming wave
    uint32_t* stop;
    int store_mode;        // 0 sc1, 1 plain + release
    int poll_sleep;        // 0 / 1
    int stream;            // 0 none, 1 every CU, 2 producer's CU only, 3 consumer's CU only, 4 all but those two
    int scalar_poll;       // 1: the consumer polls with s_load_dwordx2 glc (scalar cache path)
    int throttle;          // streaming waves keep at most this many stores in flight (0: no limit)
};

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(256) void handoff(Args a) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool prod = blockIdx.x == 0 && w == 0, cons = blockIdx.x == 1 && w == 0;
    if (prod) {
        for (int n = 0; n < NH; ++n) {
            const uint64_t t0 = now();
            while (now() - t0 < 200) __builtin_amdgcn_s_sleep(2);      // ~2 us apart
            const uint64_t g = ((uint64_t)(n + 1) << 32) | (uint32_t)n;
            uint64_t ts = 0;
            if (lane == 0) {
                if (a.store_mode == 0) {
                    ts = now();
                    __hip_atomic_store(a.gran, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    ts = now();
                    *(volatile uint64_t*)a.gran = g;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                a.t_store[n] = ts;
            }
        }
        if (lane == 0) __hip_atomic_store(a.stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (cons) {
        for (int n = 0; n < NH; ++n) {
            const uint64_t t0 = now();
            for (;;) {
                uint64_t g;
                if (a.scalar_poll)
                    asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(g) : "s"(a.gran) : "memory");
                else
                    g = __hip_atomic_load(a.gran, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(g >> 32) >= (uint32_t)(n + 1)) break;
                if (now() - t0 > 100000000) break;                  // 1 s watchdog
                if (a.poll_sleep) __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0) a.t_seen[n] = now();
        }
    } else if (a.stream == 1 || (a.stream == 2 && blockIdx.x == 0) || (a.stream == 3 && blockIdx.x == 1) ||
               (a.stream == 4 && blockIdx.x > 1) || (a.stream == 5 && blockIdx.x != 0) ||
               (a.stream == 6 && blockIdx.x != 1)) {
        // streaming waves: 16-byte nt stores, 1 KB per wave instruction, until told to stop
        const int64_t wid = (int64_t)blockIdx.x * 4 + w;   // (stream waves only)
        v4i* p = a.sink + wid * a.sink_n;
        const v4i v = v4i{lane, w, (int)blockIdx.x, 7};
        for (int64_t k = 0;; k += 64) {
            if (k + lane >= a.sink_n) k = 0;
            __builtin_nontemporal_store(v, p + k + lane);
            if (a.throttle == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if (a.throttle == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (a.throttle == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            if ((k & 4095) == 0 &&
                __hip_atomic_load(a.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                break;
        }
    }
}

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                               \
        }                                                                           \
    } while (0)

int main() {
    int ncu = 0;
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    Args a{};
    CHK(hipMalloc(&a.gran, 256));
    CHK(hipMalloc(&a.t_store, NH * 8));
    CHK(hipMalloc(&a.t_seen, NH * 8));
    CHK(hipMalloc(&a.stop, 256));
    const int64_t waves = (int64_t)ncu * 4;
    a.sink_n = ((int64_t)4 << 30) / 16 / waves;
    a.sink_n -= a.sink_n % 4096;
    CHK(hipMalloc(&a.sink, (size_t)(a.sink_n * waves * 16)));
    std::vector<uint64_t> ts(NH), tn(NH);
    const int combos[][5] = {   // stream, store_mode, poll_sleep, scalar_poll, throttle
        {0, 0, 1, 0, 0}, {1, 0, 1, 0, 0}, {4, 0, 1, 0, 0}, {5, 0, 1, 0, 0}, {6, 0, 1, 0, 0},
        {1, 0, 1, 0, 16}, {1, 0, 1, 0, 8}, {1, 0, 1, 0, 4}, {1, 0, 1, 1, 8}};
    for (const auto& cb : combos) {
        {
            {
                const int stream = cb[0], store_mode = cb[1], poll_sleep = cb[2];
                a.stream = stream;
                a.store_mode = store_mode;
                a.poll_sleep = poll_sleep;
                a.scalar_poll = cb[3];
                a.throttle = cb[4];
                CHK(hipMemset(a.gran, 0, 256));
                CHK(hipMemset(a.stop, 0, 256));
                const int grid = stream ? ncu : 2;   // (stream 2 / 3: the other CUs idle)
                hipLaunchKernelGGL(handoff, dim3(grid), dim3(256), 0, 0, a);
                CHK(hipGetLastError());
                CHK(hipDeviceSynchronize());
                CHK(hipMemcpy(ts.data(), a.t_store, NH * 8, hipMemcpyDeviceToHost));
                CHK(hipMemcpy(tn.data(), a.t_seen, NH * 8, hipMemcpyDeviceToHost));
                std::vector<double> lat;
                for (int n = 10; n < NH; ++n) lat.push_back((double)(int64_t)(tn[n] - ts[n]) * 0.01);   // us
                std::sort(lat.begin(), lat.end());
                const double t_ms = (double)(int64_t)(tn[NH - 1] - ts[0]) * 1e-5;
                printf("stream=%d throttle=%-2d store=%-13s poll=%-9s %-6s latency us: median %6.2f  p10 %6.2f  p90 %6.2f  max %7.2f  (run %.1f ms)\n",
                       stream, cb[4], store_mode ? "plain+release" : "sc1", poll_sleep ? "sleep(1)" : "back2back",
                       cb[3] ? "scalar" : "vector",
                       lat[lat.size() / 2], lat[lat.size() / 10], lat[lat.size() * 9 / 10], lat.back(), t_ms);
            }
        }
    }
    return 0;
}
