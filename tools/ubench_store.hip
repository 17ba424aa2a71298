// Microbenchmark: global store throughput on gfx950, one CU vs the whole chip,
// dword (256 B per wave instruction, the fill's per-column score store) vs
// dwordx4 (1 KB per instruction).  Each wave streams to its own region.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_store tools/ubench_store.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int X4>
__global__ void k(int* out, long long* cyc, int n, long long per_wave) {
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    char* base = (char*)out + per_wave * wave;
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
        if (X4) {
            int4 v = make_int4(i, i + 1, i + 2, i + 3);
            *(int4*)(base + (long long)i * 1024 + lane * 16) = v;
        } else {
            *(int*)(base + (long long)i * 256 + lane * 4) = i;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    long long t1 = clock64();
    if (lane == 0) cyc[wave] = t1 - t0;
}

int main() {
    int* out;
    long long* cyc;
    const long long total = 6LL << 30;
    hipMalloc(&out, total);
    hipMalloc(&cyc, 1 << 20);
    for (int x4 = 0; x4 < 2; ++x4)
        for (int blocks : {1, 256}) for (int wpb : {4, 8}) {
            const int waves = blocks * wpb;
            const int bytes_per = x4 ? 1024 : 256;
            const int n = (int)std::min<long long>(20000, total / waves / bytes_per);
            const long long per_wave = (long long)n * bytes_per;
            auto fn = x4 ? k<1> : k<0>;
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(64 * wpb), 0, 0, out, cyc, n, per_wave);
            hipEventRecord(e0);
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(64 * wpb), 0, 0, out, cyc, n, per_wave);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            long long c;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            const double gbs = (double)waves * per_wave / (ms * 1e-3) / 1e9;
            printf("%-8s blocks=%3d waves/CU=%d  %7.1f clk/instr/wave  %8.1f GB/s  (%.3f ms)\n", x4 ? "dwordx4" : "dword",
                   blocks, wpb, (double)c / n, gbs, ms);
        }
    return 0;
}
