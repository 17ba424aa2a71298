// Microbenchmark: issue cost of LDS write forms for the skew kernel's ring
// (one wave alone and 2 per SIMD): full-wave ds_write_b32, the same with only
// lane 63 enabled (exec juggling around it), ds_write_b128 from lane 63 only,
// ds_write2_b32 (two counters in one instruction).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_ldsw tools/ubench_ldsw.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V>
__global__ __launch_bounds__(1024) void k(int* out, long long* cyc, int n) {
    __shared__ __attribute__((aligned(16))) int lds[16384];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int a = (int)(uintptr_t)(__attribute__((address_space(3))) int*)&lds[256 * w + lane];
    const int a16 = (int)(uintptr_t)(__attribute__((address_space(3))) int*)&lds[256 * w + 4 * lane];
    int x = lane, y = lane + 1, z = 2, q = 3;
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
        if (V == 0)
            asm volatile("ds_write_b32 %0, %1\n ds_write_b32 %0, %1 offset:4\n ds_write_b32 %0, %1 offset:8\n ds_write_b32 %0, %1 offset:12\n"
                         "ds_write_b32 %0, %1 offset:16\n ds_write_b32 %0, %1 offset:20\n ds_write_b32 %0, %1 offset:24\n ds_write_b32 %0, %1 offset:28"
                         :: "v"(a), "v"(x) : "memory");
        if (V == 1)
            asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b32 %0, %1\n s_mov_b64 exec, s[40:41]\n"
                         "s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b32 %0, %1 offset:4\n s_mov_b64 exec, s[40:41]\n"
                         "s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b32 %0, %1 offset:8\n s_mov_b64 exec, s[40:41]\n"
                         "s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b32 %0, %1 offset:12\n s_mov_b64 exec, s[40:41]\n"
                         "s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b32 %0, %1 offset:16\n s_mov_b64 exec, s[40:41]\n"
                         "s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b32 %0, %1 offset:20\n s_mov_b64 exec, s[40:41]\n"
                         "s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b32 %0, %1 offset:24\n s_mov_b64 exec, s[40:41]\n"
                         "s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b32 %0, %1 offset:28\n s_mov_b64 exec, s[40:41]"
                         :: "v"(a), "v"(x) : "memory", "s40", "s41");
        if (V == 2) {
            typedef int v4i __attribute__((ext_vector_type(4)));
            v4i v = v4i{x, y, z, q};
            asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b32 exec_lo, 0\n s_mov_b32 exec_hi, 0x80000000\n"
                         "ds_write_b128 %0, %1\n ds_write_b128 %0, %1 offset:16\n s_mov_b64 exec, s[40:41]"
                         :: "v"(a16), "v"(v) : "memory", "s40", "s41");
        }
        if (V == 3)
            asm volatile("ds_write2_b32 %0, %1, %2 offset0:1 offset1:4" :: "v"(a), "v"(x), "v"(y) : "memory");
        if (V == 4)
            asm volatile("ds_write_b32 %0, %1 offset:4\n ds_write_b32 %0, %2 offset:16" :: "v"(a), "v"(x), "v"(y) : "memory");
        x += 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long t1 = clock64();
    if (lane == 0) cyc[w] = t1 - t0;
    out[threadIdx.x] = lds[threadIdx.x] + x;
}

template <int V>
void run(const char* name, int waves, int n, int* out, long long* cyc) {
    hipLaunchKernelGGL(k<V>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, n);
    hipDeviceSynchronize();
    long long h[16];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < waves; ++i) mx = h[i] > mx ? h[i] : mx;
    printf("%-40s waves/CU %2d: %.1f cycles per iteration\n", name, waves, mx / n);
}

int main() {
    int* out;
    long long* cyc;
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cyc, 16 * 8);
    for (int w : {1, 8}) {
        run<0>("8 x ds_write_b32 (all lanes)", w, 4000, out, cyc);
        run<1>("8 x ds_write_b32 (lane 63, exec swap)", w, 4000, out, cyc);
        run<2>("2 x ds_write_b128 (lane 63, exec swap)", w, 4000, out, cyc);
        run<3>("1 x ds_write2_b32 (counters)", w, 4000, out, cyc);
        run<4>("2 x ds_write_b32 (counters)", w, 4000, out, cyc);
    }
    return 0;
}
