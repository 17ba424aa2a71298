// Microbenchmark: cost of one anti-diagonal column step on gfx950 (design probe).
// Lane l holds cell (t - l, l) at step t; per step: per-lane s1 byte from LDS,
// substitution (cmp + cndmask), up = wave_shr1(G) (DPP), G' = max3(G, up, diag'),
// 3-bit code (G-1 minus each candidate, v_alignbit), H (v_sub), one LDS ring
// write and one 256-B score store.  Timed per wave with s_memtime for W waves
// per workgroup (W/4 waves per SIMD); the values computed are not checked.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_antidiag tools/ubench_antidiag.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define STEP(T)                                                                          \
    "ds_read_u8 %[ch], %[sa] offset:" #T "\n"                                           \
    "v_add_u32_e32 %[gm1], -1, %[g]\n"                                                  \
    "v_sub_u32_e32 %[dl], %[gm1], %[gp]\n"                                              \
    "v_mov_b32_dpp %[up], %[g] wave_shr:1 row_mask:0xf bank_mask:0xf\n"                 \
    "v_sub_u32_e32 %[dd], %[gm1], %[dg]\n"                                              \
    "v_alignbit_b32 %[acc], %[acc], %[dl], 31\n"                                        \
    "v_add_u32_e32 %[dg], %[upp], %[sub]\n"                                             \
    "v_mov_b32_e32 %[gp], %[g]\n"                                                       \
    "v_max3_i32 %[g], %[g], %[up], %[dg]\n"                                             \
    "v_sub_u32_e32 %[du], %[gm1], %[upp]\n"                                             \
    "v_alignbit_b32 %[acc], %[acc], %[du], 31\n"                                        \
    "v_alignbit_b32 %[acc], %[acc], %[dd], 31\n"                                        \
    "v_mov_b32_e32 %[upp], %[up]\n"                                                     \
    "s_waitcnt lgkmcnt(1)\n"                                                            \
    "v_cmp_eq_u32_e64 %[m], %[ch], %[c2]\n"                                             \
    "v_cndmask_b32_e64 %[sub], %[vck], %[vcm], %[m]\n"                                  \
    "v_subrev_u32_e32 %[h], %[td], %[g]\n"                                              \
    "ds_write_b32 %[ra], %[g] offset:" #T "*4\n"                                        \
    "global_store_dword %[hv], %[h], %[hb] offset:" #T "*256\n"

__global__ void k(int* out, long long* cyc, int n) {
    __shared__ int lds[4096];
    const int lane = threadIdx.x & 63;
    int g = lane, gp = 0, up = 0, upp = 0, dg = 0, gm1 = 0, dl = 0, du = 0, dd = 0, h = 0, sub = 1, ch = 0;
    unsigned acc = 0;
    uint64_t m;
    const int c2 = lane & 3, vcm = 3, vck = 1, td = 5;
    const int sa = (int)(uintptr_t)(__attribute__((address_space(3))) int*)&lds[0] + 1024 - lane;
    const int ra = (int)(uintptr_t)(__attribute__((address_space(3))) int*)&lds[2048 + lane];
    const int hv = lane * 4;
    int* hb = out + 64 * 8 * __builtin_amdgcn_readfirstlane(blockIdx.x * 16 + (threadIdx.x >> 6));
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
        asm volatile(STEP(0) STEP(1) STEP(2) STEP(3) STEP(4) STEP(5) STEP(6) STEP(7)
                     : [g] "+v"(g), [gp] "+v"(gp), [up] "+v"(up), [upp] "+v"(upp), [dg] "+v"(dg), [gm1] "+v"(gm1),
                       [dl] "+v"(dl), [du] "+v"(du), [dd] "+v"(dd), [h] "+v"(h), [sub] "+v"(sub), [ch] "+v"(ch),
                       [acc] "+v"(acc), [m] "=&s"(m)
                     : [c2] "v"(c2), [vcm] "v"(vcm), [vck] "v"(vck), [td] "s"(td), [sa] "v"(sa), [ra] "v"(ra),
                       [hv] "v"(hv), [hb] "s"(hb)
                     : "vcc", "memory");
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    long long t1 = clock64();
    out[1 << 20 | (blockIdx.x * blockDim.x + threadIdx.x)] = g + (int)acc + h;
    if (lane == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
    int* out;
    long long* cyc;
    hipMalloc(&out, 64 << 20);
    hipMalloc(&cyc, 1 << 20);
    for (int blocks : {1, 256})
        for (int W : {1, 4, 8, 12, 16}) {
            const int n = 5000;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * W), 0, 0, out, cyc, n);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * W), 0, 0, out, cyc, n);
            hipDeviceSynchronize();
            long long c[16];
            (void)hipMemcpy(c, cyc, 8 * W, hipMemcpyDeviceToHost);
            double mx = 0;
            for (int w = 0; w < W; ++w) mx = c[w] > mx ? c[w] : mx;
            printf("blocks=%3d waves/WG=%2d  %6.1f clk per step per wave\n", blocks, W, mx / n / 8);
        }
    return 0;
}
