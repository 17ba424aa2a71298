// Microbenchmark: single-wave VALU issue cost vs dependent latency on gfx950
// (plain VALU, DPP, s_nop), 16 instructions per iteration, cycles via s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ void k(int* out, long long* cyc, int n) {
  int a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    if (MODE == 0) {        // 16 independent adds (4 interleaved chains)
      asm volatile(
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (MODE == 1) { // 16 dependent adds
      asm volatile(
        "v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n"
        : "+v"(a));
    } else if (MODE == 2) { // 16 dependent DPP max with s_nop 1 between (the scan shape)
      asm volatile(
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(a));
    } else if (MODE == 3) { // 16 DPP max on 2 interleaved chains (no nops needed: 1 other + ... )
      asm volatile(
        "v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 0\n"
        "v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf\n s_nop 0\n"
        "v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf\n s_nop 0\n"
        "v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf\n s_nop 0\n"
        "v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 0\n"
        "v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf\n s_nop 0\n"
        "v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf\n s_nop 0\n"
        "v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf\n s_nop 0\n"
        : "+v"(a), "+v"(b));
    } else if (MODE == 4) { // 16 x s_nop 1
      asm volatile("s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n"
                   "s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n");
    } else if (MODE == 5) { // 16 independent v_max3 (VOP3)
      asm volatile(
        "v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %1, %1, %2, %3\n v_max3_i32 %2, %2, %3, %0\n v_max3_i32 %3, %3, %0, %1\n"
        "v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %1, %1, %2, %3\n v_max3_i32 %2, %2, %3, %0\n v_max3_i32 %3, %3, %0, %1\n"
        "v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %1, %1, %2, %3\n v_max3_i32 %2, %2, %3, %0\n v_max3_i32 %3, %3, %0, %1\n"
        "v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %1, %1, %2, %3\n v_max3_i32 %2, %2, %3, %0\n v_max3_i32 %3, %3, %0, %1\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    }
  }
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  int* out; long long* cyc; hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 1 << 16);
  const char* names[] = {"16 indep v_add", "16 dep v_add", "16 dep dpp+nop1", "16 dpp 2-chain", "16 s_nop 1", "16 indep v_max3"};
  void (*ks[])(int*, long long*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>};
  for (int waves : {1, 4, 8, 12}) for (int m = 0; m < 6; ++m) {
    int n = 20000;
    hipLaunchKernelGGL(ks[m], dim3(1), dim3(64 * waves), 0, 0, out, cyc, n);
    hipLaunchKernelGGL(ks[m], dim3(1), dim3(64 * waves), 0, 0, out, cyc, n);
    hipDeviceSynchronize();
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("waves/CU=%2d %-18s %6.2f clk/instr (per wave)\n", waves, names[m], (double)c / n / 16);
  }
  return 0;
}
