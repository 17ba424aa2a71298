// Microbenchmark: loop-carried dependency chains of one wave (cycles/iter,
// s_memtime).  Used to choose the per-column update of the fill kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define NEG ((int)0x80000000)
__device__ __forceinline__ int shr1(int old, int v) { return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int scan6(int y) {
  y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x111, 0xf, 0xf, false));
  y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x112, 0xf, 0xf, false));
  y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x114, 0xf, 0xf, false));
  y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x118, 0xf, 0xf, false));
  y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x142, 0xa, 0xf, false));
  y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x143, 0xc, 0xf, false));
  return y;
}
template <int MODE>
__global__ void chain(int* out, long long* cyc, int n, int seed) {
  __shared__ int lds[256];
  int lane = threadIdx.x & 63;
  int G = lane * seed, t = seed, acc = 0;
  int idx = ((lane * 7 + seed) & 63) * 4;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    if (MODE == 0) {            // old: shift + max3 + 6-level DPP scan
      int Y = max(max(G - 1, shr1(t, G) + (i & 3)), t);
      G = scan6(Y);
    } else if (MODE == 1) {     // bpermute gather + add + max3
      int b = max(max(G - 1, shr1(t, G) + (i & 3)), t);
      G = max(b, __builtin_amdgcn_ds_bpermute(idx, G) + 3);
    } else if (MODE == 2) {     // bpermute + an LDS write of G each step
      int b = max(max(G - 1, shr1(t, G) + (i & 3)), t);
      G = max(b, __builtin_amdgcn_ds_bpermute(idx, G) + 3);
      lds[lane] = G;
    } else if (MODE == 3) {     // ds_read dependent chain (LDS latency)
      lds[lane] = G; G = lds[(lane + 1) & 63] + 1;
    } else if (MODE == 4) {     // only shift + max3 (no scan)
      G = max(max(G - 1, shr1(t, G) + (i & 3)), t);
    } else if (MODE == 5) {     // 4-level row scan only (16-lane rows)
      int y = max(max(G - 1, shr1(t, G) + (i & 3)), t);
      y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x111, 0xf, 0xf, false));
      y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x112, 0xf, 0xf, false));
      y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x114, 0xf, 0xf, false));
      G = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x118, 0xf, 0xf, false));
    }
    acc += G;
  }
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  int* out; long long* cyc; hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 1 << 16);
  const char* names[] = {"dpp-scan6", "bpermute", "bpermute+ds_write", "ds_read chain", "shift+max3 only", "scan4(row)"};
  void (*ks[])(int*, long long*, int, int) = {chain<0>, chain<1>, chain<2>, chain<3>, chain<4>, chain<5>};
  for (int waves : {1, 2, 4, 8}) {
    for (int m = 0; m < 6; ++m) {
      int n = 100000;
      hipLaunchKernelGGL(ks[m], dim3(1), dim3(64 * waves), 0, 0, out, cyc, n, 3);
      hipDeviceSynchronize();
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a);
      hipLaunchKernelGGL(ks[m], dim3(1), dim3(64 * waves), 0, 0, out, cyc, n, 3);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("waves/WG=%d %-20s %7.1f clk/iter  %6.1f ns/iter\n", waves, names[m], (double)c / n, ms * 1e6 / n);
    }
  }
  return 0;
}
