// Microbenchmark of the fill kernel's hand-scheduled column step (same asm),
// per wave, vs waves per CU and per-superstep barriers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define NW_STEP_HEAD                                                   \
    "v_cmp_eq_u32_e32 vcc, %[ch], %[c2]\n\t"                           \
    "v_cndmask_b32_e32 %[sub], %[ck], %[cm], vcc\n\t"                  \
    "v_mov_b32_dpp %[sh], %[G] wave_shr:1 row_mask:0xf bank_mask:0xf\n\t" \
    "v_subrev_u32_e32 %[lf], %[d], %[G]\n\t"                           \
    "v_add_u32_e32 %[dg], %[sh], %[sub]\n\t"                           \
    "v_max3_i32 %[Y], %[lf], %[dg], %[top]\n\t"
#define NW_DPP(CTRL) "v_max_i32_dpp %[Y], %[Y], %[Y] " CTRL "\n\t"
#define NW_SCAN_FILLED                                                 \
    "v_cmp_eq_i32_e64 %[sa], %[pG], %[pdg]\n\tv_cmp_eq_i32_e64 %[sb], %[pG], %[sh]\n\t" \
    NW_DPP("row_shr:1 row_mask:0xf bank_mask:0xf")                     \
    "v_cmp_eq_i32_e32 vcc, %[pG], %[plf]\n\tv_lshlrev_b32_e32 %[acc], 1, %[acc]\n\t" \
    NW_DPP("row_shr:2 row_mask:0xf bank_mask:0xf")                     \
    "v_addc_co_u32_e64 %[acc], %[junk], %[acc], %[acc], vcc\n\tv_addc_co_u32_e64 %[acc], %[junk], %[acc], %[acc], %[sb]\n\t" \
    NW_DPP("row_shr:4 row_mask:0xf bank_mask:0xf")                     \
    "v_addc_co_u32_e64 %[acc], %[junk], %[acc], %[acc], %[sa]\n\tv_sub_u32_e32 %[Hp], %[pG], %[lo]\n\t" \
    NW_DPP("row_shr:8 row_mask:0xf bank_mask:0xf")                     \
    "s_nop 1\n\t" NW_DPP("row_bcast:15 row_mask:0xa bank_mask:0xf")    \
    "s_nop 1\n\tv_max_i32_dpp %[Y], %[Y], %[Y] row_bcast:31 row_mask:0xc bank_mask:0xf"
template <int BAR, int LDSW, int STORE>
__global__ void k(int* out, long long* cyc, int n, const uint8_t* s1) {
  __shared__ int lds[1024];
  int lane = threadIdx.x & 63;
  int G = 0, pG = 0, pdg = 0, plf = 0, acc = 0, Hp = 0, dg = 0, lf = 0;
  uint32_t c2 = 'A' + (lane & 3);
  int vck = 0, vcm = 2, top = -3, lo = lane;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    uint32_t ch = __builtin_amdgcn_readfirstlane('A' + (i & 3));
    int Y, sub; uint64_t sa, sb, junk; int sh = top;
    asm volatile(NW_STEP_HEAD NW_SCAN_FILLED
      : [Y] "=&v"(Y), [sh] "+v"(sh), [sub] "=&v"(sub), [dg] "=&v"(dg), [lf] "=&v"(lf), [Hp] "=&v"(Hp),
        [acc] "+v"(acc), [sa] "=&s"(sa), [sb] "=&s"(sb), [junk] "=&s"(junk)
      : [G] "v"(G), [ch] "s"(ch), [c2] "v"(c2), [ck] "v"(vck), [cm] "v"(vcm), [d] "s"(1), [top] "v"(top),
        [pG] "v"(pG), [pdg] "v"(pdg), [plf] "v"(plf), [lo] "v"(lo)
      : "vcc");
    pG = G = Y; pdg = dg; plf = lf;
    if (LDSW) lds[(threadIdx.x & 511) + (i & 7)] = G;
    if (STORE) out[(blockIdx.x * 1024 + (i & 1023)) * 64 + lane] = Hp;
    if (BAR && (i & 7) == 7) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  long long t1 = clock64();
  out[threadIdx.x] += acc + G;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  int* out; long long* cyc; uint8_t* s1;
  hipMalloc(&out, 256 << 20); hipMalloc(&cyc, 1 << 16); hipMalloc(&s1, 1 << 20);
  struct { const char* name; void (*f)(int*, long long*, int, const uint8_t*); } ks[] = {
    {"step", k<0, 0, 0>}, {"step+bar8", k<1, 0, 0>}, {"step+lds", k<0, 1, 0>},
    {"step+lds+bar8", k<1, 1, 0>}, {"step+store", k<0, 0, 1>}, {"step+lds+store+bar8", k<1, 1, 1>}};
  for (int waves : {1, 2, 4, 8, 9, 12}) for (auto& kk : ks) {
    int n = 20000;
    hipLaunchKernelGGL(kk.f, dim3(1), dim3(64 * waves), 0, 0, out, cyc, n, s1);
    hipLaunchKernelGGL(kk.f, dim3(1), dim3(64 * waves), 0, 0, out, cyc, n, s1);
    hipDeviceSynchronize();
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("waves/WG=%2d %-22s %6.1f clk/step\n", waves, kk.name, (double)c / n);
  }
  return 0;
}
