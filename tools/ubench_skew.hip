// Microbenchmark: cost of the skew kernel's generated 8-step chunk block
// (nw_skew_chunk.inc) in isolation, no ring dependencies.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I needleman-wunsch_amd/csrc \
//         -o tools/ubench_skew tools/ubench_skew.hip
//   tools/ubench_skew            -> cycles per chunk for each variant and waves/SIMD
// Variants: 0 = block only, 1 = block + the chunk's 3 nt stores,
//           2 = block + stores + the C++ bookkeeping of a middle chunk.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
struct SkewSlot { v4i a, b; v2i w; };
struct SkewRegs { int e[7]; int ein; int upc; int h[8]; uint32_t acc; int gav; uint64_t pq; };
struct SkewConst { int sd[8]; int kd[8]; uint32_t c2; int vcm, vck; uint32_t pl, ph; int cb; };
#include "nw_skew_chunk.inc"

__device__ __forceinline__ int lds_addr(const void* p) {
    return (int)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int V>
__global__ __launch_bounds__(1024) void k(int* out, long long* cyc, int n) {
    __shared__ __attribute__((aligned(16))) int lds[8192];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    SkewConst kc;
    for (int s = 0; s < 8; ++s) { kc.sd[s] = s; kc.kd[s] = -(s + 1); asm volatile("" : "+v"(kc.sd[s]), "+v"(kc.kd[s])); }
    kc.c2 = lane & 3; kc.vcm = 3; kc.vck = 1; kc.pl = 0x01010103u; kc.ph = 0x01010101u;
    kc.cb = lds_addr(&lds[64 * w]);
    asm volatile("" : "+v"(kc.c2), "+v"(kc.vcm), "+v"(kc.vck), "+v"(kc.pl), "+v"(kc.ph), "+v"(kc.cb));
    SkewRegs r; r.ein = lane; r.upc = 0; r.gav = 0;
    SkewSlot tA, tB;
    tA.a = v4i{1, 2, 3, 4}; tA.b = v4i{5, 6, 7, 8}; tA.w = v2i{0x03020100, 0x01000302};
    tB = tA;
    const int ra = lds_addr(&lds[1024 + 64 * w + lane]), rd = lds_addr(&lds[4096 + 64 * w]);
    const int wa = lds_addr(&lds[6144 + 64 * w + lane]) & ~7;
    int32_t* hb = out + (size_t)(blockIdx.x * 16 + w) * 512 * (n + 1);
    uint32_t* db = reinterpret_cast<uint32_t*>(out) + (size_t)(1 << 26) + (size_t)(blockIdx.x * 16 + w) * 64 * (n + 1);
    int hv = lane * 16, dv = lane * 4, Pc = 0, cv = 1;
    uint32_t bc = 0;
    long long t0 = clock64();
    for (int i = 0; i < n; i += 2) {
        skew_chunk_asm<false, true>(r, kc, tA, tB, Pc, -Pc, cv, ra, ra + 64, rd, wa);
        if (V >= 1) {
            asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\tglobal_store_dwordx4 %0, %3, %2 offset:1024 nt"
                         :: "v"(hv), "v"(v4i{r.h[0], r.h[1], r.h[2], r.h[3]}), "s"(hb), "v"(v4i{r.h[4], r.h[5], r.h[6], r.h[7]}) : "memory");
            asm volatile("global_store_dword %0, %1, %2 nt" :: "v"(dv), "v"(r.acc), "s"(db) : "memory");
            hv += 2048; dv += 256;
        }
        if (V >= 2) { Pc += 8; cv += 1; bc += __builtin_popcount(r.acc); if (__builtin_amdgcn_readfirstlane((int)(uint32_t)r.pq) == 12345) break; }
        skew_chunk_asm<false, true>(r, kc, tB, tA, Pc, -Pc, cv, ra, ra + 64, rd, wa);
        if (V >= 1) {
            asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\tglobal_store_dwordx4 %0, %3, %2 offset:1024 nt"
                         :: "v"(hv), "v"(v4i{r.h[0], r.h[1], r.h[2], r.h[3]}), "s"(hb), "v"(v4i{r.h[4], r.h[5], r.h[6], r.h[7]}) : "memory");
            asm volatile("global_store_dword %0, %1, %2 nt" :: "v"(dv), "v"(r.acc), "s"(db) : "memory");
            hv += 2048; dv += 256;
        }
        if (V >= 2) { Pc += 8; cv += 1; bc += __builtin_popcount(r.acc); if (__builtin_amdgcn_readfirstlane((int)(uint32_t)r.pq) == 12345) break; }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    long long t1 = clock64();
    out[(1 << 27) + blockIdx.x * blockDim.x + threadIdx.x] = r.ein + (int)r.acc + r.h[7] + (int)bc;
    if (lane == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
}

template <int V>
void run(int waves, int n, int* out, long long* cyc) {
    hipLaunchKernelGGL(k<V>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, n);
    hipDeviceSynchronize();
    long long h[16];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < waves; ++i) mx = h[i] > mx ? h[i] : mx;
    printf("variant %d  waves/CU %2d (%d per SIMD): %.1f cycles per chunk (%.1f per step)\n", V, waves,
           (waves + 3) / 4, mx / n, mx / n / 8);
}

int main() {
    int* out;
    long long* cyc;
    const int n = 2000;
    hipMalloc(&out, (size_t)1 << 30);
    hipMalloc(&cyc, 16 * 8);
    for (int waves : {1, 4, 8, 12}) {
        run<0>(waves, n, out, cyc);
        run<1>(waves, n, out, cyc);
        run<2>(waves, n, out, cyc);
    }
    return 0;
}
