// Microbenchmark: SIMD throughput of the instruction classes of the fill's
// column step on gfx950.  One workgroup of 4*k waves (k waves per SIMD), each
// wave runs a loop of 32 independent instructions of one class (8 rotating
// registers, so no DPP hazard and no dependency stall).  Prints cycles per
// instruction per wave (s_memtime) and the implied SIMD occupancy per
// instruction = (cycles/instr per wave) / (waves per SIMD).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_simd tools/ubench_simd.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define R32(X) R8(X) R8(X) R8(X) R8(X)

template <int MODE>
__global__ void k(int* out, long long* cyc, int n) {
    __shared__ int lds[64 * 16 * 8];
    int v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
    int* gp = out + 8 * 64 * 16 * blockIdx.x + 64 * __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int la = (int)(uintptr_t)(__attribute__((address_space(3))) int*)&lds[threadIdx.x * 8];
    const int go = threadIdx.x * 4;
    const int l1 = (int)(uintptr_t)(__attribute__((address_space(3))) int*)&lds[threadIdx.x];
    uint64_t s0, s1, s2, s3;
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#define OPS : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7), "=&s"(s0), "=&s"(s1), \
              "=&s"(s2), "=&s"(s3) : "v"(la), "v"(go), "s"(gp), "v"(l1) : "vcc", "memory"
#define I_ADD(r) "v_add_u32 %" #r ", %" #r ", 1\n"
#define I_MAX3(r) "v_max3_i32 %" #r ", %" #r ", %0, %1\n"
#define I_SHR(r) "v_max_i32_dpp %" #r ", %" #r ", %" #r " row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define I_B15(r) "v_max_i32_dpp %" #r ", %" #r ", %" #r " row_bcast:15 row_mask:0xa bank_mask:0xf\n"
#define I_B31(r) "v_max_i32_dpp %" #r ", %" #r ", %" #r " row_bcast:31 row_mask:0xc bank_mask:0xf\n"
#define I_WSHR(r) "v_mov_b32_dpp %" #r ", %" #r " wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define I_CMP(r) "v_cmp_eq_i32_e64 %8, %" #r ", %0\n"
#define I_ADDC(r) "v_addc_co_u32_e64 %" #r ", vcc, %" #r ", %" #r ", %8\n"
#define I_CND(r) "v_cndmask_b32_e64 %" #r ", %" #r ", %0, %8\n"
#define I_ADD3(r) "v_add3_u32 %" #r ", %" #r ", %0, %1\n"
#define I_DSW(r) "ds_write_b32 %12, %" #r " offset:" #r "\n"
#define I_GST(r) "global_store_dword %13, %" #r ", %14\n"
#define I_NOP(r) "s_nop 1\n"
#define I_SALU(r) "s_bfe_u64 %9, %8, 0x80008\n"
#define I_CMP32(r) "v_cmp_eq_i32_e32 vcc, %" #r ", %0\n"
#define I_ADDC32(r) "v_addc_co_u32_e32 %" #r ", vcc, %" #r ", %" #r ", vcc\n"
#define I_CND32(r) "v_cndmask_b32_e32 %" #r ", %" #r ", %0, vcc\n"
#define I_MAX32(r) "v_max_i32_e32 %" #r ", %" #r ", %0\n"
#define I_SUB32(r) "v_sub_u32_e32 %" #r ", %" #r ", %0\n"
#define I_DSW1(r) "ds_write_b32 %15, %" #r " offset:" #r "*4\n"
#define I_OR(r) "v_or_b32_e32 %" #r ", %0, %" #r "\n"
#define I_AND(r) "v_and_b32_e32 %" #r ", %0, %" #r "\n"
#define I_XOR(r) "v_xor_b32_e32 %" #r ", %0, %" #r "\n"
#define I_LSR(r) "v_lshrrev_b32_e32 %" #r ", 3, %" #r "\n"
#define I_MOV(r) "v_mov_b32_e32 %" #r ", %0\n"
#define I_ALIGN(r) "v_alignbit_b32 %" #r ", %" #r ", %0, 31\n"
#define I_ADDSDWA(r) "v_add_u32_sdwa %" #r ", %" #r ", %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
#define I_CMPSDWA(r) "v_cmp_eq_u32_sdwa vcc, %" #r ", %0 src0_sel:BYTE_1 src1_sel:DWORD\n"
#define I_SUBREV(r) "v_subrev_u32_e32 %" #r ", %0, %" #r "\n"
#define I_ADDDPP(r) "v_add_u32_dpp %" #r ", %" #r ", %" #r " wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define I_MAXU(r) "v_max_u32_e32 %" #r ", %0, %" #r "\n"
#define I_MED3(r) "v_med3_i32 %" #r ", %" #r ", %0, %1\n"
#define I_LSHLOR(r) "v_lshl_or_b32 %" #r ", %" #r ", 1, %0\n"
#define I_PERM(r) "v_perm_b32 %" #r ", %" #r ", %0, %1\n"
#define I_ADDCO(r) "v_add_co_u32_e32 %" #r ", vcc, %0, %" #r "\n"
#define I_MAXDPP8(r) "v_max_i32_dpp %" #r ", %" #r ", %" #r " row_shr:8 row_mask:0xf bank_mask:0xf\n"
#define I_PAIR(r) "v_cmp_eq_i32_e32 vcc, %" #r ", %0\n v_addc_co_u32_e32 %1, vcc, %1, %1, vcc\n"
        if (MODE == 0) asm volatile(R32(I_ADD) OPS);
        if (MODE == 1) asm volatile(R32(I_MAX3) OPS);
        if (MODE == 2) asm volatile(R32(I_SHR) OPS);
        if (MODE == 3) asm volatile(R32(I_B15) OPS);
        if (MODE == 4) asm volatile(R32(I_B31) OPS);
        if (MODE == 5) asm volatile(R32(I_WSHR) OPS);
        if (MODE == 6) asm volatile(R32(I_CMP) OPS);
        if (MODE == 7) asm volatile("v_cmp_eq_i32_e64 %8, %0, %1\n" R32(I_ADDC) OPS);
        if (MODE == 8) asm volatile("v_cmp_eq_i32_e64 %8, %0, %1\n" R32(I_CND) OPS);
        if (MODE == 9) asm volatile(R32(I_ADD3) OPS);
        if (MODE == 10) asm volatile(R32(I_DSW) OPS);
        if (MODE == 11) asm volatile(R32(I_GST) OPS);
        if (MODE == 12) asm volatile(R32(I_NOP) OPS);
        if (MODE == 13) asm volatile("s_mov_b64 %8, 0x1234\n" R32(I_SALU) OPS);
        if (MODE == 14) asm volatile(R32(I_CMP32) OPS);
        if (MODE == 15) asm volatile("v_cmp_eq_i32_e32 vcc, %0, %1\n" R32(I_ADDC32) OPS);
        if (MODE == 16) asm volatile("v_cmp_eq_i32_e32 vcc, %0, %1\n" R32(I_CND32) OPS);
        if (MODE == 17) asm volatile(R32(I_MAX32) OPS);
        if (MODE == 18) asm volatile(R32(I_SUB32) OPS);
        if (MODE == 19) asm volatile(R32(I_DSW1) OPS);
        if (MODE == 20) asm volatile(R8(I_PAIR) R8(I_PAIR) OPS);
        if (MODE == 21) asm volatile(R32(I_OR) OPS);
        if (MODE == 22) asm volatile(R32(I_AND) OPS);
        if (MODE == 23) asm volatile(R32(I_XOR) OPS);
        if (MODE == 24) asm volatile(R32(I_LSR) OPS);
        if (MODE == 25) asm volatile(R32(I_MOV) OPS);
        if (MODE == 26) asm volatile(R32(I_ALIGN) OPS);
        if (MODE == 27) asm volatile(R32(I_ADDSDWA) OPS);
        if (MODE == 28) asm volatile(R32(I_CMPSDWA) OPS);
        if (MODE == 29) asm volatile(R32(I_SUBREV) OPS);
        if (MODE == 30) asm volatile(R32(I_ADDDPP) OPS);
        if (MODE == 31) asm volatile(R32(I_MAXU) OPS);
        if (MODE == 32) asm volatile(R32(I_MED3) OPS);
        if (MODE == 33) asm volatile(R32(I_LSHLOR) OPS);
        if (MODE == 34) asm volatile(R32(I_PERM) OPS);
        if (MODE == 35) asm volatile(R32(I_ADDCO) OPS);
        if (MODE == 36) asm volatile(R32(I_MAXDPP8) OPS);
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x + 1000000] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + (int)s0;
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

int main() {
    int* out;
    long long* cyc;
    hipMalloc(&out, 64 << 20);
    hipMalloc(&cyc, 1 << 16);
    const char* names[] = {"v_add_u32", "v_max3_i32", "dpp max row_shr:1", "dpp max row_bcast:15",
                           "dpp max row_bcast:31", "v_mov_dpp wave_shr:1", "v_cmp_e64 -> sgpr", "v_addc (sgpr carry)",
                           "v_cndmask_e64 (sgpr)", "v_add3_u32", "ds_write_b32", "global_store_dword",
                           "s_nop 1", "s_bfe_u64 (salu)", "v_cmp_e32 -> vcc", "v_addc_e32 (vcc)",
                           "v_cndmask_e32 (vcc)", "v_max_i32_e32", "v_sub_u32_e32", "ds_write_b32 stride1",
                           "cmp_e32+addc_e32 pair/2", "v_or_b32", "v_and_b32", "v_xor_b32",
                           "v_lshrrev_b32", "v_mov_b32", "v_alignbit_b32", "v_add_u32_sdwa byte", "v_cmp_eq_sdwa byte",
                           "v_subrev_u32", "v_add_u32_dpp wave_shr", "v_max_u32_e32", "v_med3_i32", "v_lshl_or_b32",
                           "v_perm_b32", "v_add_co_u32_e32", "dpp max row_shr:8"};
    void (*ks[])(int*, long long*, int) = {k<0>,  k<1>,  k<2>,  k<3>,  k<4>,  k<5>,  k<6>,  k<7>,  k<8>,  k<9>,
                                           k<10>, k<11>, k<12>, k<13>, k<14>, k<15>, k<16>, k<17>, k<18>, k<19>,
                                           k<20>, k<21>, k<22>, k<23>, k<24>, k<25>, k<26>, k<27>, k<28>, k<29>,
                                           k<30>, k<31>, k<32>, k<33>, k<34>, k<35>, k<36>};
    printf("%-24s %s\n", "instruction", "clk/instr per wave @ 1,2,3,4 waves/SIMD  -> SIMD clk per instr");
    for (int m = 0; m < 37; ++m) {
        printf("%-24s", names[m]);
        double occ = 0;
        for (int wps = 1; wps <= 4; ++wps) {
            const int waves = 4 * wps, n = 4000;
            hipLaunchKernelGGL(ks[m], dim3(1), dim3(64 * waves), 0, 0, out, cyc, n);
            hipLaunchKernelGGL(ks[m], dim3(1), dim3(64 * waves), 0, 0, out, cyc, n);
            hipDeviceSynchronize();
            long long c[16];
            hipMemcpy(c, cyc, 8 * waves, hipMemcpyDeviceToHost);
            double mx = 0;
            for (int w = 0; w < waves; ++w) mx = c[w] > mx ? c[w] : mx;
            const double cpi = mx / n / 32;
            printf(" %6.2f", cpi);
            occ = cpi / wps;
        }
        printf("   -> %5.2f\n", occ);
    }
    return 0;
}
