// valu_rate.hip -- calibration microbenchmark (not part of the product): sustained
// wave64 VALU issue rate per SIMD on this GPU for the instruction classes k_acs uses
// (32-bit add, packed 16-bit add/min, DPP move, 16-bit compare into a lane mask) and
// the float kinds the demod uses (f32, packed f32, f64).
// Grid: 32 waves per CU (8 per SIMD), each with 8 independent dependency chains.
// Prints cycles per wave-instruction per SIMD (2.0 = full rate of a SIMD-32).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) (void)(x)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(64) void k_rate(uint32_t *out, int iters) {
    uint32_t v[8];
    const uint32_t k1 = threadIdx.x * 7 + 1;
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = threadIdx.x * 13 + c;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int c = 0; c < 8; c++) {
                if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 1) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 2) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf" : "+v"(v[c]));
                else if constexpr (OP == 3) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 4) asm volatile("v_cmp_gt_u16_sdwa vcc, %0, %1 src0_sel:WORD_1 src1_sel:WORD_1" :: "v"(v[c]), "v"(k1) : "vcc");
                else if constexpr (OP == 5) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 6) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 7) asm volatile("v_rcp_f32 %0, %0" : "+v"(v[c]));
                else if constexpr (OP == 8) asm volatile("v_rndne_f32 %0, %0" : "+v"(v[c]));
                else if constexpr (OP == 9) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(v[c]));
                else if constexpr (OP == 10) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 11) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(v[c]));
                else if constexpr (OP == 12) asm volatile("v_mov_b32 %0, %1" : "=v"(v[c]) : "v"(v[(c + 1) & 7]));
                else if constexpr (OP == 13) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(v[c]), "+v"(v[(c + 4) & 7]));
                else if constexpr (OP == 14) asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %0, %1 row_shr:4 row_mask:0xf bank_mask:0xa" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 15) asm volatile("v_pk_sub_i16 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 16) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 17) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 18) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 19) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 20) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 21) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 22) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 23) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 24) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 25) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(v[c]));
                else if constexpr (OP == 26) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 27) asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(v[c]), "v"(k1) : "vcc");
            }
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s ^= v[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

// the same for 64-bit operands (register pairs): packed f32 and f64
template <int OP>
__global__ __launch_bounds__(64) void k_rate64(uint64_t *out, int iters) {
    uint64_t v[8];
    const uint64_t k1 = threadIdx.x * 7 + 1;
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = threadIdx.x * 13 + c;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int c = 0; c < 8; c++) {
                if constexpr (OP == 0) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 3) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 4) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
                else if constexpr (OP == 5) asm volatile("v_add_f64 %0, %0, %1" : "+v"(v[c]) : "v"(k1));
            }
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s ^= v[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int OP, bool W64 = false>
static void run(const char *name, int cus) {
    const int waves = cus * 32, iters = 2000;
    uint64_t *d;
    CK(hipMalloc(&d, sizeof(uint64_t) * waves * 64));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto launch = [&](int it) {
        if constexpr (W64) hipLaunchKernelGGL(k_rate64<OP>, dim3(waves), dim3(64), 0, 0, d, it);
        else hipLaunchKernelGGL(k_rate<OP>, dim3(waves), dim3(64), 0, 0, (uint32_t *)d, it);
    };
    for (int w = 0; w < 20; w++) launch(200);      // clocks up
    launch(10);
    hipEventRecord(a);
    launch(iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const double instrs_per_simd = (double)8 /*waves per SIMD*/ * iters * 16 * 8;
    const double cycles = ms * 1e-3 * clk_khz * 1e3;
    printf("%-28s %8.3f ms  %.2f cycles per wave-instruction per SIMD (clock %.2f GHz)\n", name, ms,
           cycles / instrs_per_simd, clk_khz / 1e6);
    hipFree(d);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    run<0>("v_add_u32", cus);
    run<1>("v_pk_add_u16", cus);
    run<2>("v_mov_b32_dpp quad_perm", cus);
    run<3>("v_pk_min_u16", cus);
    run<4>("v_cmp_gt_u16_sdwa", cus);
    run<5>("v_add_f32", cus);
    run<6>("v_fmac_f32", cus);
    run<7>("v_rcp_f32", cus);
    run<8>("v_rndne_f32", cus);
    run<9>("v_cvt_i32_f32", cus);
    run<10>("v_bfi_b32", cus);
    run<11>("v_lshrrev_b32", cus);
    run<12>("v_mov_b32", cus);
    run<13>("v_permlane32_swap", cus);
    run<14>("s_nop1+v_add_u32_dpp row_shr", cus);
    run<15>("v_pk_sub_i16", cus);
    run<16>("v_alignbit_b32", cus);
    run<17>("v_and_or_b32", cus);
    run<18>("v_lshl_or_b32", cus);
    run<19>("v_cndmask_b32", cus);
    run<20>("v_xor_b32", cus);
    run<21>("v_perm_b32", cus);
    run<22>("v_mul_f32", cus);
    run<23>("v_add_u32_e64 (VOP3)", cus);
    run<24>("v_sub_u32", cus);
    run<25>("v_lshlrev_b32", cus);
    run<26>("v_pk_max_i16", cus);
    run<27>("v_cmp_gt_u32", cus);
    run<0, true>("v_pk_add_f32", cus);
    run<1, true>("v_pk_fma_f32", cus);
    run<2, true>("v_pk_mul_f32", cus);
    run<3, true>("v_fma_f64", cus);
    run<4, true>("v_mul_f64", cus);
    run<5, true>("v_add_f64", cus);
    return 0;
}
