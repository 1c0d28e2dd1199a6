// acs_step.hip -- calibration microbenchmark (not part of the product): cost of one
// trellis step of k_acs's packed two-codeword ACS (k_viterbi.hip: bcast, 2 packed adds,
// 2 compares into lane masks, 2 decision shift-ins, packed min), with the branch
// metrics in registers so only the step's own instructions run.  32 waves per CU
// (8 per SIMD).  Reports SIMD cycles per wave-step from the shader clock (s_memtime)
// and from the wall clock at the nominal frequency, so the sustained clock shows too.
//   VAR 0: the step as k_acs runs it
//   VAR 1: metrics only (no decisions)
//   VAR 2: decisions from one packed subtract (sign bits) shifted in per 16-bit half
//   VAR 3/4: the same with a 32-bit shift and a bit-field insert (compiler / v_bfi_b32)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_pk(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

template <int M>
__device__ __forceinline__ void bcast(uint32_t x, uint32_t &P, uint32_t &Q) {
    if constexpr (M == 1) {
        P = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xA0, 0xF, 0xF, false);
        Q = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xF5, 0xF, 0xF, false);
    } else if constexpr (M == 2) {
        P = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x44, 0xF, 0xF, false);
        Q = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xEE, 0xF, 0xF, false);
    } else if constexpr (M == 4) {
        Q = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x104, 0xF, 0x5, false);
        P = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x114, 0xF, 0xA, false);
    } else if constexpr (M == 8) {
        Q = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x108, 0xF, 0x3, false);
        P = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x118, 0xF, 0xC, false);
    } else if constexpr (M == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        P = r[0];
        Q = r[1];
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        P = r[0];
        Q = r[1];
    }
}
__device__ __forceinline__ uint32_t shift_in(uint32_t acc, uint64_t mask) {
    uint32_t r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(acc), "s"(mask));
    return r;
}

template <int VAR, int J>
__device__ __forceinline__ void step(uint32_t &x, uint32_t &a0, uint32_t &a1, const uint32_t (&bm)[12]) {
    constexpr int rho = J % 6;
    uint32_t P, Q;
    bcast<(32 >> rho)>(x, P, Q);
    const u16x2 A = as_pk(P) + as_pk(bm[2 * rho]), B = as_pk(Q) + as_pk(bm[2 * rho + 1]);
    if constexpr (VAR == 0) {
        a0 = shift_in(a0, __builtin_amdgcn_ballot_w64(A.x > B.x));
        a1 = shift_in(a1, __builtin_amdgcn_ballot_w64(A.y > B.y));
    } else if constexpr (VAR == 2) {
        const uint32_t d = as_u32(B - A);                  // sign bit of each half = (A > B)
        a0 = as_u32(as_pk(a0) >> (u16x2){1, 1});
        a0 = (d & 0x80008000u) | a0;
    } else if constexpr (VAR == 3) {                       // bit-field insert, compiler's choice
        const uint32_t d = as_u32(B - A);
        a0 = (d & 0x80008000u) | ((a0 >> 1) & 0x7FFF7FFFu);
    } else if constexpr (VAR == 4) {                       // v_bfi_b32 with the mask in an SGPR
        const uint32_t d = as_u32(B - A);
        uint32_t r;
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x80008000u), "v"(d), "v"(a0 >> 1));
        a0 = r;
    }
    x = as_u32(__builtin_elementwise_min(A, B));
}

template <int VAR>
__global__ __launch_bounds__(64, 8) void k_step(uint32_t *out, uint64_t *clk, int iters) {
    uint32_t bm[12];
#pragma unroll
    for (int i = 0; i < 12; i++) bm[i] = (threadIdx.x * (i + 3)) & 0x03FF03FFu;
    uint32_t x = threadIdx.x, a0 = 0, a1 = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        [&]<int... J>(std::integer_sequence<int, J...>) { (step<VAR, J>(x, a0, a1, bm), ...); }
        (std::make_integer_sequence<int, 30>{});
        x = as_u32(as_pk(x) - as_pk(__builtin_amdgcn_readfirstlane(x) & 0x0FFF0FFFu));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = x ^ a0 ^ a1;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int VAR>
static void run(const char *name, int cus, int clk_khz) {
    const int waves = cus * 32, iters = 4000;
    uint32_t *d;
    uint64_t *c;
    (void)hipMalloc(&d, sizeof(uint32_t) * waves * 64);
    (void)hipMalloc(&c, sizeof(uint64_t) * waves);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_step<VAR>, dim3(waves), dim3(64), 0, 0, d, c, 10);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_step<VAR>, dim3(waves), dim3(64), 0, 0, d, c, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t *h = new uint64_t[waves];
    (void)hipMemcpy(h, c, sizeof(uint64_t) * waves, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < waves; i++) mean += (double)h[i] / waves;
    const double wave_steps_per_simd = 8.0 * iters * 30;
    // s_memtime counts the shader clock: a wave's span covers 8 waves' steps on its SIMD
    printf("%-44s %8.3f ms  wall@nominal %.1f cyc/step  s_memtime %.1f cyc/step  -> sustained clock %.2f GHz\n", name,
           ms, ms * 1e-3 * clk_khz * 1e3 / wave_steps_per_simd, mean / wave_steps_per_simd,
           mean / (ms * 1e-3) / 1e9);
    delete[] h;
    (void)hipFree(d);
    (void)hipFree(c);
}

int main() {
    int cus = 0, clk = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    run<0>("ACS step as k_acs (2 cmp + 2 addc)", cus, clk);
    run<1>("metrics only (no decisions)", cus, clk);
    run<2>("decisions via packed sub + shift (3 ops)", cus, clk);
    run<3>("decisions via packed sub + lshr/and/or", cus, clk);
    run<4>("decisions via packed sub + lshr + v_bfi", cus, clk);
    return 0;
}
