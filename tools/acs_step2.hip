// acs_step2.hip -- calibration microbenchmark (not part of the product): SIMD cycles per
// wave-step of two formulations of the packed two-codeword ACS step, branch metrics in
// registers, one decision word (30 steps, the 6 relabelling phases 5 times) per trip,
// 8 waves per SIMD.
//   VAR 0: the product's step (k_viterbi.hip acs_word_cw): candidates A = x[lane & ~M] + ta,
//          B = x[lane | M] + tb (DPP / bank-masked DPP / swizzle / permlane32), decisions
//          from one packed subtract's sign bits, collected per step pair by v_perm + v_bfi
//   VAR 1: own / partner candidates with the decision in the metric's LSB: metrics doubled,
//          every lane's metric carries bit M of its lane in the LSB (x = bfi(1, c, x'));
//          C_own = x + t_own, C_par = x[lane ^ M] + t_par (one DPP add: quad_perm, row_ror:8;
//          swizzle for M = 4, 16; permlane32 for 32), x' = min -> LSB = (B chosen);
//          collected per step pair by v_perm + v_add + v_bfi
//   VAR 2: VAR 1 with M = 4 through two DPP moves (row_half_mirror, quad_perm) instead of
//          the swizzle
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_pk(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
template <int A, int B> struct R {};
template <int I, int N, class F> __device__ __forceinline__ void sfor(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

#define DPP_ADD(ctl) "v_add_u32_dpp %0, %1, %2 " ctl
#define DPP_ADD_NOP(ctl) "s_nop 1\n\tv_add_u32_dpp %0, %1, %2 " ctl
template <int M>
__device__ __forceinline__ void cand(uint32_t x, uint32_t ta, uint32_t tb, uint32_t &A, uint32_t &B) {
    if constexpr (M == 1) {
        asm(DPP_ADD_NOP("quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf") : "=&v"(A) : "v"(x), "v"(ta));
        asm(DPP_ADD("quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf") : "=&v"(B) : "v"(x), "v"(tb));
    } else if constexpr (M == 2) {
        asm(DPP_ADD_NOP("quad_perm:[0,1,0,1] row_mask:0xf bank_mask:0xf") : "=&v"(A) : "v"(x), "v"(ta));
        asm(DPP_ADD("quad_perm:[2,3,2,3] row_mask:0xf bank_mask:0xf") : "=&v"(B) : "v"(x), "v"(tb));
    } else if constexpr (M == 16) {
        A = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x0F) + ta;
        B = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (0x10 << 5)) + tb;
    } else if constexpr (M == 4) {
        asm("v_add_u32 %0, %2, %3\n\tv_add_u32 %1, %2, %4\n\t"
            "v_add_u32_dpp %0, %2, %3 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
            "v_add_u32_dpp %1, %2, %4 row_shl:4 row_mask:0xf bank_mask:0x5"
            : "=&v"(A), "=&v"(B) : "v"(x), "v"(ta), "v"(tb));
    } else if constexpr (M == 8) {
        asm("v_add_u32 %0, %2, %3\n\tv_add_u32 %1, %2, %4\n\t"
            "v_add_u32_dpp %0, %2, %3 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
            "v_add_u32_dpp %1, %2, %4 row_shl:8 row_mask:0xf bank_mask:0x3"
            : "=&v"(A), "=&v"(B) : "v"(x), "v"(ta), "v"(tb));
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        A = r[0] + ta;
        B = r[1] + tb;
    }
}
// partner value x[lane ^ M] plus t (VAR 1/2), M < 32
template <int M, int VAR>
__device__ __forceinline__ uint32_t par_add(uint32_t x, uint32_t t) {
    if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false) + t;   // [1,0,3,2]
    else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false) + t;   // [2,3,0,1]
    else if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false) + t;  // row_ror:8
    else if constexpr (M == 4 && VAR == 2) {
        const int m = __builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);                          // row_half_mirror
        return (uint32_t)__builtin_amdgcn_update_dpp(0, m, 0x1B, 0xF, 0xF, false) + t;                         // [3,2,1,0]
    } else return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (M << 10)) + t;                        // xor M
}

template <int VAR>
__global__ __launch_bounds__(64, 8) void k_bench(uint32_t *out, const uint32_t *bmin, int trips) {
    const int lane = threadIdx.x;
    uint32_t t[12], c[6];
#pragma unroll
    for (int i = 0; i < 12; i++) t[i] = bmin[i * 64 + lane];
#pragma unroll
    for (int r = 0; r < 6; r++) c[r] = ((lane >> (5 - r)) & 1) ? 0x00010001u : 0u;
    // held in registers (an asm definition cannot be re-loaded inside the loop)
#pragma unroll
    for (int i = 0; i < 12; i++) asm volatile("" : "+v"(t[i]));
#pragma unroll
    for (int r = 0; r < 6; r++) asm volatile("" : "+v"(c[r]));
    uint32_t x = lane == 0 ? 0u : 0x003F003Fu, acc = 0;
    for (int it = 0; it < trips; it++) {
        uint32_t w = 0, w0 = 0, dp = 0;
        sfor<0, 30>([&](auto jc) {
            constexpr int j = decltype(jc)::value, rho = j % 6, M = 32 >> rho;
            if constexpr (VAR == 0) {
                uint32_t A, B;
                cand<M>(x, t[2 * rho], t[2 * rho + 1], A, B);
                const uint32_t d = as_u32(as_pk(B) - as_pk(A));
                x = as_u32(__builtin_elementwise_min(as_pk(A), as_pk(B)));
                if constexpr ((j & 1) == 0) dp = d;
                else {
                    uint32_t r;
                    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x01010101u << ((j >> 1) & 7)),
                        "v"(__builtin_amdgcn_perm(d, dp, 0x0B0A0908u)), "v"(w));
                    w = r;
                }
            } else {
                uint32_t xn;
                if constexpr (M == 32) {
                    auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
                    xn = as_u32(__builtin_elementwise_min(as_pk(r[0] + t[2 * rho]), as_pk(r[1] + t[2 * rho + 1])));
                } else {
                    const uint32_t co = x + t[2 * rho], cp = par_add<M, VAR>(x, t[2 * rho + 1]);
                    xn = as_u32(__builtin_elementwise_min(as_pk(co), as_pk(cp)));
                }
                // the next step's lane-type marker into the LSBs
                uint32_t r;
                asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x00010001u), "v"(c[(rho + 1) % 6]), "v"(xn));
                x = r;
                if constexpr ((j & 1) == 0) dp = xn;
                else {
                    uint32_t q, w2;
                    asm("v_add_u32 %0, %1, %1" : "=v"(w2) : "v"(w));                 // w << 1, full rate
                    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(q) : "s"(0x01010101u),
                        "v"(__builtin_amdgcn_perm(xn, dp, 0x06040200u)), "v"(w2));
                    w = q;
                }
            }
            if constexpr (j == 15) { w0 = w; w = 0; }
        });
        acc += __builtin_amdgcn_perm(w, w0, 0x06040200u) ^ __builtin_amdgcn_perm(w, w0, 0x07050301u);
    }
    out[blockIdx.x * 64 + lane] = acc ^ x;
}

int main() {
#pragma clang diagnostic ignored "-Wunused-result"
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int waves = ncu * 4 * 8 * 4, trips = 2000;
    uint32_t *out, *bm;
    hipMalloc(&out, sizeof(uint32_t) * 64 * waves);
    hipMalloc(&bm, sizeof(uint32_t) * 64 * 12);
    uint32_t h[64 * 12];
    for (int i = 0; i < 64 * 12; i++) h[i] = ((i * 2654435761u) >> 7) & 0x03FE03FEu;
    hipMemcpy(bm, h, sizeof h, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *name[3] = {"product (A/B, sub sign bits, perm+bfi)", "own/partner + LSB decision, M=4 swizzle",
                           "own/partner + LSB decision, M=4 two DPP"};
    for (int rep = 0; rep < 2; rep++)
        for (int v = 0; v < 3; v++) {
            auto k = v == 0 ? k_bench<0> : v == 1 ? k_bench<1> : k_bench<2>;
            hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, out, bm, 20);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, out, bm, trips);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double steps = (double)waves * trips * 30 / (ncu * 4);     // wave-steps per SIMD
            printf("VAR %d %-44s %8.3f ms  %.2f cycles per wave-step per SIMD at 2.4 GHz\n", v, name[v], ms,
                   ms * 1e-3 * 2.4e9 / steps);
        }
    return 0;
}
