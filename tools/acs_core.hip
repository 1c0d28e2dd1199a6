// acs_core.hip -- calibration microbenchmark (not part of the product): SIMD cycles per
// trellis step of variants of k_viterbi.hip's ACS word (acs_word_cw), branch metrics
// read from an LDS table per step exactly as k_acs reads them, no tile loader and no
// decision stores (the words are folded into a register).  8 waves per SIMD.
//   lane moves  (MV bit 0) M = 16/32 through the LDS crossbar (ds_swizzle / ds_bpermute)
//               instead of v_permlane16/32_swap; (bit 1) M = 4/8 through ds_swizzle
//               instead of 2 adds + 2 bank-masked DPP adds
//   decisions   DV 0: shift + v_bfi per step (k_acs); DV 1: two steps' sign bytes joined
//               by one v_perm, inserted by one v_bfi per pair
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <utility>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_pk(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ int rotl6(int x, int r) { return ((x << r) | (x >> (6 - r))) & 63; }
__device__ __forceinline__ int parity(int v) { return __popc(v) & 1; }
template <int I, int N, class F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}
constexpr int WS = 30, BRS = 122;

#define DPP_ADD(ctl) "v_add_u32_dpp %0, %1, %2 " ctl
#define DPP_ADD_NOP(ctl) "s_nop 1\n\tv_add_u32_dpp %0, %1, %2 " ctl
template <int M, int MV>
__device__ __forceinline__ void cand(uint32_t x, uint32_t ta, uint32_t tb, uint32_t &A, uint32_t &B, int lane) {
    if constexpr (M == 1) {
        asm(DPP_ADD_NOP("quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf") : "=&v"(A) : "v"(x), "v"(ta));
        asm(DPP_ADD("quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf") : "=&v"(B) : "v"(x), "v"(tb));
    } else if constexpr (M == 2) {
        asm(DPP_ADD_NOP("quad_perm:[0,1,0,1] row_mask:0xf bank_mask:0xf") : "=&v"(A) : "v"(x), "v"(ta));
        asm(DPP_ADD("quad_perm:[2,3,2,3] row_mask:0xf bank_mask:0xf") : "=&v"(B) : "v"(x), "v"(tb));
    } else if constexpr ((M == 4 || M == 8) && (MV & 2)) {
        constexpr int pa = 0x1F & ~M, pb = 0x1F | (M << 5);
        A = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, pa) + ta;
        B = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, pb) + tb;
    } else if constexpr (M == 4) {
        A = x + ta;
        B = x + tb;
        asm(DPP_ADD("row_shr:4 row_mask:0xf bank_mask:0xa") : "+v"(A) : "v"(x), "v"(ta));
        asm(DPP_ADD("row_shl:4 row_mask:0xf bank_mask:0x5") : "+v"(B) : "v"(x), "v"(tb));
    } else if constexpr (M == 8) {
        A = x + ta;
        B = x + tb;
        asm(DPP_ADD("row_shr:8 row_mask:0xf bank_mask:0xc") : "+v"(A) : "v"(x), "v"(ta));
        asm(DPP_ADD("row_shl:8 row_mask:0xf bank_mask:0x3") : "+v"(B) : "v"(x), "v"(tb));
    } else if constexpr (M == 16 && (MV & 1)) {
        A = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x0F) + ta;
        B = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x21F) + tb;
    } else if constexpr (M == 32 && (MV & 1)) {
        A = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (lane & 31), (int)x) + ta;
        B = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (lane | 32), (int)x) + tb;
    } else if constexpr (M == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        A = r[0] + ta;
        B = r[1] + tb;
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        A = r[0] + ta;
        B = r[1] + tb;
    }
}
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(a), "v"(b));
    return r;
}

template <int MV, int DV>
__device__ __forceinline__ void word(const uint32_t *bm, const uint32_t (&row)[6], uint32_t &x, uint32_t &c0,
                                     uint32_t &c1, int lane) {
    const uint32_t *rp[6];
#pragma unroll
    for (int r = 0; r < 6; r++) rp[r] = bm + row[r];
    uint32_t w = 0, w0 = 0, dprev = 0;
    sfor<0, WS>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int rho = j % 6;
        const uint2 t = *(const uint2 *)(rp[rho] + 2 * j);
        uint32_t A, B;
        cand<(32 >> rho), MV>(x, t.x, t.y, A, B, lane);
        const uint32_t d = as_u32(as_pk(B) - as_pk(A));
        if constexpr (DV == 0) {
            w = bfi(0x80008000u, d, w >> 1);
            if constexpr (j == WS / 2 - 1) w0 = w;
        } else {
            if constexpr ((j & 1) == 0) {
                dprev = d;
            } else {
                w = bfi(0x80808080u, __builtin_amdgcn_perm(d, dprev, 0x07050301u), w >> 1);
                if constexpr (j == 15) { w0 = w; w = 0; }
            }
        }
        x = as_u32(__builtin_elementwise_min(as_pk(A), as_pk(B)));
    });
    if constexpr (DV == 0) {
        c0 ^= ((w0 >> 1) & 0x7FFFu) | ((w << 14) & 0x3FFF8000u);
        c1 ^= ((w0 >> 17) & 0x7FFFu) | ((w >> 2) & 0x3FFF8000u);
    } else {
        c0 ^= __builtin_amdgcn_perm(w, w0, 0x06040200u);
        c1 ^= __builtin_amdgcn_perm(w, w0, 0x07050301u);
    }
    const uint32_t x0 = __builtin_amdgcn_readfirstlane(x);
    const uint32_t lo = x0 & 0xFFFFu, hi = x0 >> 16;
    const uint32_t c = (lo > 6120u ? lo - 6120u : 0u) | ((hi > 6120u ? hi - 6120u : 0u) << 16);
    x = as_u32(as_pk(x) - as_pk(c));
}

template <int MV, int DV>
__global__ __launch_bounds__(64, 8) void k_core(uint32_t *out, int iters) {
    __shared__ uint32_t bm[8 * BRS];
    const int lane = threadIdx.x;
    for (int i = lane; i < 8 * BRS; i += 64) bm[i] = ((i * 2654435761u) >> 7) & 0x01FF01FFu;
    __syncthreads();
    uint32_t row[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        const int i = rotl6(lane, r) & 31;
        const int q = parity((2 * i) & 0155) | (parity((2 * i) & 0117) << 1) | (parity((2 * i) & 0123) << 2);
        const bool upper = (lane >> (5 - r)) & 1;
        row[r] = (uint32_t)((upper ? q ^ 7 : q) * BRS);
    }
    uint32_t x = lane == 0 ? 0u : 0x003F003Fu, c0 = 0, c1 = 0;
    for (int it = 0; it < iters; it++) word<MV, DV>(bm, row, x, c0, c1, lane);
    out[blockIdx.x * 64 + lane] = x ^ c0 ^ c1;
}

template <int MV, int DV>
static void run(const char *name, int cus) {
    const int waves = cus * 32, iters = 2000;
    uint32_t *d;
    (void)hipMalloc(&d, sizeof(uint32_t) * waves * 64);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((k_core<MV, DV>), dim3(waves), dim3(64), 0, 0, d, 50);
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((k_core<MV, DV>), dim3(waves), dim3(64), 0, 0, d, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    const double wave_steps_per_simd = 8.0 * iters * WS;
    printf("%-52s %8.3f ms  %.1f cycles per wave-step per SIMD at 2.4 GHz\n", name, best,
           best * 1e-3 * 2.4e9 / wave_steps_per_simd);
    (void)hipFree(d);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    run<0, 0>("k_acs today (permlane swaps, bank-masked DPP, bfi/step)", cus);
    run<0, 1>("decisions by v_perm pairs", cus);
    run<1, 0>("M=16/32 via LDS crossbar", cus);
    run<2, 0>("M=4/8 via ds_swizzle", cus);
    run<1, 1>("M=16/32 LDS + perm pairs", cus);
    run<3, 0>("M=4..32 LDS", cus);
    run<3, 1>("M=4..32 LDS + perm pairs", cus);
    return 0;
}
