// dab_device.h -- device-side building blocks for the gfx950 DAB path:
// Mode-I constants, exact-rounding complex helpers, lane-exchange helpers
// and the wave64 2048-point FFT used by the sync, block-0 and demod kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "dab_kernels.h"

namespace dab {

// The 32 x 64 transpose inside fft2048 runs one column parity at a time, so the
// scratch holds 32 rows of 32 (+1 pad) float2: rows k1, column n2 >> 1.  Row
// stride 33 float2 = 66 dwords puts the 32 rows a reader lane set touches in
// distinct bank pairs (ds_read_b64: bank (a/4) mod 64).
constexpr int FFT_LDS_STRIDE = 33;
constexpr int FFT_LDS_FLOAT2 = 32 * FFT_LDS_STRIDE;     // 8,448 B per wave

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

__device__ __forceinline__ constexpr int brev5(int k) {
    return ((k & 1) << 4) | ((k & 2) << 2) | (k & 4) | ((k & 8) >> 2) | ((k & 16) >> 4);
}

// e^{-2 pi i m/32}, e^{-2 pi i m/64}: double-rounded-to-float literals
__device__ constexpr float kW32r[32] = {0x1.0000000000000p+0f, 0x1.f6297c0000000p-1f, 0x1.d906bc0000000p-1f, 0x1.a9b6620000000p-1f, 0x1.6a09e60000000p-1f, 0x1.1c73b40000000p-1f, 0x1.87de2a0000000p-2f, 0x1.8f8b840000000p-3f, 0x1.1a62640000000p-54f, -0x1.8f8b840000000p-3f, -0x1.87de2a0000000p-2f, -0x1.1c73b40000000p-1f, -0x1.6a09e60000000p-1f, -0x1.a9b6620000000p-1f, -0x1.d906bc0000000p-1f, -0x1.f6297c0000000p-1f, -0x1.0000000000000p+0f, -0x1.f6297c0000000p-1f, -0x1.d906bc0000000p-1f, -0x1.a9b6620000000p-1f, -0x1.6a09e60000000p-1f, -0x1.1c73b40000000p-1f, -0x1.87de2a0000000p-2f, -0x1.8f8b840000000p-3f, -0x1.a793940000000p-53f, 0x1.8f8b840000000p-3f, 0x1.87de2a0000000p-2f, 0x1.1c73b40000000p-1f, 0x1.6a09e60000000p-1f, 0x1.a9b6620000000p-1f, 0x1.d906bc0000000p-1f, 0x1.f6297c0000000p-1f};
__device__ constexpr float kW32i[32] = {-0x0.0p+0f, -0x1.8f8b840000000p-3f, -0x1.87de2a0000000p-2f, -0x1.1c73b40000000p-1f, -0x1.6a09e60000000p-1f, -0x1.a9b6620000000p-1f, -0x1.d906bc0000000p-1f, -0x1.f6297c0000000p-1f, -0x1.0000000000000p+0f, -0x1.f6297c0000000p-1f, -0x1.d906bc0000000p-1f, -0x1.a9b6620000000p-1f, -0x1.6a09e60000000p-1f, -0x1.1c73b40000000p-1f, -0x1.87de2a0000000p-2f, -0x1.8f8b840000000p-3f, -0x1.1a62640000000p-53f, 0x1.8f8b840000000p-3f, 0x1.87de2a0000000p-2f, 0x1.1c73b40000000p-1f, 0x1.6a09e60000000p-1f, 0x1.a9b6620000000p-1f, 0x1.d906bc0000000p-1f, 0x1.f6297c0000000p-1f, 0x1.0000000000000p+0f, 0x1.f6297c0000000p-1f, 0x1.d906bc0000000p-1f, 0x1.a9b6620000000p-1f, 0x1.6a09e60000000p-1f, 0x1.1c73b40000000p-1f, 0x1.87de2a0000000p-2f, 0x1.8f8b840000000p-3f};
__device__ constexpr float kW64r[64] = {0x1.0000000000000p+0f, 0x1.fd88da0000000p-1f, 0x1.f6297c0000000p-1f, 0x1.e9f4160000000p-1f, 0x1.d906bc0000000p-1f, 0x1.c38b300000000p-1f, 0x1.a9b6620000000p-1f, 0x1.8bc8060000000p-1f, 0x1.6a09e60000000p-1f, 0x1.44cf320000000p-1f, 0x1.1c73b40000000p-1f, 0x1.e2b5d40000000p-2f, 0x1.87de2a0000000p-2f, 0x1.2940620000000p-2f, 0x1.8f8b840000000p-3f, 0x1.917a6c0000000p-4f, 0x1.1a62640000000p-54f, -0x1.917a6c0000000p-4f, -0x1.8f8b840000000p-3f, -0x1.2940620000000p-2f, -0x1.87de2a0000000p-2f, -0x1.e2b5d40000000p-2f, -0x1.1c73b40000000p-1f, -0x1.44cf320000000p-1f, -0x1.6a09e60000000p-1f, -0x1.8bc8060000000p-1f, -0x1.a9b6620000000p-1f, -0x1.c38b300000000p-1f, -0x1.d906bc0000000p-1f, -0x1.e9f4160000000p-1f, -0x1.f6297c0000000p-1f, -0x1.fd88da0000000p-1f, -0x1.0000000000000p+0f, -0x1.fd88da0000000p-1f, -0x1.f6297c0000000p-1f, -0x1.e9f4160000000p-1f, -0x1.d906bc0000000p-1f, -0x1.c38b300000000p-1f, -0x1.a9b6620000000p-1f, -0x1.8bc8060000000p-1f, -0x1.6a09e60000000p-1f, -0x1.44cf320000000p-1f, -0x1.1c73b40000000p-1f, -0x1.e2b5d40000000p-2f, -0x1.87de2a0000000p-2f, -0x1.2940620000000p-2f, -0x1.8f8b840000000p-3f, -0x1.917a6c0000000p-4f, -0x1.a793940000000p-53f, 0x1.917a6c0000000p-4f, 0x1.8f8b840000000p-3f, 0x1.2940620000000p-2f, 0x1.87de2a0000000p-2f, 0x1.e2b5d40000000p-2f, 0x1.1c73b40000000p-1f, 0x1.44cf320000000p-1f, 0x1.6a09e60000000p-1f, 0x1.8bc8060000000p-1f, 0x1.a9b6620000000p-1f, 0x1.c38b300000000p-1f, 0x1.d906bc0000000p-1f, 0x1.e9f4160000000p-1f, 0x1.f6297c0000000p-1f, 0x1.fd88da0000000p-1f};
__device__ constexpr float kW64i[64] = {-0x0.0p+0f, -0x1.917a6c0000000p-4f, -0x1.8f8b840000000p-3f, -0x1.2940620000000p-2f, -0x1.87de2a0000000p-2f, -0x1.e2b5d40000000p-2f, -0x1.1c73b40000000p-1f, -0x1.44cf320000000p-1f, -0x1.6a09e60000000p-1f, -0x1.8bc8060000000p-1f, -0x1.a9b6620000000p-1f, -0x1.c38b300000000p-1f, -0x1.d906bc0000000p-1f, -0x1.e9f4160000000p-1f, -0x1.f6297c0000000p-1f, -0x1.fd88da0000000p-1f, -0x1.0000000000000p+0f, -0x1.fd88da0000000p-1f, -0x1.f6297c0000000p-1f, -0x1.e9f4160000000p-1f, -0x1.d906bc0000000p-1f, -0x1.c38b300000000p-1f, -0x1.a9b6620000000p-1f, -0x1.8bc8060000000p-1f, -0x1.6a09e60000000p-1f, -0x1.44cf320000000p-1f, -0x1.1c73b40000000p-1f, -0x1.e2b5d40000000p-2f, -0x1.87de2a0000000p-2f, -0x1.2940620000000p-2f, -0x1.8f8b840000000p-3f, -0x1.917a6c0000000p-4f, -0x1.1a62640000000p-53f, 0x1.917a6c0000000p-4f, 0x1.8f8b840000000p-3f, 0x1.2940620000000p-2f, 0x1.87de2a0000000p-2f, 0x1.e2b5d40000000p-2f, 0x1.1c73b40000000p-1f, 0x1.44cf320000000p-1f, 0x1.6a09e60000000p-1f, 0x1.8bc8060000000p-1f, 0x1.a9b6620000000p-1f, 0x1.c38b300000000p-1f, 0x1.d906bc0000000p-1f, 0x1.e9f4160000000p-1f, 0x1.f6297c0000000p-1f, 0x1.fd88da0000000p-1f, 0x1.0000000000000p+0f, 0x1.fd88da0000000p-1f, 0x1.f6297c0000000p-1f, 0x1.e9f4160000000p-1f, 0x1.d906bc0000000p-1f, 0x1.c38b300000000p-1f, 0x1.a9b6620000000p-1f, 0x1.8bc8060000000p-1f, 0x1.6a09e60000000p-1f, 0x1.44cf320000000p-1f, 0x1.1c73b40000000p-1f, 0x1.e2b5d40000000p-2f, 0x1.87de2a0000000p-2f, 0x1.2940620000000p-2f, 0x1.8f8b840000000p-3f, 0x1.917a6c0000000p-4f};

// ---- complex products with the reference's rounding (two products, one add;
// never fused) -- std::complex<float> operator* in a non-fast-math x86 build.
__device__ __forceinline__ float2 cmul_exact(float2 a, float2 b) {
#pragma clang fp contract(off)
    float ac = a.x * b.x, bd = a.y * b.y, ad = a.x * b.y, bc = a.y * b.x;
    return make_float2(ac - bd, ad + bc);
}
__device__ __forceinline__ float2 cmul_conj_exact(float2 a, float2 b) {   // a * conj(b)
#pragma clang fp contract(off)
    float nb = -b.y;
    float ac = a.x * b.x, bd = a.y * nb, ad = a.x * nb, bc = a.y * b.x;
    return make_float2(ac - bd, ad + bc);
}
// FFT-internal product (fused is fine inside the transform)
__device__ __forceinline__ float2 cmul(float2 a, float wr, float wi) {
    return make_float2(fmaf(a.x, wr, -a.y * wi), fmaf(a.x, wi, a.y * wr));
}

// ---- lane exchanges -------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dppu(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_XOR1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int DPP_XOR3 = 0x1B;        // quad_perm [3,2,1,0]
constexpr int DPP_ROR8 = 0x128;       // row_ror:8 == xor 8 inside a 16-lane row
constexpr int DPP_HMIRROR = 0x141;    // row_half_mirror: i -> 7-i inside 8 lanes

// value held by lane (lane ^ MASK)
template <int MASK>
__device__ __forceinline__ uint32_t xchg(uint32_t v, int lane) {
    if constexpr (MASK == 1) return dppu<DPP_XOR1>(v);
    else if constexpr (MASK == 2) return dppu<DPP_XOR2>(v);
    else if constexpr (MASK == 4) return dppu<DPP_XOR3>(dppu<DPP_HMIRROR>(v));
    else if constexpr (MASK == 8) return dppu<DPP_ROR8>(v);
    else if constexpr (MASK == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else {
        static_assert(MASK == 32, "xor mask");
        auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
}

__device__ __forceinline__ float wave_sum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ---- 32-point in-register DIF FFT: input natural order, X[k] ends in v[brev5(k)]
template <int M>
__device__ __forceinline__ float2 tw32(float2 d) {
    if constexpr (M == 0) return d;
    else if constexpr (M == 8) return make_float2(d.y, -d.x);           // * (-i)
    else return cmul(d, kW32r[M], kW32i[M]);
}
template <int LEN>
__device__ __forceinline__ void dif_stage(float2 (&v)[32]) {
    constexpr int H = LEN / 2;
    sfor<0, 32 / LEN>([&](auto sc) {
        constexpr int s = decltype(sc)::value * LEN;
        sfor<0, H>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            float2 a = v[s + j], b = v[s + j + H];
            v[s + j] = make_float2(a.x + b.x, a.y + b.y);
            v[s + j + H] = tw32<j * (32 / LEN)>(make_float2(a.x - b.x, a.y - b.y));
        });
    });
}
__device__ __forceinline__ void fft32(float2 (&v)[32]) {
    dif_stage<32>(v); __builtin_amdgcn_sched_barrier(0);
    dif_stage<16>(v); __builtin_amdgcn_sched_barrier(0);
    dif_stage<8>(v); __builtin_amdgcn_sched_barrier(0);
    dif_stage<4>(v); __builtin_amdgcn_sched_barrier(0);
    dif_stage<2>(v); __builtin_amdgcn_sched_barrier(0);
}

// ---- wave64 FFT of 2048 points, forward (e^{-j}), unscaled, in place.
// in : lane n2 holds x[n2 + 64*n1] in v[n1]
// out: lane L = (k1 = L>>1, r = L&1) holds X[k1 + 32*brev5(i) + 1024*r] in v[i]
//      (register slot i <-> k2 = brev5(i); tables indexed [i][lane] follow it)
// lds: FFT_LDS_FLOAT2 float2 of this wave's scratch.
// tw : per-lane twiddle bases, loaded once per kernel by load_twiddles():
//      A[a] = W2048^{n2*a} (a = 0..7), B[b] = W2048^{n2*8b} (b = 0..3), so that
//      W2048^{n2*k1} = A[k1&7] * B[k1>>3] with one rounding.
struct Twiddles {
    float2 A_[8], B_[4];
    __device__ __forceinline__ float2 A(int a) const { return A_[a]; }
    __device__ __forceinline__ float2 B(int b) const { return B_[b]; }
};
// the same bases read from a workgroup-shared LDS copy of the [12][64] table at
// each use (k_demod: keeps 24 VGPRs free for the previous symbol's spectrum)
struct TwiddlesLds {
    const float2 *t;        // table + lane
    __device__ __forceinline__ float2 A(int a) const { return t[a * 64]; }
    __device__ __forceinline__ float2 B(int b) const { return t[(8 + b) * 64]; }
};
__device__ __forceinline__ void load_twiddles(Twiddles &t, const float2 *__restrict__ tab, int lane) {
#pragma unroll
    for (int a = 0; a < 8; a++) t.A_[a] = tab[a * 64 + lane];                // rows 0..7: n2*a
#pragma unroll
    for (int b = 0; b < 4; b++) t.B_[b] = tab[(8 + b) * 64 + lane];          // rows 8..11: n2*8b
}
// per-lane select by a constant lane mask: lanes in MASK take b, the others a.
// As a v_cndmask on register values (a C select of two array elements may be
// folded into one load through a selected pointer, which demotes the array to
// scratch).
template <uint64_t MASK>
__device__ __forceinline__ float sel_lanes(float a, float b) {
    float d;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(MASK));
    return d;
}

// One column parity of the fft2048 transpose: lanes with r == PH write their 32
// values (column k1 = lane>>1 of every row), then take back their own row k1.
// Every lane issues the reads (no divergent branch: the register allocator would
// otherwise keep old and new values live together); the other parity keeps its
// registers through a select.
template <int PH>
__device__ __forceinline__ void fft_transpose_half(float2 (&v)[32], float2 *lds, int k1, int r) {
    if (r == PH) {
        sfor<0, 32>([&](auto kc) {
            constexpr int q = decltype(kc)::value;
            lds[q * FFT_LDS_STRIDE + k1] = v[brev5(q)];
        });
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float2 *row = lds + k1 * FFT_LDS_STRIDE;
    constexpr uint64_t MINE = PH ? 0xAAAAAAAAAAAAAAAAull : 0x5555555555555555ull;
    sfor<0, 32>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        const float2 t = row[m];
        v[m] = make_float2(sel_lanes<MINE>(v[m].x, t.x), sel_lanes<MINE>(v[m].y, t.y));
        if constexpr ((m & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class TW>
__device__ __forceinline__ void fft2048(float2 (&v)[32], float2 *lds, const TW &tw, int lane) {
    fft32(v);
    sfor<0, 32>([&](auto kc) {
        constexpr int k1 = decltype(kc)::value;
        constexpr int a = k1 & 7, b = k1 >> 3;
        float2 y = v[brev5(k1)];
        if constexpr (k1 != 0) {
            float2 w;
            if constexpr (a == 0) w = tw.B(b);
            else if constexpr (b == 0) w = tw.A(a);
            else {
                float2 ta = tw.A(a);
                asm volatile("" : "+v"(ta.x), "+v"(ta.y));   // keep the product in the loop (no LICM spill)
                const float2 tb = tw.B(b);
                w = cmul(ta, tb.x, tb.y);
            }
            y = cmul(y, w.x, w.y);
        }
        v[brev5(k1)] = y;
        if constexpr ((k1 & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    });
    // transpose: lane (k1 = lane>>1, r = lane&1) takes row k1, columns n2 = 2m + r.
    // Lanes of parity r write all their 32 values (column n2>>1 of every row) and
    // then read back their own row, so each phase frees exactly the registers it
    // refills and the scratch holds half the matrix.
    const int k1 = lane >> 1, r = lane & 1;
    fft_transpose_half<0>(v, lds, k1, r);
    fft_transpose_half<1>(v, lds, k1, r);
    fft32(v);
    const float sg = r ? -1.0f : 1.0f;
    sfor<0, 32>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int k2 = brev5(i);
        float2 u = v[i];
        float2 own = u;
        if constexpr (k2 != 0) {
            float2 t = cmul(u, kW64r[k2], kW64i[k2]);
            own = r ? t : u;
        }
        float rx = dppf<DPP_XOR1>(own.x), ry = dppf<DPP_XOR1>(own.y);
        v[i] = make_float2(fmaf(sg, own.x, rx), fmaf(sg, own.y, ry));
        if constexpr ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    });
}

// v_writelane through the LLVM intrinsic (no clang builtin in this toolchain)
extern "C" __device__ int llvm_amdgcn_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");

}  // namespace dab
