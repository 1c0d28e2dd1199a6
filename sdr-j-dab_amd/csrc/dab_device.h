// dab_device.h -- device-side building blocks for the gfx950 DAB path:
// compile-time loops, exact-rounding complex helpers and lane-exchange helpers
// (the workgroup FFT2048 is in k_demod.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "dab_kernels.h"

namespace dab {

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
// e^{2 pi i t / 2048000} in double from the factor tables (dab_kernels.h, NCO_*)
__device__ __forceinline__ double2 nco_value_d(const double2 *tab, int32_t t) {
#pragma clang fp contract(off)
    const uint32_t a = (uint32_t)t / 16000u;
    const uint32_t r = (uint32_t)t - a * 16000u;
    const double2 A = tab[a], B = tab[128 + (r >> 7)], C = tab[253 + (r & 127u)];
    const double pr = __builtin_fma(B.x, C.x, -(B.y * C.y));
    const double pi = __builtin_fma(B.x, C.y, B.y * C.x);
    const double vr = __builtin_fma(A.x, pr, -(A.y * pi));
    const double vi = __builtin_fma(A.x, pi, A.y * pr);
    return make_double2(vr, vi);
}
// oscillatorTable[t], bit-exact: the double value rounded to float
__device__ __forceinline__ float2 nco_value(const double2 *tab, int32_t t) {
    const double2 v = nco_value_d(tab, t);
    return make_float2((float)v.x, (float)v.y);
}
// ---- recorded-IQ sample formats read by the front-end kernels (dabgpu.h DABGPU_IQ_*):
// the conversion of the reference's file readers, exact in float, done in the load:
//   F32  interleaved cf32 as virtualInput::getSamples hands it over
//   S16  .sdr PCM16 (wavfiles.cpp:172, sf_readf_float: x / 32768)
//   U8   .raw (rawfiles.cpp:115-117: float(x - 128) / 128.0 = x / 128 - 1)
// raw: what a prefetch register holds (8, 4 or 2 bytes per sample); bps: bytes per sample.
// cvt: the sample as the reader hands it over; scaled: the same times 2^scale_exp (the
// integer the file holds, one instruction less per value: the demod keeps its samples,
// spectra and FreqCorr scaled by that power of two -- every float rounding commutes with it
// -- and unscales only what leaves it in absolute units); unscale = 2^-scale_exp.
template <int FMT> struct IqFmt;
template <> struct IqFmt<DABGPU_IQ_F32> {
    typedef float2 raw;
    static constexpr int bps = 8;
    static constexpr float unscale = 1.0f;
    __device__ static raw load(__amdgpu_buffer_rsrc_t r, int32_t off) {
        return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    }
    __device__ static float2 cvt(raw v) { return v; }
    __device__ static float2 scaled(raw v) { return v; }
};
template <> struct IqFmt<DABGPU_IQ_S16> {
    typedef uint32_t raw;
    static constexpr int bps = 4;
    static constexpr float unscale = 0x1p-15f;
    __device__ static raw load(__amdgpu_buffer_rsrc_t r, int32_t off) { return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0); }
    __device__ static float2 scaled(raw v) {
        return make_float2((float)(int32_t)(int16_t)(v & 0xFFFFu), (float)((int32_t)v >> 16));
    }
    __device__ static float2 cvt(raw v) {
        const float2 s = scaled(v);
        return make_float2(s.x * unscale, s.y * unscale);
    }
};
template <> struct IqFmt<DABGPU_IQ_U8> {
    typedef uint32_t raw;
    static constexpr int bps = 2;
    static constexpr float unscale = 0x1p-7f;
    __device__ static raw load(__amdgpu_buffer_rsrc_t r, int32_t off) { return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0); }
    __device__ static float2 scaled(raw v) {        // x - 128 (exact)
        return make_float2((float)(v & 0xFFu) - 128.0f, (float)((v >> 8) & 0xFFu) - 128.0f);
    }
    __device__ static float2 cvt(raw v) {
        // (float)(x - 128) / 128 == x * 2^-7 - 1 exactly (x < 256): one fma per value
        return make_float2(__builtin_fmaf((float)(v & 0xFFu), 0x1p-7f, -1.0f), __builtin_fmaf((float)((v >> 8) & 0xFFu), 0x1p-7f, -1.0f));
    }
};
// sample i of a stream starting at `base` (plain loads, for the kernels that gather)
template <int FMT>
__device__ __forceinline__ float2 iq_at(const void *base, int64_t i) {
    if constexpr (FMT == DABGPU_IQ_F32) return ((const float2 *)base)[i];
    else if constexpr (FMT == DABGPU_IQ_S16) return IqFmt<FMT>::cvt(((const uint32_t *)base)[i]);
    else return IqFmt<FMT>::cvt(((const uint16_t *)base)[i]);
}
template <int FMT>
__device__ __forceinline__ const void *iq_stream(const void *iq, int64_t base) {
    return (const char *)iq + base * IqFmt<FMT>::bps;
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

// v_writelane through the LLVM intrinsic (no clang builtin in this toolchain)
extern "C" __device__ int llvm_amdgcn_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");

}  // namespace dab
