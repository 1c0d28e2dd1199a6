// k_demod.hip -- the OFDM front end of a frame on one 256-thread workgroup, gfx950:
//   k_demod_wg<GEN, SYNC>  phaseReference::findIndex (phasereference.cpp:60-88, SYNC),
//                          get_snr of block 0 (ofdm-decoder.cpp:212-230) and
//                          ofdmDecoder::processToken x 75 (ofdm-decoder.cpp:167-190)
//                          + the FreqCorr guard correlation (ofdm-processor.cpp:424-438)
//   k_prs_wg<GEN>          findIndex alone (frames whose block 0 the host must see first)
//   k_block0_wg<GEN>       ofdmDecoder::processBlock_0 (ofdm-decoder.cpp:85-162): get_snr
//                          and the coarse offset, freqSyncMethod 0, 1 or 2
//
// One workgroup of 256 threads (4 waves) per (frame, chunk of symbols).  The
// 2048-point FFT of a symbol is shared by the workgroup, 8 points per thread:
//   pass 1  n = t + 256 m        radix-8 over m, twiddle W2048^(t k1)  -> LDS
//   pass 2  t = t' + 32 m        radix-8 over m, twiddle W256^(t' k2)  -> LDS
//   pass 3  t' = t'' + 4 m       radix-8 over m, twiddle W32^(t'' k3)  (registers)
//   pass 4  radix-4 over t'' across the 4 lanes of a quad (DPP, no LDS)
// after which thread t (quad g = t>>2 = 8 k1 + k2, t'' = t&3) holds
// X[k1 + 8 k2 + 64 k3 + 512 brev2(t'')] for k3 = 0..7.  About 110 VGPRs per thread
// (4 waves per SIMD) instead of a whole FFT per wave: the next symbol's samples are
// loaded into registers while the current one is transformed, and enough waves are
// resident to cover HBM latency -- the kernel streams at the HBM roofline's pace.
// DQPSK (r = X conj(P), q = -re/(|re|+|im|), int16 (q*127)) runs on the thread's own
// bins; the previous symbol's bins stay in its registers.  Soft bits leave through a
// 6 KB LDS stage as coalesced 8-byte stores.
#include "dab_device.h"
#include "dab_kernels.h"

namespace dab {

constexpr int DT = 256;                 // threads per demod workgroup
constexpr int ZROW = 36;                // pass-2 output rows of 32 (+4 pad: conflict-free pass-3 reads)
constexpr int EXN = 2048 + 64 * (ZROW - 32);   // FFT exchange buffer (float2)
#ifndef DEMOD_WG_PER_SIMD
#define DEMOD_WG_PER_SIMD 4     // resident workgroups per CU (= waves per SIMD): <= 128 VGPRs, <= 40 KB LDS
#endif

__device__ __forceinline__ int32_t nco_index2(int32_t lp0, int32_t phase, int64_t j) {
    int64_t t = ((int64_t)lp0 - j * (int64_t)phase) % INPUT_RATE;
    return (int32_t)(t < 0 ? t + INPUT_RATE : t);
}
__device__ __forceinline__ int32_t nco_mod(int64_t v) {
    const int64_t t = v % INPUT_RATE;
    return (int32_t)(t < 0 ? t + INPUT_RATE : t);
}
// x - d, x + d mod INPUT_RATE for x, d in [0, INPUT_RATE)
__device__ __forceinline__ int32_t nco_sub(int32_t x, int32_t d) {
    x -= d;
    return x < 0 ? x + INPUT_RATE : x;
}
__device__ __forceinline__ int32_t nco_add(int32_t x, int32_t d) {
    x += d;
    return x >= INPUT_RATE ? x - INPUT_RATE : x;
}
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// (int16_t)(q * 127.0) exactly as the reference computes it: q promoted to double
// (ofdm-decoder.cpp:188-189): 3 instructions (cvt, mul_f64, truncating cvt)
__device__ __forceinline__ int trunc127d(float q) { return (int)((double)q * 127.0); }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmulw(float2 a, float2 w) { return cmul(a, w.x, w.y); }

// forward 8-point DFT in place, natural order in and out (radix-2 DIF, W8 = e^{-j pi/4})
__device__ __forceinline__ void dft8(float2 (&a)[8]) {
    constexpr float c = 0.70710678118654752440f;
    float2 b[8];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        b[j] = cadd(a[j], a[j + 4]);
        b[j + 4] = csub(a[j], a[j + 4]);
    }
    b[5] = make_float2(c * (b[5].x + b[5].y), c * (b[5].y - b[5].x));        // * W8^1
    b[6] = make_float2(b[6].y, -b[6].x);                                     // * W8^2 = -j
    b[7] = make_float2(c * (b[7].y - b[7].x), -c * (b[7].x + b[7].y));       // * W8^3
    float2 d[8];
#pragma unroll
    for (int h = 0; h < 8; h += 4) {
        d[h + 0] = cadd(b[h + 0], b[h + 2]);
        d[h + 1] = cadd(b[h + 1], b[h + 3]);
        d[h + 2] = csub(b[h + 0], b[h + 2]);
        const float2 t = csub(b[h + 1], b[h + 3]);
        d[h + 3] = make_float2(t.y, -t.x);                                   // * W4^1 = -j
    }
    // last radix-2 stage; DIF output index = brev3(position)
    a[0] = cadd(d[0], d[1]);
    a[4] = csub(d[0], d[1]);
    a[2] = cadd(d[2], d[3]);
    a[6] = csub(d[2], d[3]);
    a[1] = cadd(d[4], d[5]);
    a[5] = csub(d[4], d[5]);
    a[3] = cadd(d[6], d[7]);
    a[7] = csub(d[6], d[7]);
}

// radix-2 butterfly across lanes at xor distance M inside a quad:
// lanes with bit M clear get v + partner, lanes with it set get partner - v
// (a DPP move + fma; a v_mul + v_add_f32_dpp form measured 2 % slower in this kernel)
template <int M>
__device__ __forceinline__ float quad_bfly(float v, float sign) {
    constexpr int ctrl = M == 2 ? 0x4E : 0xB1;          // quad_perm [2,3,0,1] / [1,0,3,2]
    // every quad_perm source lane exists: bound_ctrl with full masks, so no old value
    // (a zeroed destination per move) is needed
    const float p = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), ctrl, 0xF, 0xF, true));
    return fmaf(sign, v, p);
}

// the same butterfly with the lane's sign on the partner: own + sign * partner (upper lanes
// get minus the butterfly's value; fft2048_wg<true> tracks that sign as tw.tau)
// The compiler does not fold a DPP move into v_fmac_f32 (it folds add / mul), so the fused
// form is written out: v_fmac_f32_dpp acc = dpp(src) * sign + acc with acc = src = v, one
// VALU instead of a DPP move and an fma, the same single rounding.  The s_nop 1 is the two
// wait states a DPP read needs after the VALU write of its source (the hazard recognizer
// does not look inside inline assembly).
// (GFX9 DPP syntax and wait states: gfx942 / gfx950 only; elsewhere -- and in the host
// pass -- the same value as a DPP move and an fma.  Not volatile: the asm has no side
// effect beyond its output, so the compiler may schedule around it.)
template <int M>
__device__ __forceinline__ float quad_bfly_s(float v, float sign) {
#if defined(__gfx950__) || defined(__gfx942__)
    float r;
    if constexpr (M == 2)
        asm("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1"
            : "=v"(r) : "v"(v), "v"(sign), "0"(v));
    else
        asm("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1"
            : "=v"(r) : "v"(v), "v"(sign), "0"(v));
    return r;
#else
    constexpr int ctrl = M == 2 ? 0x4E : 0xB1;
    const float p = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), ctrl, 0xF, 0xF, true));
    return fmaf(p, sign, v);
#endif
}

// v[m] *= oscillatorTable[localPhase] sample by sample (ofdm-processor.cpp:186-201).
// GEN: localPhase steps by -phase per sample, the table rebuilt from the factor tables
// in LDS (nco_value; the 16 MB table itself would cost a cache line per sample);
// otherwise phase == 0 and every sample uses oscillatorTable[lp0].
template <bool GEN>
__device__ __forceinline__ void mix(float2 (&v)[8], const float2 *__restrict__ osc, const double2 *ncl, int32_t lp0,
                                   int32_t phase, int64_t first, int64_t origin) {
    // v[m] = sample first + 256 m of a getSamples segment that started at `origin`
    if (!GEN || phase == 0) {
        const float2 f = osc[lp0];
#pragma unroll
        for (int m = 0; m < 8; m++) v[m] = cmul_exact(v[m], f);
    } else {
        int32_t t = nco_index2(lp0, phase, first - origin + 1);
        const int32_t step = (int32_t)((((int64_t)256 * phase) % INPUT_RATE + INPUT_RATE) % INPUT_RATE);
#pragma unroll
        for (int m = 0; m < 8; m++) {
            v[m] = cmul_exact(v[m], nco_value(ncl, t));
            t -= step;
            if (t < 0) t += INPUT_RATE;
        }
    }
}
template <bool GEN>
__device__ __forceinline__ float2 mix1(float2 v, const float2 *__restrict__ osc, const double2 *ncl, int32_t lp0,
                                       int32_t phase, int64_t pos, int64_t origin) {
    if (!GEN || phase == 0) return cmul_exact(v, osc[lp0]);
    return cmul_exact(v, nco_value(ncl, nco_index2(lp0, phase, pos - origin + 1)));
}
// the factor tables into LDS (GEN kernels only; callers __syncthreads before use)
template <bool GEN>
__device__ __forceinline__ void nco_setup(double2 *ncl, const OfdmTables &T, int t) {
    if constexpr (GEN)
        for (int i = t; i < NCO_USED; i += DT) ncl[i] = T.nco[i];
}

struct DemodTw {
    const float2 *w1;             // LDS table W2048^(t k) at [(k - 1) * 256 + t], k = 1..7
    const float2 *w2;             // LDS table W256^(t' k) at [(k - 1) * 32 + t']: consecutive lanes, no bank conflicts
    const float2 *w3;             // LDS table W32^(t'' k) at [(k - 1) * 4 + t'']: a quad's 4 values in 4 different banks
    float sg2, sg1;               // quad butterfly signs (+1 lower lane, -1 upper)
    float tau;                    // fft2048_wg<true>'s output sign of this lane (t'' = 1, 2: -1)
    bool rot;                     // lane t'' == 3 multiplies by -j between the two stages
};

// the FFT of the 8 samples a[] (n = t + 256 m) of every thread; ex: 2048 + pad float2 of LDS.
// SIGNED: each lane's outputs come out times tw.tau (+-1, exact): pass 4's butterflies then
// take the partner's value as the fma's multiplicand (own + sign * partner), which the
// compiler folds into one v_fmac_f32_dpp per value and stage instead of a DPP move and an
// fma.  For DQPSK the sign cancels (X_l conj(X_{l-1}) with both scaled by the same tau: the
// same products, bit for bit), and |X| is unchanged; the callers that need X itself use
// SIGNED = false.
// passes 1-3 of fft2048_wg: afterwards thread t (quad g = t >> 2, t'' = t & 3) holds in a[k3]
// the radix-4 input t'' of group (g, k3), twiddled by W32^(t'' k3)
__device__ __forceinline__ void fft2048_p123(float2 (&a)[8], float2 *ex, const DemodTw &tw, int t) {
    // pass 1
    dft8(a);
#pragma unroll
    for (int k = 1; k < 8; k++) a[k] = cmulw(a[k], tw.w1[(k - 1) * DT + t]);
#pragma unroll
    for (int k = 0; k < 8; k++) ex[k * 256 + t] = a[k];
    __syncthreads();
    // pass 2: k1 = t >> 5, t' = t & 31
    const int k1 = t >> 5, tp = t & 31;
#pragma unroll
    for (int m = 0; m < 8; m++) a[m] = ex[k1 * 256 + tp + 32 * m];
    __syncthreads();
    dft8(a);
#pragma unroll
    for (int k = 1; k < 8; k++) a[k] = cmulw(a[k], tw.w2[(k - 1) * 32 + tp]);
#pragma unroll
    for (int k = 0; k < 8; k++) ex[(k1 * 8 + k) * ZROW + tp] = a[k];
    __syncthreads();
    // pass 3: g = t >> 2 (= 8 k1 + k2), t'' = t & 3
    const int g = t >> 2, tq = t & 3;
#pragma unroll
    for (int m = 0; m < 8; m++) a[m] = ex[g * ZROW + tq + 4 * m];
    dft8(a);
    if (tq) {                                      // t'' = 0: all twiddles 1
#pragma unroll
        for (int k = 1; k < 8; k++) a[k] = cmulw(a[k], tw.w3[(k - 1) * 4 + tq]);
    }
}
template <bool SIGNED = false>
__device__ __forceinline__ void fft2048_wg(float2 (&a)[8], float2 *ex, const DemodTw &tw, int t) {
    fft2048_p123(a, ex, tw, t);
    // pass 4: radix-4 over the quad's t''; lane t'' ends with K'' = brev2(t'')
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if constexpr (SIGNED) {
            float2 v = make_float2(quad_bfly_s<2>(a[k].x, tw.sg2), quad_bfly_s<2>(a[k].y, tw.sg2));
            if (tw.rot) v = make_float2(v.y, -v.x);
            a[k] = make_float2(quad_bfly_s<1>(v.x, tw.sg1), quad_bfly_s<1>(v.y, tw.sg1));
        } else {
            float2 v = make_float2(quad_bfly<2>(a[k].x, tw.sg2), quad_bfly<2>(a[k].y, tw.sg2));
            if (tw.rot) v = make_float2(v.y, -v.x);
            a[k] = make_float2(quad_bfly<1>(v.x, tw.sg1), quad_bfly<1>(v.y, tw.sg1));
        }
    }
}


// The data symbols' FFT tail (round 6, k_demod_wg): instead of pass 4's DPP radix-4 across
// the quad, pass 3's outputs go through LDS inside the quad that produced them -- the 4
// values t'' = 0..3 of group (g, k3) at ex[g * ZROW + 4 k3 + t''], i.e. row g, which only
// quad g reads or writes from pass 3 on (each lane overwrites the entries it read in pass 3),
// so the wave's own program order is all the ordering needed -- and thread t = 4 g + a takes
// the groups (g, a) and (g, a + 4): the radix-4 over t'' in registers, with the same
// operations as pass 4 (x0 +- x2, x1 +- x3, -j, then the sums: the spectrum bit for bit).
// Of a group's outputs X[K''] (bin b0(g) + 64 k3 + 512 K''), K'' = 0 and 3 are carriers
// (bins 1..511, 1536..2047), K'' = 1 only for k3 <= 3 (512..767) and K'' = 2 only for
// k3 >= 4 (1280..1535): every thread holds exactly 6 carriers -- thread 0 the carrier at
// bin 768 (group (0, 4), K'' = 1) in place of the DC bin -- so DQPSK and the soft bits run
// on 6 slots, not 8 bins.
struct Quad4 { float2 s02, d02, s13, d13; };
__device__ __forceinline__ float2 rotmj(float2 d) { return make_float2(d.y, -d.x); }      // -j d
__device__ __forceinline__ Quad4 r4_terms(const float2 (&x)[4]) {
    return {cadd(x[0], x[2]), csub(x[0], x[2]), cadd(x[1], x[3]), csub(x[1], x[3])};
}
// X[K''] of a group: X0 = s02 + s13, X1 = d02 - j d13, X2 = s02 - s13, X3 = d02 + j d13
__device__ __forceinline__ float2 r4_out(const Quad4 &q, int K) {
    return K == 0 ? cadd(q.s02, q.s13) : K == 1 ? cadd(q.d02, rotmj(q.d13)) : K == 2 ? csub(q.s02, q.s13)
                                                                             : csub(q.d02, rotmj(q.d13));
}
__device__ __forceinline__ void fft2048_tail(const float2 (&a)[8], float2 *ex, int t, Quad4 &qa, Quad4 &qb) {
    const int g = t >> 2, tq = t & 3;
    float2 *row = ex + g * ZROW;
    float2 xa[4], xb[4];
    // (k3, t'') at row[8 t'' + k3]: a lane's 8 values contiguous (4 b128 stores), the groups
    // read as 8 b64 loads whose 32-lane halves hit 64 distinct banks (72 g + 16 u + 2 a
    // words).  (The layout row[4 k3 + t''] -- 8 b64 stores, 4 b128 loads -- measured the same,
    // profiles/r06_demod_tail_ab.txt.)
    float4 *w = (float4 *)(row + 8 * tq);
#pragma unroll
    for (int k = 0; k < 8; k += 2) w[k >> 1] = make_float4(a[k].x, a[k].y, a[k + 1].x, a[k + 1].y);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int u = 0; u < 4; u++) {
        xa[u] = row[8 * u + tq];
        xb[u] = row[8 * u + tq + 4];
    }
    qa = r4_terms(xa);
    qb = r4_terms(xb);
}
// the FFT bin of output (group grp = 0: k3 = a, 1: k3 = a + 4; K'') of thread t
__device__ __forceinline__ int tail_bin(int t, int grp, int K) {
    const int g = t >> 2, a = t & 3;
    return (g >> 3) + 8 * (g & 7) + 64 * (a + 4 * grp) + 512 * K;
}
// slot j -> (group, K''): A0 A1 A3 B0 B2 B3 (thread 0: B1 for A0)
__device__ __forceinline__ int slot_bin(int t, int j) {
    constexpr int grp[6] = {0, 0, 0, 1, 1, 1}, kk[6] = {0, 1, 3, 0, 2, 3};
    return (t == 0 && j == 0) ? tail_bin(t, 1, 1) : tail_bin(t, grp[j], kk[j]);
}
__device__ __forceinline__ void tail_slots(const Quad4 &A, const Quad4 &B, int t, float2 (&S)[6]) {
    S[0] = r4_out(A, 0);
    S[1] = r4_out(A, 1);
    S[2] = r4_out(A, 3);
    S[3] = r4_out(B, 0);
    S[4] = r4_out(B, 2);
    S[5] = r4_out(B, 3);
    if (__builtin_amdgcn_readfirstlane(t) < 64) {      // wave 0 (uniform): thread 0's carrier 768
        const float2 b1 = r4_out(B, 1);
        if (t == 0) S[0] = b1;
    }
}
// all 8 outputs (get_snr, the display feed, the test hook): X[4 grp + K''] at tail_bin(t, grp, K'')
__device__ __forceinline__ void tail_all(const Quad4 &A, const Quad4 &B, float2 (&X)[8]) {
#pragma unroll
    for (int K = 0; K < 4; K++) {
        X[K] = r4_out(A, K);
        X[4 + K] = r4_out(B, K);
    }
}

// twiddle tables of fft2048_wg in LDS, laid out per pass so that a wave's reads are
// conflict-free (the values are the W2048 table's entries: W256^j = W2048^(8 j),
// W32^j = W2048^(64 j))
struct TwLds {
    float2 w1[7 * DT];      // pass 1: LDS instead of 14 VGPRs (room for the guard prefetch)
    float2 w2[7 * 32];
    float2 w3[7 * 4];
};
__device__ __forceinline__ DemodTw tw_setup(TwLds &L, const OfdmTables &T, int t) {
#pragma unroll
    for (int k = 1; k < 8; k++) L.w1[(k - 1) * DT + t] = T.w2048[(t * k) & 2047];
    if (t < 7 * 32) L.w2[t] = T.w2048[(8 * ((t & 31) * (t / 32 + 1))) & 2047];
    if (t < 7 * 4) L.w3[t] = T.w2048[(64 * ((t & 3) * (t / 4 + 1))) & 2047];
    DemodTw tw;
    const int tq = t & 3;
    tw.w1 = L.w1;
    tw.w2 = L.w2;
    tw.w3 = L.w3;
    tw.sg2 = (tq & 2) ? -1.0f : 1.0f;
    tw.sg1 = (tq & 1) ? -1.0f : 1.0f;
    tw.tau = (tq == 1 || tq == 2) ? -1.0f : 1.0f;
    tw.rot = tq == 3;
    return tw;
}
// FFT bin held in a[k3] by thread t after fft2048_wg
__device__ __forceinline__ int bin0_of(int t) {
    const int g = t >> 2, tq = t & 3, k1 = g >> 3, k2 = g & 7;
    return k1 + 8 * k2 + 512 * (((tq & 1) << 1) | (tq >> 1));
}

// workgroup reductions (4 waves): sum of floats; max with the lowest index on ties
struct RedLds {
    float f[2 * (DT / 64)];
    int32_t i[DT / 64];
};
__device__ __forceinline__ float wg_sum(float v, RedLds &R, int t, int slot) {
    v = wave_sum(v);
    if ((t & 63) == 0) R.f[slot * (DT / 64) + (t >> 6)] = v;
    __syncthreads();
    float r = R.f[slot * (DT / 64)];
#pragma unroll
    for (int w = 1; w < DT / 64; w++) r += R.f[slot * (DT / 64) + w];
    return r;
}
__device__ __forceinline__ void wg_argmax(float &best, int &bidx, RedLds &R, int t) {
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bidx, o);
        if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
    }
    __syncthreads();
    if ((t & 63) == 0) { R.f[t >> 6] = best; R.i[t >> 6] = bidx; }
    __syncthreads();
    best = R.f[0];
    bidx = R.i[0];
#pragma unroll
    for (int w = 1; w < DT / 64; w++)
        if (R.f[w] > best || (R.f[w] == best && R.i[w] < bidx)) { best = R.f[w]; bidx = R.i[w]; }
}

// findIndex (phasereference.cpp:60-88) of the T_u window in a[] (n = t + 256 m, mixed):
// X = FFT(x); r = IFFT(X conj(ref)) = conj(FFT(conj(X conj(ref)))) / 2048; argmax |r|
// with the first index on ties; -|Max / mean| - 1 when Max < level * mean.
// Returns startIndex on every thread.
__device__ __forceinline__ int32_t prs_corr_wg(float2 (&a)[8], float2 *ex, const DemodTw &tw, int t,
                                               const float2 *__restrict__ ref, int level, RedLds &R,
                                               float &maxv, float &sumv) {
    fft2048_wg(a, ex, tw, t);
    const int b0 = bin0_of(t);
    __syncthreads();                                     // pass 3 of the FFT read ex
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int b = b0 + 64 * k;
        const float2 r = cmul_conj_exact(a[k], ref[b]);
        ex[b] = make_float2(r.x, -r.y);
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; m++) a[m] = ex[t + 256 * m];
    __syncthreads();
    fft2048_wg(a, ex, tw, t);
    constexpr float scale = 1.0f / 2048.0f;            // common_ifft::Scale (fft.cpp:115-121), exact
    float sum = 0.0f, best = -10000.0f;
    int bidx = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < 8; k++) {                        // increasing time index per thread
        const float v = hypotf(a[k].x * scale, -a[k].y * scale);
        sum += v;
        if (v > best) { best = v; bidx = b0 + 64 * k; }
    }
    sum = wg_sum(sum, R, t, 1);
    wg_argmax(best, bidx, R, t);
    maxv = best;
    sumv = sum;
    if (best < (float)level * sum / 2048.0f) return (int32_t)(-fabsf(best / (sum / 2048.0f)) - 1.0f);
    return bidx;
}

// get_snr (ofdm-decoder.cpp:212-230) of the block-0 spectrum in a[] (bins b0 + 64 k):
// noise = mean |X| over bins 1034..1259 and 788..1013, signal = mean over 1664..2047 and
// 0..383; get_db(signal) - get_db(noise) with get_db(x) = 20 log10((x + 1) / 256)
// (dab-constants.h:107-109).  The sums are workgroup trees (the reference adds in bin
// order): a display value, equal to the sequential one except within float rounding
// of a dB boundary.
template <class BinOf>
__device__ __forceinline__ int16_t snr_wg_b(const float2 (&a)[8], BinOf bin_of, RedLds &R, int t, float unscale) {
    float noise = 0.0f, signal = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int b = bin_of(k);
        const float v = hypotf(a[k].x * unscale, a[k].y * unscale);      // (a power of two: exact)
        if ((b >= 1034 && b < 1260) || (b >= 788 && b < 1014)) noise += v;
        if (b >= 1664 || b < 384) signal += v;
    }
    noise = wg_sum(noise, R, t, 0);
    __syncthreads();
    signal = wg_sum(signal, R, t, 1);
    noise /= 452;
    const float db_s = 20 * log10f((signal / 768 + 1) / (float)256);
    const float db_n = 20 * log10f((noise + 1) / (float)256);
    return (int16_t)(db_s - db_n);
}
__device__ __forceinline__ int16_t snr_wg(const float2 (&a)[8], int t, RedLds &R, float unscale = 1.0f) {
    const int b0 = bin0_of(t);
    return snr_wg_b(a, [&](int k) { return b0 + 64 * k; }, R, t, unscale);
}

// (int16_t)((double)q * 127.0) for q = RN(-re / ab1) and the same for im -- the
// reference's soft bit (ofdm-decoder.cpp:188-189) -- without two IEEE divisions on the
// common path.  x' = re * (rcp(ab1) * -127) is within 127 * 2^-22 (rcp 1 ulp, two
// roundings) + 127 * 2^-25 (the rounding of q itself) < D of the exact 127 q, so its
// truncation (v_cvt_i32_f32 truncates) equals the reference's unless x' lies within D
// of an integer.  Those values (about 1 in 10^4, zero included) and operands outside
// the reciprocal's comfortable range take the exact path: IEEE division, double product.
// BOUNDED: the samples are integers of a recorded format (|x| <= 2^15), so ab1 < 2^55 and
// the reciprocal never leaves the normal range on the large side; ab1 = 0 (or a denormal
// the reciprocal flushes) makes x' inf or NaN, so e is NaN and !(e >= D) takes the exact
// path -- the range compare is only needed for cf32 input of arbitrary magnitude
template <bool BOUNDED = false>
__device__ __forceinline__ bool soft_fast(float2 r1, float ab1, int &ir, int &ii) {
#pragma clang fp contract(off)
    constexpr float D = 0x1p-14f;
    const float m = __builtin_amdgcn_rcpf(ab1) * -127.0f;
    const float xr = r1.x * m, xi = r1.y * m;
    const float e = fminf(fabsf(xr - rintf(xr)), fabsf(xi - rintf(xi)));
    ir = (int)xr;
    ii = (int)xi;
    if constexpr (BOUNDED) {
        return !(e >= D);
    } else {
        // ab1 (>= 0 or NaN) outside [2^-100, 2^100]: one unsigned compare on its bits
        const bool range = (__float_as_uint(ab1) - 0x0D800000u) > 0x64000000u;
        return e < D || range;
    }
}
__device__ __forceinline__ void soft_pair(float2 r1, float ab1, int &ir, int &ii) {
    if (soft_fast(r1, ab1, ir, ii)) {
        ir = trunc127d(-r1.x / ab1);
        ii = trunc127d(-r1.y / ab1);
    }
}

// The soft bits of symbol l leave through an LDS stage of 1536 {re, im} int16 pairs
// (one 32-bit write per carrier), read back by carrier quads (two 8-byte pair reads) and
// stored as re / im groups: output rows stay [3072] = re[1536] | im[1536].  The stage
// keeps carriers in pairs at host-chosen words (T.stage_of_bin, T.stage_pair;
// stage_layout.h): the de-interleave's scattered stores then hit distinct banks in each
// 32-lane half (3 two-way collisions per symbol, the lower bound, instead of 158 extra
// cycles), and each pair read covers the 64 banks.  Bins that carry nothing write to 32
// dump words, each store half-wave's at banks its carriers leave free.
constexpr int STG = K + 32;

template <bool GEN, bool SYNC, bool R8, int FMT, bool DUMP>
__global__ __launch_bounds__(DT, DEMOD_WG_PER_SIMD) void k_demod_wg(const void *__restrict__ iq,
                                                    const dabgpu_frame *__restrict__ frames, int nchunks,
                                                    OfdmTables T, int16_t *__restrict__ soft,
                                                    float *__restrict__ softf, float2 *__restrict__ fcpart,
                                                    DemodAux aux) {
    __shared__ __attribute__((aligned(16))) float2 ex[EXN];
    // the soft-bit stage and the FreqCorr partials reuse the FFT exchange buffer (after
    // the FFT's last LDS pass, behind a barrier): 34 KB per workgroup
    uint32_t *st = (uint32_t *)ex;
    static_assert(STG * 4 <= sizeof(ex), "stage fits the exchange buffer");
    float2 *fcw = ex;
    __shared__ TwLds twl;
    __shared__ RedLds red;
    const int t = threadIdx.x;
    // the NCO factor tables are read from global memory (6 KB, cache-resident): the symbol
    // loop's recurrences need them only at a chunk's start, and 6 KB less LDS per workgroup
    // (34 KB) leaves room on a CU beside four workgroups for a traceback wave
    const double2 *ncl = T.nco;
    const DemodTw tw = tw_setup(twl, T, t);
    __syncthreads();
    const int item = blockIdx.x;
    const int fi = item / nchunks, ch = item % nchunks;
    dabgpu_frame fr = frames[fi];
    const void *s = iq_stream<FMT>(iq, fr.iq_base);
    using Fmt = IqFmt<FMT>;
    constexpr int BPS = Fmt::bps;
    bool skip = false;
    if constexpr (SYNC) {
        // the frame starts where findIndex finds it (block0 = window + startIndex,
        // ofdm-processor.cpp:344-368): every chunk of the frame correlates the window
        // itself, chunk 0 reports.  A frame whose sync fails, or whose symbols are not
        // all there yet, is skipped (the host's replay does not commit it).
        if (fr.window < 0 || fr.window + TU > fr.n_samples || fr.lp_window < 0 || fr.lp_window >= INPUT_RATE) {
            if (t == 0) {
                atomicOr(T.err, KERR_FRAME);
                if (ch == 0) aux.si[fi] = -1;
            }
            skip = true;
        } else {
            float2 a[8];
#pragma unroll
            for (int m = 0; m < 8; m++) a[m] = iq_at<FMT>(s, fr.window + t + 256 * m);
            mix<GEN>(a, T.osc, ncl, fr.lp_window, fr.phase_a, fr.window + t, fr.window);
            float mx, sm;
            const int32_t si = prs_corr_wg(a, ex, tw, t, T.ref, aux.level, red, mx, sm);
            if (ch == 0 && t == 0) {
                aux.si[fi] = si;
                if (aux.maxv) aux.maxv[fi] = mx;
                if (aux.sumv) aux.sumv[fi] = sm;
            }
            if (si < 0) {
                skip = true;
            } else {
                fr.block0 = fr.window + si;
                const int64_t m = ((int64_t)fr.lp_window - ((int64_t)TU + si) * (int64_t)fr.phase_a) % INPUT_RATE;
                fr.lp_data = (int32_t)(m < 0 ? m + INPUT_RATE : m);
                skip = fr.block0 + TU + (int64_t)NSYM * TS > fr.n_samples;
            }
            __syncthreads();                             // ex reused below
        }
    }
    const int per = (NSYM + nchunks - 1) / nchunks;
    const int l0 = 1 + ch * per, l1 = min(NSYM + 1, l0 + per);
    float2 fc = make_float2(0.0f, 0.0f);
    // frame_ok: every read inside the stream (the caller guarantees the descriptor)
    const bool ok = fr.window >= 0 && fr.block0 >= fr.window && fr.block0 + TU + (int64_t)NSYM * TS <= fr.n_samples &&
                    fr.lp_window >= 0 && fr.lp_window < INPUT_RATE && fr.lp_data >= 0 && fr.lp_data < INPUT_RATE;
    if (!ok && !skip && t == 0) atomicOr(T.err, KERR_FRAME);
    if (l0 <= NSYM && ok && !skip) {
        const int64_t dorg = fr.block0 + TU;           // first sample of segment B
        // LDS stage byte address of each of this thread's 6 carrier slots (fft2048_tail), and
        // the stage words of the carrier pairs its read-back quads q = t, t + DT take
        uint32_t cb[6], rq[2];
        {
#pragma unroll
            for (int j = 0; j < 6; j++) cb[j] = (uint32_t)T.stage_of_bin[slot_bin(t, j)] * 4u;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int q = t + DT * i;
                rq[i] = q < K / 4 ? (uint32_t)T.stage_pair[2 * q] | ((uint32_t)T.stage_pair[2 * q + 1] << 16) : 0u;
            }
        }
        // the frame's samples and soft-bit rows through buffer descriptors (wave-uniform
        // bases: 32-bit offsets, the 8 samples of a thread a scalar offset apart, no
        // 64-bit address arithmetic per symbol)
        const void *fb = (const char *)s + fr.block0 * BPS;
        const __amdgpu_buffer_rsrc_t rin =
            __builtin_amdgcn_make_buffer_rsrc((void *)fb, (short)0, (TU + NSYM * TS) * BPS, 0x00020000);
        // soft-bit rows: int16, or RING8 bytes (v + 127) in the pipeline's ring
        constexpr int esz = R8 ? 1 : 2;
        char *orow = (char *)soft + (int64_t)fr.out_slot * NSYM * SYMBITS * esz;
        const __amdgpu_buffer_rsrc_t rout =
            __builtin_amdgcn_make_buffer_rsrc((void *)orow, (short)0, NSYM * SYMBITS * esz, 0x00020000);
        // the {re, im} pair of a carrier in the stage: int16 each, + 127 each for RING8
        auto spair = [&](int ir, int ii) -> uint32_t {
            const uint32_t v = __builtin_amdgcn_perm((uint32_t)ii, (uint32_t)ir, 0x05040100u);
            if constexpr (!R8) return v;
            return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, v) + (u16x2){RING8_BIAS, RING8_BIAS});
        };
        // off: byte offset from block 0; the prefetch registers hold the raw samples (8, 4
        // or 2 bytes), converted when the symbol's turn comes
        auto ld = [&](int32_t off) -> typename Fmt::raw { return Fmt::load(rin, off); };
        // the 6 carrier slots of symbols l and l - 1 alternate between A and B (the loop runs
        // two symbols per trip), so neither is copied into the other per symbol
        float2 A[6], B[6];
        typename Fmt::raw nx[8], ng6, ng7;
        // warm-up symbol l0 - 1 (block 0, the PRS, for the first chunk)
        int32_t ov = (l0 * TS + t) * BPS;                     // this thread's sample 0 of symbol l
        {
            const int64_t u = fr.block0 + (int64_t)(l0 - 1) * TS;
            const int32_t o = ((l0 - 1) * TS + t) * BPS;
            float2 x[8];
#pragma unroll
            for (int m = 0; m < 8; m++) x[m] = Fmt::scaled(ld(o + 256 * BPS * m));
            if (l0 == 1) mix<GEN>(x, T.osc, ncl, fr.lp_window, fr.phase_a, u + t, fr.window);
            else mix<GEN>(x, T.osc, ncl, fr.lp_data, fr.phase_b, u + t, dorg);
            // symbol l0's samples in flight during the warm-up FFT
            ng6 = ld(ov - 512 * BPS);
            ng7 = ld(ov - 256 * BPS);
#pragma unroll
            for (int m = 0; m < 8; m++) nx[m] = ld(ov + 256 * BPS * m);
            fft2048_p123(x, ex, tw, t);
            Quad4 qa, qb;
            fft2048_tail(x, ex, t, qa, qb);
            tail_slots(qa, qb, t, B);
            if (l0 == 1 && aux.snr) {                   // processBlock_0's get_snr (ofdm-decoder.cpp:93)
                float2 X[8];
                tail_all(qa, qb, X);
                const int16_t v = snr_wg_b(X, [&](int k) { return tail_bin(t, k >> 2, k & 3); }, red, t, Fmt::unscale);
                if (t == 0) aux.snr[fi] = v;
            }
        }
        __syncthreads();                                // the tail read ex: the first symbol's pass 1 writes it
        // NCO of segment B (round 4): thread t's samples of symbol l are n = t + 256 m, so
        // their oscillatorTable indices step by -d256 per m and by -dsym per symbol (mod
        // 2048000).  The exact e^{2 pi i ti / N} of the chunk's first sample (the factor
        // tables, in double) then follows the index by complex double recurrences
        // -- x R = e^{-2 pi i d256 / N} per sample, x D = e^{-2 pi i dsym / N} per symbol,
        // both wave-uniform SGPR pairs -- rounded to float per sample: the table's value
        // (its float rounding of the same double) except within ~1e-13 of a rounding
        // boundary, as the relative error of the double recurrence grows by ~2^-53 per
        // step.  The per-sample table rebuild cost 28 VALU + 3 conflicted LDS gathers per
        // sample; this is 6 f64 ops.  Phase 0: oscillatorTable[lp_data].
        const float2 f0 = T.osc[fr.lp_data];
        const int32_t ph = fr.phase_b;
        auto uni = [](double v) {               // wave-uniform double -> SGPR pair
            const uint64_t b = __builtin_bit_cast(uint64_t, v);
            const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
            const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
            return __builtin_bit_cast(double, lo | (hi << 32));
        };
        auto cmul_d = [](double2 x, double yr, double yi) {
            return make_double2(__builtin_fma(x.x, yr, -(x.y * yi)), __builtin_fma(x.x, yi, x.y * yr));
        };
        double2 w = make_double2(1.0, 0.0);     // e^{2 pi i ti / N}, ti: this thread's sample 0 of symbol l
        double rr = 1.0, ri = 0.0, dr = 1.0, di = 0.0;
        float2 efc = make_float2(1.0f, 0.0f);   // FreqCorr of mixed samples = raw x oscillatorTable[-T_u phase]
        if (GEN && ph != 0) {
            const int32_t d256 = nco_mod(256 * (int64_t)ph), dsym = nco_mod((int64_t)TS * ph);
            w = nco_value_d(ncl, nco_index2(fr.lp_data, ph, fr.block0 + (int64_t)l0 * TS + t - dorg + 1));
            const double2 r = nco_value_d(ncl, nco_mod(-(int64_t)d256));
            const double2 d = nco_value_d(ncl, nco_mod(-(int64_t)dsym));
            rr = uni(r.x); ri = uni(r.y);
            dr = uni(d.x); di = uni(d.y);

            efc = nco_value(ncl, nco_mod(-(int64_t)TU * ph));
        }
        // symbol l: S = its 6 carrier slots (computed here), P = symbol l - 1's
        auto sym = [&](const int l, float2 (&S)[6], const float2 (&P)[6]) __attribute__((always_inline)) {
            // this symbol's samples and its guard samples, all loaded one symbol ahead
            // (a guard load issued here would expose a full HBM latency per symbol).  The
            // loads after the chunk's last symbol are not conditional: past the frame they
            // read the buffer's out-of-range zeros, inside it a symbol nobody uses
            float2 a[8];
#pragma unroll
            for (int m = 0; m < 8; m++) a[m] = Fmt::scaled(nx[m]);
            const float2 g6 = Fmt::scaled(ng6), g7 = Fmt::scaled(ng7);
            {
                const int32_t o1 = ov + TS * BPS;
                ng6 = ld(o1 - 512 * BPS);
                ng7 = ld(o1 - 256 * BPS);
#pragma unroll
                for (int m = 0; m < 8; m++) nx[m] = ld(o1 + 256 * BPS * m);
            }
            ov += TS * BPS;
            // FreqCorr over i in [T_u, T_s) on the samples before the NCO: the mixed
            // product x[i] conj(x[i - T_u]) is the raw one times oscillatorTable[-T_u phase]
            // (efc, applied once at the end)
            if (t >= 8) {
                const float2 p = cmul_conj_exact(a[6], g6);
                fc.x += p.x; fc.y += p.y;
            }
            {
                const float2 p = cmul_conj_exact(a[7], g7);
                fc.x += p.x; fc.y += p.y;
            }
            if (!GEN || ph == 0) {
#pragma unroll
                for (int m = 0; m < 8; m++) a[m] = cmul_exact(a[m], f0);
            } else {
                double2 v = w;
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    a[m] = cmul_exact(a[m], make_float2((float)v.x, (float)v.y));
                    if (m < 7) v = cmul_d(v, rr, ri);
                }
                w = cmul_d(w, dr, di);
            }
            if constexpr (DUMP) {                      // test hook: the FFT's input, mixed
                float2 *mp = aux.mix + ((int64_t)fr.out_slot * NSYM + (l - 1)) * TU;
#pragma unroll
                for (int m = 0; m < 8; m++) mp[t + 256 * m] = make_float2(a[m].x * Fmt::unscale, a[m].y * Fmt::unscale);
            }
            fft2048_p123(a, ex, tw, t);
            Quad4 qa, qb;
            fft2048_tail(a, ex, t, qa, qb);
            tail_slots(qa, qb, t, S);
            const bool disp = aux.disp && l == aux.disp_token;
            if (DUMP || disp) {                        // all 8 outputs: the test hook, the display feed
                float2 X[8];
                tail_all(qa, qb, X);
                if constexpr (DUMP) {                  // ... the FFT's output (the scale taken out: exact)
                    float2 *sp = aux.spec + ((int64_t)fr.out_slot * NSYM + (l - 1)) * TU;
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        sp[tail_bin(t, k >> 2, k & 3)] = make_float2(X[k].x * Fmt::unscale, X[k].y * Fmt::unscale);
                }
                if (disp) {                            // the display token's carriers (ofdm-decoder.cpp:197-205)
                    float2 *dp = aux.disp + (int64_t)fr.out_slot * K;
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        const int b = tail_bin(t, k >> 2, k & 3);
                        const float2 v = make_float2(X[k].x * Fmt::unscale, X[k].y * Fmt::unscale);
                        if (b < K / 2) dp[b] = v;
                        else if (b >= TU - 1 - K / 2 && b < TU - 1) dp[b - (TU - 1 - K)] = v;
                    }
                }
            }
            __syncthreads();                           // the tail's reads of ex done: st reuses it
            // DQPSK + soft bits of the 6 slots, fast path first; the few carriers whose
            // truncation the fast path cannot decide (soft_fast) are redone exactly after
            // all 6 (one divergent branch per symbol instead of one per carrier)
            // (the flag is a lane mask in SGPRs: the rare lanes recompute which need it)
            bool risky = false;
#pragma unroll
            for (int k = 0; k < 6; k++) {
                const float2 r1 = cmul_conj_exact(S[k], P[k]);
                // ibits = (int16_t)(q * 127.0), q = -re / ab1 (IEEE float division) and
                // ab1 = |re| + |im| (ofdm-decoder.cpp:185-189)
                const float ab1 = fabsf(r1.x) + fabsf(r1.y);
                int ir, ii;
                risky |= soft_fast<FMT != DABGPU_IQ_F32>(r1, ab1, ir, ii);
                *(uint32_t *)((char *)st + cb[k]) = spair(ir, ii);
            }
            if (risky) {
#pragma unroll
                for (int k = 0; k < 6; k++) {
                    const float2 r1 = cmul_conj_exact(S[k], P[k]);
                    const float ab1 = fabsf(r1.x) + fabsf(r1.y);
                    int ir, ii;
                    if (soft_fast<FMT != DABGPU_IQ_F32>(r1, ab1, ir, ii))
                        *(uint32_t *)((char *)st + cb[k]) = spair(trunc127d(-r1.x / ab1), trunc127d(-r1.y / ab1));
                }
            }
            if (softf) {                               // parity tests only: the float soft values
                float *sf = softf + ((int64_t)fr.out_slot * NSYM + (l - 1)) * SYMBITS;
#pragma unroll
                for (int k = 0; k < 6; k++) {
                    const int c = T.carrier_of_bin[slot_bin(t, k)];
                    const float2 r1 = cmul_conj_exact(S[k], P[k]);
                    const float ab1 = fabsf(r1.x) + fabsf(r1.y);
                    sf[c] = -r1.x / ab1;
                    sf[K + c] = -r1.y / ab1;
                }
            }
            __syncthreads();
            // carriers 4q..4q+3, q < 384: re to row[4q..], im to row[K + 4q..]
            const int32_t rowb = (l - 1) * SYMBITS * esz;
            // carriers 4q, 4q+1 and 4q+2, 4q+3: two pair words of the stage
            auto quad = [&](int i) {
                const uint2 a = *(const uint2 *)(st + (rq[i] & 0xFFFFu));
                const uint2 b = *(const uint2 *)(st + (rq[i] >> 16));
                return make_uint4(a.x, a.y, b.x, b.y);
            };
            if constexpr (R8) {                        // the low bytes of each half
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const int q = t + DT * i;
                    if (q >= K / 4) break;
                    const uint4 w = quad(i);
                    const uint32_t xy = __builtin_amdgcn_perm(w.y, w.x, 0x06040200u);   // re0 im0 re1 im1
                    const uint32_t zw = __builtin_amdgcn_perm(w.w, w.z, 0x06040200u);   // re2 im2 re3 im3
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(zw, xy, 0x06040200u), rout, rowb + 4 * q, 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(zw, xy, 0x07050301u), rout, rowb + K + 4 * q, 0, 0);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const int q = t + DT * i;
                    if (q >= K / 4) break;
                    const uint4 w = quad(i);
                    const uint2 re = make_uint2(__builtin_amdgcn_perm(w.y, w.x, 0x05040100u),
                                                __builtin_amdgcn_perm(w.w, w.z, 0x05040100u));
                    const uint2 im = make_uint2(__builtin_amdgcn_perm(w.y, w.x, 0x07060302u),
                                                __builtin_amdgcn_perm(w.w, w.z, 0x07060302u));
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32, re), rout, rowb + 8 * q, 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32, im), rout, rowb + 2 * K + 8 * q, 0, 0);
                }
            }
            __syncthreads();
        };
        for (int l = l0; l < l1; l += 2) {
            sym(l, A, B);
            if (l + 1 < l1) sym(l + 1, B, A);
        }
        fc = cmulw(fc, efc);
        fc.x *= Fmt::unscale * Fmt::unscale;           // the partial sums in absolute units (exact)
        fc.y *= Fmt::unscale * Fmt::unscale;
    }
    fc.x = wave_sum(fc.x);
    fc.y = wave_sum(fc.y);
    if ((t & 63) == 0) fcw[t >> 6] = fc;
    __syncthreads();
    if (t == 0) {
        float2 f = fcw[0];
        for (int w = 1; w < DT / 64; w++) { f.x += fcw[w].x; f.y += fcw[w].y; }
        fcpart[item] = f;
    }
}

// findIndex alone, one workgroup per frame (the host needs startIndex before block 0
// while the coarse AFC is pending)
template <bool GEN, int FMT>
__global__ __launch_bounds__(DT) void k_prs_wg(const void *__restrict__ iq, const dabgpu_frame *__restrict__ frames,
                                               OfdmTables T, DemodAux aux) {
    __shared__ float2 ex[EXN];
    __shared__ TwLds twl;
    __shared__ RedLds red;
    const int t = threadIdx.x, f = blockIdx.x;
    __shared__ double2 ncl[GEN ? NCO_USED : 1];
    const DemodTw tw = tw_setup(twl, T, t);
    nco_setup<GEN>(ncl, T, t);
    __syncthreads();
    const dabgpu_frame fr = frames[f];
    if (fr.window < 0 || fr.window + TU > fr.n_samples || fr.lp_window < 0 || fr.lp_window >= INPUT_RATE) {
        if (t == 0) {
            atomicOr(T.err, KERR_FRAME);
            aux.si[f] = -1;
        }
        return;
    }
    const void *s = iq_stream<FMT>(iq, fr.iq_base);
    float2 a[8];
#pragma unroll
    for (int m = 0; m < 8; m++) a[m] = iq_at<FMT>(s, fr.window + t + 256 * m);
    mix<GEN>(a, T.osc, ncl, fr.lp_window, fr.phase_a, fr.window + t, fr.window);
    float mx, sm;
    const int32_t si = prs_corr_wg(a, ex, tw, t, T.ref, aux.level, red, mx, sm);
    if (t == 0) {
        aux.si[f] = si;
        if (aux.maxv) aux.maxv[f] = mx;
        if (aux.sumv) aux.sumv[f] = sm;
    }
}

// processBlock_0 (ofdm-decoder.cpp:85-162), one workgroup per frame: FFT of block 0
// (segment A of the NCO), get_snr, and when frames[f].flags & 1 the coarse offset of
// freqSyncMethod `method` in carriers (100 - 2048 when method 2 finds nothing, 100
// means "no estimate" for method 1 -- the reference's values).
template <bool GEN, int FMT>
__global__ __launch_bounds__(DT) void k_block0_wg(const void *__restrict__ iq, const dabgpu_frame *__restrict__ frames,
                                                  OfdmTables T, int method, int16_t *__restrict__ correction,
                                                  int16_t *__restrict__ snr) {
#pragma clang fp contract(off)
    __shared__ float2 ex[EXN];
    __shared__ TwLds twl;
    __shared__ RedLds red;
    __shared__ float val[2048];                          // |X| (method 0) or per-candidate sums
    __shared__ float cv[96];                             // method 1: correlationVector
    const int t = threadIdx.x, f = blockIdx.x;
    __shared__ double2 ncl[GEN ? NCO_USED : 1];
    const DemodTw tw = tw_setup(twl, T, t);
    nco_setup<GEN>(ncl, T, t);
    __syncthreads();
    const dabgpu_frame fr = frames[f];
    if (fr.window < 0 || fr.block0 < fr.window || fr.block0 + TU > fr.n_samples || fr.lp_window < 0 ||
        fr.lp_window >= INPUT_RATE) {
        if (t == 0) {
            atomicOr(T.err, KERR_FRAME);
            correction[f] = 0;
            if (snr) snr[f] = 0;
        }
        return;
    }
    const void *s = iq_stream<FMT>(iq, fr.iq_base);
    float2 a[8];
#pragma unroll
    for (int m = 0; m < 8; m++) a[m] = iq_at<FMT>(s, fr.block0 + t + 256 * m);
    mix<GEN>(a, T.osc, ncl, fr.lp_window, fr.phase_a, fr.block0 + t, fr.window);
    fft2048_wg(a, ex, tw, t);
    {
        const int16_t v = snr_wg(a, t, red);
        if (t == 0 && snr) snr[f] = v;
    }
    if (!(fr.flags & 1)) {                               // f2Correction off: no estimate
        if (t == 0) correction[f] = 0;
        return;
    }
    __syncthreads();
    const int b0 = bin0_of(t);
#pragma unroll
    for (int k = 0; k < 8; k++) ex[b0 + 64 * k] = a[k];  // natural bin order
    if (method == 0) {
#pragma unroll
        for (int k = 0; k < 8; k++) val[b0 + 64 * k] = hypotf(a[k].x, a[k].y);
    }
    __syncthreads();
    auto argpair = [&](int i, int j) -> float {          // arg (X[i] conj(X[j]))
        const float2 p = cmul_conj_exact(ex[i & 2047], ex[j & 2047]);
        return atan2f(p.y, p.x);
    };
    if (method == 1) {                                   // ofdm-decoder.cpp:106-127
        if (t < 72 + 18) cv[t] = argpair(2048 - 36 + t, 2048 - 36 + t + 1);
        __syncthreads();
        if (t < 72) {
            float sum = 0.0f;
            for (int j = 1; j < 18; j++) sum += fabsf(T.refarg[j] * cv[t + j]);
            val[t] = sum;
        }
        __syncthreads();
        if (t == 0) {
            float MMax = 0.0f;
            int index = 100;
            for (int i = 0; i < 72; i++)
                if (val[i] > MMax) { MMax = val[i]; index = i; }
            correction[f] = (int16_t)(2048 - 36 + index - 2048);
        }
    } else if (method == 2) {                            // ofdm-decoder.cpp:128-161
        if (t < 72) {
            const int i = 2048 - 36 + t;
            const double pi = M_PI;
            const float a1 = (float)fabs(fabs((double)argpair(i + 1, i + 2) / pi) - 1);
            const float a2 = (float)fabs(fabs((double)argpair(i + 2, i + 3) / pi) - 1);
            const float a3 = fabsf(argpair(i + 3, i + 4));
            const float a4 = fabsf(argpair(i + 4, i + 5));
            const float a5 = fabsf(argpair(i + 5, i + 6));
            const float c1 = (float)fabs(fabs((double)argpair(i + 17, i + 19) / pi) - 1);
            const float c2 = fabsf(argpair(i + 19, i + 20));
            const float c3 = fabsf(argpair(i + 20, i + 21));
            const float c4 = fabsf(argpair(i + 21, i + 22));
            val[t] = a1 + a2 + a3 + a4 + a5 + c1 + c2 + c3 + c4;
        }
        __syncthreads();
        if (t == 0) {
            float Mmin = 1000.0f;
            int index = 100;
            for (int k = 0; k < 72; k++)
                if (val[k] < Mmin) { Mmin = val[k]; index = 2048 - 36 + k; }
            correction[f] = (int16_t)(index - 2048);
        }
    } else {                                             // getMiddle (ofdm-decoder.cpp:233-258), sequential
        if (t == 0) {
            float sum = 0.0f, oldMax = 0.0f;
            int maxIndex = 0;
            for (int i = 40; i < 1536 + 40; i++) sum += val[(1024 + i) & 2047];
            for (int i = 40; i < 2048 - (1536 - 40); i++) {
                sum -= val[(1024 + i) & 2047];
                sum += val[(1024 + i + 1536) & 2047];
                if (sum > oldMax) { sum = oldMax; maxIndex = i; }
            }
            correction[f] = (int16_t)(maxIndex - (2048 - 1536) / 2);
        }
    }
}

// One OFDM symbol at a time, for the single-symbol ofdmDecoder interface
// (ofdm-decoder.cpp:85-190): kind 0 = block 0 (FFT of samples[0, T_u), the spectrum
// becomes the phase reference), kind 1 = a data symbol (FFT of samples[T_g, T_s),
// DQPSK against the stored spectrum -> ibits[3072], spectrum := this symbol's).  The
// samples are already NCO-mixed by the caller (ofdmProcessor::getSamples); spec holds
// the previous spectrum in natural bin order.  One workgroup.
__global__ __launch_bounds__(DT) void k_symbol_wg(const float2 *__restrict__ smp, int kind, OfdmTables T,
                                                  float2 *__restrict__ spec, int16_t *__restrict__ ibits) {
    __shared__ float2 ex[EXN];
    __shared__ TwLds twl;
    const int t = threadIdx.x;
    const DemodTw tw = tw_setup(twl, T, t);
    __syncthreads();
    const float2 *x = smp + (kind ? TG : 0);
    float2 a[8];
#pragma unroll
    for (int m = 0; m < 8; m++) a[m] = x[t + 256 * m];
    fft2048_wg(a, ex, tw, t);
    const int b0 = bin0_of(t);
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int b = b0 + 64 * k;
        if (kind) {
            const int c = T.carrier_of_bin[b];
            if (c >= 0) {
                const float2 r1 = cmul_conj_exact(a[k], spec[b]);
                int ir, ii;
                soft_pair(r1, fabsf(r1.x) + fabsf(r1.y), ir, ii);
                ibits[c] = (int16_t)ir;
                ibits[K + c] = (int16_t)ii;
            }
        }
        spec[b] = a[k];
    }
}

// get_snr (ofdm-decoder.cpp:212-230) of a spectrum in natural bin order: the
// ofdmDecoder::get_snr drop-in, the same workgroup reduction as the fused kernels'
__global__ __launch_bounds__(DT) void k_snr_wg(const float2 *__restrict__ spec, int16_t *__restrict__ out) {
    __shared__ RedLds red;
    const int t = threadIdx.x, b0 = bin0_of(t);
    float2 a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = spec[b0 + 64 * k];
    const int16_t v = snr_wg(a, t, red);
    if (t == 0) *out = v;
}
hipError_t launch_snr(hipStream_t st, const float *spec, int16_t *out) {
    hipLaunchKernelGGL(k_snr_wg, dim3(1), dim3(DT), 0, st, (const float2 *)spec, out);
    return hipGetLastError();
}

// the kernels' NCO over a range of table indices (exhaustive parity check)
__global__ __launch_bounds__(DT) void k_nco_eval(OfdmTables T, int32_t first, int32_t n, float2 *__restrict__ out) {
    __shared__ double2 ncl[NCO_USED];
    nco_setup<true>(ncl, T, threadIdx.x);
    __syncthreads();
    for (int32_t i = blockIdx.x * DT + threadIdx.x; i < n; i += gridDim.x * DT) out[i] = nco_value(ncl, first + i);
}
hipError_t launch_nco_eval(hipStream_t st, const OfdmTables &T, int32_t first, int32_t n, float2 *out) {
    const int blocks = (int)std::min<int64_t>(2048, ((int64_t)n + DT - 1) / DT);
    hipLaunchKernelGGL(k_nco_eval, dim3(blocks), dim3(DT), 0, st, T, first, n, out);
    return hipGetLastError();
}

hipError_t launch_symbol(hipStream_t st, const float *smp, int kind, const OfdmTables &T, float *spec, int16_t *ibits) {
    hipLaunchKernelGGL(k_symbol_wg, dim3(1), dim3(DT), 0, st, (const float2 *)smp, kind, T, (float2 *)spec, ibits);
    return hipGetLastError();
}

hipError_t launch_demod(hipStream_t st, const void *iq, const dabgpu_frame *fr, int n, int nchunks,
                        const OfdmTables &T, int16_t *soft, float *softf, float *fcpart, bool general,
                        const DemodAux &aux) {
    if (n <= 0) return hipSuccess;
    const dim3 grid(n * nchunks), block(DT);
    float2 *fp = (float2 *)fcpart;
#define DEMOD_GO(G, S, R, F, D) \
    hipLaunchKernelGGL((k_demod_wg<G, S, R, F, D>), grid, block, 0, st, iq, fr, nchunks, T, soft, softf, fp, aux)
#define DEMOD_GS(R, F)                                              \
    do {                                                            \
        if (aux.si) { if (general) DEMOD_GO(true, true, R, F, false); else DEMOD_GO(false, true, R, F, false); } \
        else { if (general) DEMOD_GO(true, false, R, F, false); else DEMOD_GO(false, false, R, F, false); }     \
    } while (0)
    if (aux.mix) {                                     // the NCO / FFT test hook (GEN kernels only)
        if (!general || !aux.spec) return hipErrorInvalidValue;
        if (!aux.si) {                                 // the operator form: cf32 in, int16 out
            if (aux.ring8 || aux.fmt != DABGPU_IQ_F32) return hipErrorInvalidValue;
            DEMOD_GO(true, false, false, DABGPU_IQ_F32, true);
        } else {                                       // the pipeline's form: findIndex, RING8, any format
            if (!aux.ring8) return hipErrorInvalidValue;
            if (aux.fmt == DABGPU_IQ_S16) DEMOD_GO(true, true, true, DABGPU_IQ_S16, true);
            else if (aux.fmt == DABGPU_IQ_U8) DEMOD_GO(true, true, true, DABGPU_IQ_U8, true);
            else if (aux.fmt == DABGPU_IQ_F32) DEMOD_GO(true, true, true, DABGPU_IQ_F32, true);
            else return hipErrorInvalidValue;
        }
    } else if (aux.ring8) {                            // the pipeline's RING8 ring, any sample format
        if (aux.fmt == DABGPU_IQ_S16) DEMOD_GS(true, DABGPU_IQ_S16);
        else if (aux.fmt == DABGPU_IQ_U8) DEMOD_GS(true, DABGPU_IQ_U8);
        else if (aux.fmt == DABGPU_IQ_F32) DEMOD_GS(true, DABGPU_IQ_F32);
        else return hipErrorInvalidValue;
    } else {                                           // the operators: cf32 in, int16 out
        if (aux.fmt != DABGPU_IQ_F32) return hipErrorInvalidValue;
        DEMOD_GS(false, DABGPU_IQ_F32);
    }
#undef DEMOD_GS
#undef DEMOD_GO
    return hipGetLastError();
}

#define FMT_DISPATCH(fmt, GO)                                       \
    do {                                                            \
        if ((fmt) == DABGPU_IQ_F32) GO(DABGPU_IQ_F32);              \
        else if ((fmt) == DABGPU_IQ_S16) GO(DABGPU_IQ_S16);         \
        else if ((fmt) == DABGPU_IQ_U8) GO(DABGPU_IQ_U8);           \
        else return hipErrorInvalidValue;                           \
    } while (0)

hipError_t launch_prs_sync(hipStream_t st, const void *iq, int fmt, const dabgpu_frame *fr, int n, const OfdmTables &T,
                           int level, int32_t *si, float *mx, float *sm, bool general) {
    if (n <= 0) return hipSuccess;
    DemodAux aux{};
    aux.si = si;
    aux.maxv = mx;
    aux.sumv = sm;
    aux.level = level;
#define PRS_GO(F)                                                                                   \
    do {                                                                                            \
        if (general) hipLaunchKernelGGL((k_prs_wg<true, F>), dim3(n), dim3(DT), 0, st, iq, fr, T, aux);  \
        else hipLaunchKernelGGL((k_prs_wg<false, F>), dim3(n), dim3(DT), 0, st, iq, fr, T, aux);         \
    } while (0)
    FMT_DISPATCH(fmt, PRS_GO);
#undef PRS_GO
    return hipGetLastError();
}

hipError_t launch_block0(hipStream_t st, const void *iq, int fmt, const dabgpu_frame *fr, int n, const OfdmTables &T,
                         int method, int16_t *corr, int16_t *snr, bool general) {
    if (n <= 0) return hipSuccess;
#define B0_GO(F)                                                                                                 \
    do {                                                                                                         \
        if (general) hipLaunchKernelGGL((k_block0_wg<true, F>), dim3(n), dim3(DT), 0, st, iq, fr, T, method, corr, snr); \
        else hipLaunchKernelGGL((k_block0_wg<false, F>), dim3(n), dim3(DT), 0, st, iq, fr, T, method, corr, snr);        \
    } while (0)
    FMT_DISPATCH(fmt, B0_GO);
#undef B0_GO
    return hipGetLastError();
}
#undef FMT_DISPATCH

}  // namespace dab
