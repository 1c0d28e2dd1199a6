// k_demod.hip -- ofdmDecoder::processToken x 75 per frame (ofdm-decoder.cpp:167-190)
// + the FreqCorr guard correlation (ofdm-processor.cpp:424-438), for gfx950.
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
#ifndef DEMOD_WG_PER_SIMD
#define DEMOD_WG_PER_SIMD 3     // resident workgroups per CU (= waves per SIMD): <= 168 VGPRs
#endif

__device__ __forceinline__ int32_t nco_index2(int32_t lp0, int32_t phase, int64_t j) {
    int64_t t = ((int64_t)lp0 - j * (int64_t)phase) % INPUT_RATE;
    return (int32_t)(t < 0 ? t + INPUT_RATE : t);
}

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
template <int M>
__device__ __forceinline__ float quad_bfly(float v, float sign) {
    constexpr int ctrl = M == 2 ? 0x4E : 0xB1;          // quad_perm [2,3,0,1] / [1,0,3,2]
    const float p = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false));
    return fmaf(sign, v, p);
}

template <bool GEN>
__device__ __forceinline__ void mix(float2 (&v)[8], const float2 *__restrict__ osc, int32_t lp0, int32_t phase,
                                   int64_t first, int64_t origin) {
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
            v[m] = cmul_exact(v[m], osc[t]);
            t -= step;
            if (t < 0) t += INPUT_RATE;
        }
    }
}
template <bool GEN>
__device__ __forceinline__ float2 mix1(float2 v, const float2 *__restrict__ osc, int32_t lp0, int32_t phase,
                                       int64_t pos, int64_t origin) {
    if (!GEN || phase == 0) return cmul_exact(v, osc[lp0]);
    return cmul_exact(v, osc[nco_index2(lp0, phase, pos - origin + 1)]);
}

struct DemodTw {
    const float2 *w1;             // LDS table W2048^(t k) at [(k - 1) * 256 + t], k = 1..7
    const float2 *w2;             // LDS table W256^(t' k) at [(k - 1) * 32 + t']: consecutive lanes, no bank conflicts
    const float2 *w3;             // LDS table W32^(t'' k) at [(k - 1) * 4 + t'']: a quad's 4 values in 4 different banks
    float sg2, sg1;               // quad butterfly signs (+1 lower lane, -1 upper)
    bool rot;                     // lane t'' == 3 multiplies by -j between the two stages
};

// the FFT of the 8 samples a[] (n = t + 256 m) of every thread; ex: 2048 + pad float2 of LDS
__device__ __forceinline__ void fft2048_wg(float2 (&a)[8], float2 *ex, const DemodTw &tw, int t) {
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
    // pass 4: radix-4 over the quad's t''; lane t'' ends with K'' = brev2(t'')
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float2 v = make_float2(quad_bfly<2>(a[k].x, tw.sg2), quad_bfly<2>(a[k].y, tw.sg2));
        if (tw.rot) v = make_float2(v.y, -v.x);
        a[k] = make_float2(quad_bfly<1>(v.x, tw.sg1), quad_bfly<1>(v.y, tw.sg1));
    }
}

template <bool GEN>
__global__ __launch_bounds__(DT, DEMOD_WG_PER_SIMD) void k_demod_wg(const float2 *__restrict__ iq,
                                                    const dabgpu_frame *__restrict__ frames, int nchunks,
                                                    OfdmTables T, int16_t *__restrict__ soft,
                                                    float *__restrict__ softf, float2 *__restrict__ fcpart,
                                                    const int32_t *__restrict__ si) {
    __shared__ float2 ex[2048 + 64 * (ZROW - 32)];
    __shared__ int16_t st[2 * K + 2 * DT];
    __shared__ float2 fcw[DT / 64];
    // twiddles, laid out per pass so that a wave's reads are conflict-free (the values
    // are the W2048 table's entries: W256^j = W2048^(8 j), W32^j = W2048^(64 j))
    __shared__ float2 w1s[7 * DT];      // pass 1: LDS instead of 14 VGPRs (room for the guard prefetch)
    __shared__ float2 w2s[7 * 32];
    __shared__ float2 w3s[7 * 4];
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 1; k < 8; k++) w1s[(k - 1) * DT + t] = T.w2048[(t * k) & 2047];
    if (t < 7 * 32) w2s[t] = T.w2048[(8 * ((t & 31) * (t / 32 + 1))) & 2047];
    if (t < 7 * 4) w3s[t] = T.w2048[(64 * ((t & 3) * (t / 4 + 1))) & 2047];
    __syncthreads();
    const int item = blockIdx.x;
    const int fi = item / nchunks, ch = item % nchunks;
    dabgpu_frame fr = frames[fi];
    // FRAME_SI_ON_DEVICE: the frame starts where k_prs_sync found it (block0 = window +
    // startIndex, ofdm-processor.cpp:360-368) -- no host round trip between the two;
    // a frame whose sync failed or whose symbols are not all there yet is skipped
    // (the host's replay does not commit it)
    bool skip = false;
    if (si && (fr.flags & FRAME_SI_ON_DEVICE)) {
        const int32_t s = si[fi];
        if (s < 0) {
            skip = true;
        } else {
            fr.block0 = fr.window + s;
            const int64_t m = ((int64_t)fr.lp_window - ((int64_t)TU + s) * (int64_t)fr.phase_a) % INPUT_RATE;
            fr.lp_data = (int32_t)(m < 0 ? m + INPUT_RATE : m);
            skip = fr.block0 + TU + (int64_t)NSYM * TS > fr.n_samples;
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
        const float2 *s = iq + fr.iq_base;
        const int64_t dorg = fr.block0 + TU;           // first sample of segment B
        DemodTw tw;
        {
            const int tq = t & 3;
            tw.w2 = w2s;
            tw.w3 = w3s;
            tw.w1 = w1s;
            tw.sg2 = (tq & 2) ? -1.0f : 1.0f;
            tw.sg1 = (tq & 1) ? -1.0f : 1.0f;
            tw.rot = tq == 3;
        }
        // carriers of this thread's 8 bins (-1: none), two int16 per register
        uint32_t cb[4];
        {
            const int g = t >> 2, tq = t & 3, k1 = g >> 3, k2 = g & 7;
            const int kk = ((tq & 1) << 1) | (tq >> 1);
#pragma unroll
            for (int k3 = 0; k3 < 8; k3 += 2)
                cb[k3 >> 1] = (uint32_t)(uint16_t)T.carrier_of_bin[k1 + 8 * k2 + 64 * k3 + 512 * kk] |
                              ((uint32_t)(uint16_t)T.carrier_of_bin[k1 + 8 * k2 + 64 * (k3 + 1) + 512 * kk] << 16);
        }
        float2 a[8], nx[8], P[8], ng6, ng7;
        // warm-up symbol l0 - 1 (the PRS for the first chunk)
        {
            const int64_t u = fr.block0 + (int64_t)(l0 - 1) * TS;
#pragma unroll
            for (int m = 0; m < 8; m++) a[m] = s[u + t + 256 * m];
            if (l0 == 1) mix<GEN>(a, T.osc, fr.lp_window, fr.phase_a, u + t, fr.window);
            else mix<GEN>(a, T.osc, fr.lp_data, fr.phase_b, u + t, dorg);
        }
        {
            const int64_t u = fr.block0 + (int64_t)l0 * TS;
            ng6 = s[u - 512 + t];
            ng7 = s[u - 256 + t];
#pragma unroll
            for (int m = 0; m < 8; m++) nx[m] = s[u + t + 256 * m];
        }
        fft2048_wg(a, ex, tw, t);
#pragma unroll
        for (int k = 0; k < 8; k++) P[k] = a[k];
        for (int l = l0; l < l1; l++) {
            const int64_t u0 = fr.block0 + (int64_t)l * TS;
            // this symbol's samples and its guard samples, all loaded one symbol ahead
            // (a guard load issued here would expose a full HBM latency per symbol)
#pragma unroll
            for (int m = 0; m < 8; m++) a[m] = nx[m];
            float2 g6 = ng6, g7 = ng7;
            if (l + 1 < l1) {
                const int64_t u1 = u0 + TS;
                ng6 = s[u1 - 512 + t];
                ng7 = s[u1 - 256 + t];
#pragma unroll
                for (int m = 0; m < 8; m++) nx[m] = s[u1 + t + 256 * m];
            }
            mix<GEN>(a, T.osc, fr.lp_data, fr.phase_b, u0 + t, dorg);
            g6 = mix1<GEN>(g6, T.osc, fr.lp_data, fr.phase_b, u0 - 512 + t, dorg);
            g7 = mix1<GEN>(g7, T.osc, fr.lp_data, fr.phase_b, u0 - 256 + t, dorg);
            if (t >= 8) {                              // FreqCorr over i in [T_u, T_s)
                const float2 p = cmul_conj_exact(a[6], g6);
                fc.x += p.x; fc.y += p.y;
            }
            {
                const float2 p = cmul_conj_exact(a[7], g7);
                fc.x += p.x; fc.y += p.y;
            }
            fft2048_wg(a, ex, tw, t);
            float *sf = softf ? softf + ((int64_t)fr.out_slot * NSYM + (l - 1)) * SYMBITS : nullptr;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const float2 r1 = cmul_conj_exact(a[k], P[k]);
                P[k] = a[k];
                // q = -re / (|re| + |im|): one reciprocal for both (<= 1 ulp; the FFT
                // before it already differs from FFTW3f's by more)
                const float inv = __builtin_amdgcn_rcpf(fabsf(r1.x) + fabsf(r1.y));
                const float qr = -r1.x * inv, qi = -r1.y * inv;
                const int c = (int)(int16_t)((k & 1) ? (cb[k >> 1] >> 16) : (cb[k >> 1] & 0xFFFFu));
                st[c >= 0 ? c : 2 * K + t] = (int16_t)trunc127d(qr);
                st[c >= 0 ? K + c : 2 * K + DT + t] = (int16_t)trunc127d(qi);
                if (sf && c >= 0) { sf[c] = qr; sf[K + c] = qi; }
            }
            __syncthreads();
            int2 *dst = (int2 *)(soft + ((int64_t)fr.out_slot * NSYM + (l - 1)) * SYMBITS);
            const int2 *src = (const int2 *)st;
#pragma unroll
            for (int i = 0; i < 3; i++) dst[t + DT * i] = src[t + DT * i];
            __syncthreads();
        }
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

hipError_t launch_demod(hipStream_t st, const float *iq, const dabgpu_frame *fr, int n, int nchunks,
                        const OfdmTables &T, int16_t *soft, float *softf, float *fcpart, bool general,
                        const int32_t *si) {
    if (n <= 0) return hipSuccess;
    const dim3 grid(n * nchunks), block(DT);
    if (general)
        hipLaunchKernelGGL(k_demod_wg<true>, grid, block, 0, st, (const float2 *)iq, fr, nchunks, T, soft, softf,
                           (float2 *)fcpart, si);
    else
        hipLaunchKernelGGL(k_demod_wg<false>, grid, block, 0, st, (const float2 *)iq, fr, nchunks, T, soft, softf,
                           (float2 *)fcpart, si);
    return hipGetLastError();
}

}  // namespace dab
