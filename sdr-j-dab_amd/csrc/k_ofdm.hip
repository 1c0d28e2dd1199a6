// k_ofdm.hip -- OFDM front-end kernels for gfx950 (one wave64 per work item):
//   k_prs_sync : phaseReference::findIndex   (phasereference.cpp:60-88)
//   k_block0   : ofdmDecoder::processBlock_0 (ofdm-decoder.cpp:85-127, method 1)
//   (k_demod, processToken x 75 + FreqCorr: k_demod.hip)
//   k_acquire  : ofdmProcessor::run notSynced..SyncOnEndNull (ofdm-processor.cpp:274-338)
// Every sample read applies the getSamples NCO (ofdm-processor.cpp:217-226).
#include "dab_device.h"
#include "dab_kernels.h"

namespace dab {

// sample j (1-based count inside a getSamples segment that started with
// localPhase lp0): oscillatorTable[(lp0 - j*phase) mod 2048000]
__device__ __forceinline__ int32_t nco_index(int32_t lp0, int32_t phase, int64_t j) {
    int64_t t = ((int64_t)lp0 - j * (int64_t)phase) % INPUT_RATE;
    return (int32_t)(t < 0 ? t + INPUT_RATE : t);
}

// Load 32 samples per lane: lane n2 gets stream[start + n2 + 64*n1] into v[n1],
// NCO-mixed as samples of a segment whose first sample is `origin`.
template <bool GEN, int N>
__device__ __forceinline__ void load_mixed(const float2 *__restrict__ s, int64_t start, int32_t lp0,
                                           int32_t phase, int64_t origin, const float2 *__restrict__ osc,
                                           float2 (&v)[N], int lane) {
#pragma unroll
    for (int i = 0; i < N; i++) v[i] = s[start + lane + 64 * i];
    if (!GEN || phase == 0) {
        const float2 f = osc[lp0];
#pragma unroll
        for (int i = 0; i < N; i++) v[i] = cmul_exact(v[i], f);
    } else {
        int32_t t = nco_index(lp0, phase, start + lane - origin + 1);
        int32_t step = (int32_t)((((int64_t)64 * phase) % INPUT_RATE + INPUT_RATE) % INPUT_RATE);
#pragma unroll
        for (int i = 0; i < N; i++) {
            v[i] = cmul_exact(v[i], osc[t]);
            t -= step;
            if (t < 0) t += INPUT_RATE;
            if ((i & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// a frame descriptor must keep every read inside its stream (else: flag + skip)
__device__ __forceinline__ bool frame_ok(const dabgpu_frame &fr, int64_t last_excl, int32_t *err) {
    const bool ok = fr.window >= 0 && fr.block0 >= fr.window && last_excl <= fr.n_samples &&
                    fr.lp_window >= 0 && fr.lp_window < INPUT_RATE && fr.lp_data >= 0 && fr.lp_data < INPUT_RATE;
    if (!ok && threadIdx.x == 0) atomicOr(err, KERR_FRAME);
    return ok;
}

// trunc((double)q * 127.0) computed exactly in fp32 (ofdm-decoder.cpp:188-189)
__device__ __forceinline__ int trunc127(float q) {
    float hi = __fmul_rn(q, 127.0f);
    float lo = fmaf(q, 127.0f, -hi);
    const float t = truncf(hi);
    const float adj = (t == hi) ? ((hi > 0.0f && lo < 0.0f) ? -1.0f : ((hi < 0.0f && lo > 0.0f) ? 1.0f : 0.0f)) : 0.0f;
    return (int)(t + adj);
}

template <bool GEN>
__global__ __launch_bounds__(64) void k_prs_sync(const float2 *__restrict__ iq,
                                                 const dabgpu_frame *__restrict__ frames, int n,
                                                 OfdmTables T, int level, int32_t *__restrict__ start_index,
                                                 float *__restrict__ maxv, float *__restrict__ sumv) {
    __shared__ float2 lds[2048];                    // FFT scratch, then the whole correlation
    const int lane = threadIdx.x, f = blockIdx.x;
    if (f >= n) return;
    const dabgpu_frame fr = frames[f];
    if (!frame_ok(fr, fr.window + TU, T.err)) {
        if (lane == 0) start_index[f] = -1;
        return;
    }
    const float2 *s = iq + fr.iq_base;
    Twiddles tw;
    load_twiddles(tw, T.tw, lane);
    float2 v[32];
    load_mixed<GEN>(s, fr.window, fr.lp_window, fr.phase_a, fr.window, T.osc, v, lane);
    fft2048(v, lds, tw, lane);
    const int k1 = lane >> 1, r = lane & 1;
    sfor<0, 32>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        float2 rr = cmul_conj_exact(v[i], T.ref_l[i * 64 + lane]);
        lds[k1 + 32 * brev5(i) + 1024 * r] = rr;
    });
#pragma unroll
    for (int n1 = 0; n1 < 32; n1++) {
        float2 a = lds[lane + 64 * n1];
        v[n1] = make_float2(a.x, -a.y);             // IFFT via conj(FFT(conj(.)))
    }
    fft2048(v, lds, tw, lane);
    const float scale = 1.0f / 2048.0f;
    float sum = 0.0f, best = -10000.0f;
    int bidx = 0x7fffffff;
    sfor<0, 32>([&](auto kc) {                      // increasing time index per lane
        constexpr int k2 = decltype(kc)::value;
        constexpr int i = brev5(k2);
        float a = hypotf(v[i].x * scale, -v[i].y * scale);
        sum += a;
        if (a > best) { best = a; bidx = k1 + 32 * k2 + 1024 * r; }
    });
    sum = wave_sum(sum);
    for (int o = 32; o > 0; o >>= 1) {
        float ob = __shfl_xor(best, o);
        int oi = __shfl_xor(bidx, o);
        if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
    }
    if (lane == 0) {
        int32_t res;
        if (best < (float)level * sum / 2048.0f) res = (int32_t)(-fabsf(best / (sum / 2048.0f)) - 1.0f);
        else res = bidx;
        start_index[f] = res;
        if (maxv) maxv[f] = best;
        if (sumv) sumv[f] = sum;
    }
}

template <bool GEN>
__global__ __launch_bounds__(64) void k_block0(const float2 *__restrict__ iq,
                                               const dabgpu_frame *__restrict__ frames, int n,
                                               OfdmTables T, int16_t *__restrict__ correction) {
    __shared__ float2 lds[2048 + 48];               // FFT scratch, then the spectrum + 90 phase differences
    const int lane = threadIdx.x, f = blockIdx.x;
    if (f >= n) return;
    const dabgpu_frame fr = frames[f];
    if (!(fr.flags & 1)) {
        if (lane == 0) correction[f] = 0;
        return;
    }
    if (!frame_ok(fr, fr.block0 + TU, T.err)) {
        if (lane == 0) correction[f] = 0;
        return;
    }
    const float2 *s = iq + fr.iq_base;
    Twiddles tw;
    load_twiddles(tw, T.tw, lane);
    float2 v[32];
    load_mixed<GEN>(s, fr.block0, fr.lp_window, fr.phase_a, fr.window, T.osc, v, lane);
    fft2048(v, lds, tw, lane);
    const int k1 = lane >> 1, r = lane & 1;
    sfor<0, 32>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        lds[k1 + 32 * brev5(i) + 1024 * r] = v[i];
    });
    float *corr = (float *)(lds + 2048);
    for (int i = lane; i < 90; i += 64) {
        int b = (2048 - 36 + i) & 2047;
        float2 p = cmul_conj_exact(lds[b], lds[(b + 1) & 2047]);
        corr[i] = atan2f(p.y, p.x);
    }
    float best = 0.0f;
    int bidx = 100;
    for (int i = lane; i < 72; i += 64) {
        float sum = 0.0f;
        for (int j = 1; j < 18; j++) sum += fabsf(__fmul_rn(T.refarg[j], corr[i + j]));
        if (sum > best || (sum == best && sum > 0.0f && i < bidx)) { best = sum; bidx = i; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        float ob = __shfl_xor(best, o);
        int oi = __shfl_xor(bidx, o);
        if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
    }
    if (lane == 0) correction[f] = (int16_t)(bidx - 36);
}

// ---- acquisition: one thread per stream runs the reference's sequential
// null search exactly (double-precision sLevel IIR, float envelope sums).
__device__ __forceinline__ float jan_abs(float2 z) { return fabsf(z.x) + fabsf(z.y); }

__global__ void k_acquire(const float2 *__restrict__ iq, const AcqJob *__restrict__ jobs, int n,
                          const float2 *__restrict__ osc, AcqResult *__restrict__ res) {
#pragma clang fp contract(off)
    const int si = blockIdx.x * blockDim.x + threadIdx.x;
    if (si >= n) return;
    const AcqJob jb = jobs[si];
    const float2 *x = iq + jb.iq_base;
    int64_t pos = jb.start;
    const int64_t end = jb.end;
    int32_t lp = jb.local_phase;
    const int32_t ph = jb.phase;
    float sLevel = 0.0f;
    float env[64];
    int32_t attempts = 0;
    auto get = [&](int32_t phase, float2 &out) -> bool {
        if (pos >= end) return false;
        float2 t = x[pos++];
        lp -= phase;
        lp = (lp + INPUT_RATE) % INPUT_RATE;
        t = cmul_exact(t, osc[lp]);
        sLevel = (float)(0.00001 * (double)jan_abs(t) + (1 - 0.00001) * (double)sLevel);
        out = t;
        return true;
    };
    float2 smp;
    for (;;) {
        attempts++;
        sLevel = 0.0f;
        for (int i = 0; i < 20 * TS; i++)
            if (!get(0, smp)) goto fail;
        int idx = 0;
        float cur = 0.0f;
        for (int i = 0; i < 50; i++) {
            if (!get(0, smp)) goto fail;
            env[idx & 63] = jan_abs(smp);
            cur += env[idx & 63];
            idx++;
        }
        int32_t counter = 0;
        bool restart = false;
        while (cur / 50 > 0.40 * sLevel) {
            if (!get(ph, smp)) goto fail;
            env[idx & 63] = jan_abs(smp);
            cur += env[idx & 63] - env[(idx - 50) & 63];
            idx++;
            if (++counter > TF) { restart = true; break; }
        }
        if (restart) continue;
        counter = 0;
        while (cur / 50 < 0.75 * sLevel) {
            if (!get(ph, smp)) goto fail;
            env[idx & 63] = hypotf(smp.x, smp.y);
            cur += env[idx & 63] - env[(idx - 50) & 63];
            idx++;
            if (++counter > TNULL + 50) { restart = true; break; }
        }
        if (restart) continue;
        res[si].window = pos;
        res[si].local_phase = lp;
        res[si].status = 0;
        res[si].attempts = attempts;
        return;
    }
fail:
    res[si].window = pos;
    res[si].local_phase = lp;
    res[si].status = -1;
    res[si].attempts = attempts;
}

// per-frame FreqCorr = sum of the chunk partials (fixed order: deterministic)
__global__ void k_fc_reduce(const float2 *__restrict__ part, int nchunks, int n, float2 *__restrict__ out) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n) return;
    float2 a = make_float2(0.0f, 0.0f);
    for (int c = 0; c < nchunks; c++) { a.x += part[f * nchunks + c].x; a.y += part[f * nchunks + c].y; }
    out[f] = a;
}

// ---- launchers -----------------------------------------------------------
hipError_t launch_fc_reduce(hipStream_t st, const float *part, int nchunks, int n, float *out) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fc_reduce, dim3((n + 63) / 64), dim3(64), 0, st, (const float2 *)part, nchunks, n, (float2 *)out);
    return hipGetLastError();
}
hipError_t launch_prs_sync(hipStream_t st, const float *iq, const dabgpu_frame *fr, int n, const OfdmTables &T,
                           int level, int32_t *si, float *mx, float *sm, bool general) {
    if (n <= 0) return hipSuccess;
    if (general) hipLaunchKernelGGL(k_prs_sync<true>, dim3(n), dim3(64), 0, st, (const float2 *)iq, fr, n, T, level, si, mx, sm);
    else hipLaunchKernelGGL(k_prs_sync<false>, dim3(n), dim3(64), 0, st, (const float2 *)iq, fr, n, T, level, si, mx, sm);
    return hipGetLastError();
}
hipError_t launch_block0(hipStream_t st, const float *iq, const dabgpu_frame *fr, int n, const OfdmTables &T,
                         int16_t *corr, bool general) {
    if (n <= 0) return hipSuccess;
    if (general) hipLaunchKernelGGL(k_block0<true>, dim3(n), dim3(64), 0, st, (const float2 *)iq, fr, n, T, corr);
    else hipLaunchKernelGGL(k_block0<false>, dim3(n), dim3(64), 0, st, (const float2 *)iq, fr, n, T, corr);
    return hipGetLastError();
}
hipError_t launch_acquire(hipStream_t st, const float *iq, const AcqJob *jobs, int n, const float2 *osc,
                          AcqResult *res) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_acquire, dim3((n + 63) / 64), dim3(64), 0, st, (const float2 *)iq, jobs, n, osc, res);
    return hipGetLastError();
}

}  // namespace dab

namespace dab {

// Recorded IQ to cf32 (dabgpu.h, DABGPU_IQ_*): one thread per 16 input values, 16-byte
// loads (u8) / 2 x 16-byte loads (s16) and 4 x 16-byte stores; HBM-bound
// (5 or 6 bytes per value).  The tail (n_values % 16) is done value by value.
template <int FMT>
__global__ __launch_bounds__(256) void k_iq_convert(const void *__restrict__ src, int64_t n_values,
                                                    float *__restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t v0 = i * 16;
    if (v0 >= n_values) return;
    float f[16];
    if (v0 + 16 <= n_values) {
        if constexpr (FMT == DABGPU_IQ_U8) {
            const uint4 w = ((const uint4 *)src)[i];
            const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int k = 0; k < 16; k++) f[k] = (float)((int)((u[k >> 2] >> (8 * (k & 3))) & 0xFFu) - 128) / 128.0f;
        } else {
            const uint4 a = ((const uint4 *)src)[2 * i], b = ((const uint4 *)src)[2 * i + 1];
            const uint32_t u[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int k = 0; k < 16; k++) f[k] = (float)(int16_t)(u[k >> 1] >> (16 * (k & 1))) * (1.0f / 32768.0f);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) ((float4 *)dst)[4 * i + q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
    } else {
        for (int64_t v = v0; v < n_values; v++) {
            if constexpr (FMT == DABGPU_IQ_U8) dst[v] = (float)((int)((const uint8_t *)src)[v] - 128) / 128.0f;
            else dst[v] = (float)((const int16_t *)src)[v] * (1.0f / 32768.0f);
        }
    }
}

hipError_t launch_iq_convert(hipStream_t st, int format, const void *src, int64_t n_values, float *dst) {
    if (n_values <= 0) return hipSuccess;
    const int64_t threads = (n_values + 15) / 16;
    const dim3 grid((unsigned)((threads + 255) / 256));
    if (format == DABGPU_IQ_U8) hipLaunchKernelGGL(k_iq_convert<DABGPU_IQ_U8>, grid, dim3(256), 0, st, src, n_values, dst);
    else if (format == DABGPU_IQ_S16) hipLaunchKernelGGL(k_iq_convert<DABGPU_IQ_S16>, grid, dim3(256), 0, st, src, n_values, dst);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace dab
