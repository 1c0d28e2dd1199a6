// k_ofdm.hip -- OFDM front-end helpers for gfx950:
//   k_acquire    : ofdmProcessor::run notSynced..SyncOnEndNull (ofdm-processor.cpp:274-338)
//   k_fc_reduce  : per-frame FreqCorr from the demod's partial sums
//   k_iq_convert : recorded .raw / .sdr samples to cf32
// (findIndex, processBlock_0 and processToken: k_demod.hip)
// Every sample read applies the getSamples NCO (ofdm-processor.cpp:217-226).
#include "dab_device.h"
#include "dab_kernels.h"

namespace dab {

// ---- acquisition: ofdmProcessor::run notSynced / SyncOnNull / SyncOnEndNull
// (ofdm-processor.cpp:274-338), one wave per stream.  Everything that does not depend
// on the search's outcome is computed by all 64 lanes: the NCO index of a sample is a
// closed form of its position inside the attempt (phase 0 for the 20*T_s + 50 samples
// that build sLevel, coarse+fine after), so lanes mix a block of samples and form
// their L1 norms (jan_abs) and magnitudes (abs) in parallel.  The reference's state
// machine then walks the block from LDS: the double-precision sLevel IIR rounded to
// float at every sample, the 50-sample envelope sum and the dip / end-of-dip
// thresholds.  A restart (goto notSynced) changes the mixing of the
// samples after it: the block is recomputed from there.
__device__ __forceinline__ float jan_abs(float2 z) { return fabsf(z.x) + fabsf(z.y); }

constexpr int ACQ_BLK = 1024;                       // samples per block
constexpr int ACQ_WARM = 20 * TS;                    // sLevel build-up (phase 0)
constexpr int ACQ_INIT = 50;                         // first envelope samples (phase 0)

// localPhase after reading sample p of an attempt that started at sample a with
// localPhase lpa: phase 0 for the first ACQ_WARM + ACQ_INIT samples, then `ph`
__device__ __forceinline__ int32_t acq_lp(int64_t p, int64_t a, int32_t lpa, int32_t ph) {
    const int64_t k = p - a - (ACQ_WARM + ACQ_INIT);
    if (k < 0) return lpa;
    const int64_t t = ((int64_t)lpa - (k + 1) * (int64_t)ph) % INPUT_RATE;
    return (int32_t)(t < 0 ? t + INPUT_RATE : t);
}

// Only the two chains are sequential.  Per sample the sLevel IIR needs its own chain
// (cvt, mul, add, cvt: the 0.00001 * jan_abs term is formed by all lanes beforehand,
// pj[]), the envelope sum one float add of a difference the lanes formed beforehand: the
// value leaving the 50-sample window entered 50 samples earlier, before the group or
// inside it.  While searching, lane 0 runs both chains over a group of 64 samples, then
// the 64 lanes test the 64 states side by side and the group keeps the states up to the
// first test that fails (the reference's loop stops there).  The threshold tests
// (currentStrength / 50 against 0.40 / 0.75 * sLevel, a float division compared in
// double) take a multiply by 0.02f and fall back to the IEEE division only within 2^-21
// of the threshold: the quotient and the product differ by less than 2^-22 of it.
__device__ __forceinline__ bool q50_gt(float cur, double t) {     // fl(cur / 50) > t
#pragma clang fp contract(off)
    const double qa = (double)(cur * 0.02f);
    if (fabs(qa - t) > 0x1p-21 * fabs(qa)) return qa > t;
    return (double)(cur / 50) > t;
}
__device__ __forceinline__ bool q50_lt(float cur, double t) {     // fl(cur / 50) < t
#pragma clang fp contract(off)
    const double qa = (double)(cur * 0.02f);
    if (fabs(qa - t) > 0x1p-21 * fabs(qa)) return qa < t;
    return (double)(cur / 50) < t;
}
__device__ __forceinline__ float slevel_next(float s, double pj) {
#pragma clang fp contract(off)                                     // two roundings, as the reference's mulsd + addsd
    return (float)(pj + (1 - 0.00001) * (double)s);                // ofdm-processor.cpp:225
}

template <int FMT>
__global__ __launch_bounds__(64) void k_acquire(const void *__restrict__ iq, const AcqJob *__restrict__ jobs, int n,
                                                const float2 *__restrict__ osc, AcqResult *__restrict__ res) {
#pragma clang fp contract(off)
    // a group reads up to 64 samples past its start: the arrays carry 64 zeros behind the block
    __shared__ __attribute__((aligned(16))) float ja[ACQ_BLK + 64];
    __shared__ __attribute__((aligned(16))) float hy[ACQ_BLK + 64];
    __shared__ __attribute__((aligned(16))) double pj[ACQ_BLK + 64];
    __shared__ float env[64];                        // the 50-sample envelope window (ring of 64)
    __shared__ __attribute__((aligned(16))) float dd[64];      // group: v_u - (value leaving at u)
    __shared__ __attribute__((aligned(16))) float2 sc[65];     // group: (sLevel, strength) before sample u
    const int lane = threadIdx.x;
    if ((int)blockIdx.x >= n) return;
    ja[ACQ_BLK + lane] = 0.0f;
    hy[ACQ_BLK + lane] = 0.0f;
    pj[ACQ_BLK + lane] = 0.0;
    // a latency-bound chain on one lane: first pick on its SIMD, so a search launched while
    // the pipeline's ACS waves fill the SIMDs (a sync loss) is not starved of issue slots
    __builtin_amdgcn_s_setprio(3);
    const AcqJob jb = jobs[blockIdx.x];
    const void *x = iq_stream<FMT>(iq, jb.iq_base);
    const int32_t ph = jb.phase;
    int64_t a = jb.start, pos = jb.start;            // attempt start, next unread sample
    int32_t lpa = jb.local_phase;                    // localPhase at the attempt start
    // the search state, the same in every lane (ofdm-processor.cpp:274-338)
    enum { WARM, INIT, NULLS, ENDNULL };
    int st = WARM, w = 0, idx = 0, counter = 0;
    float sLevel = 0.0f, cur = 0.0f;
    int32_t attempts = jb.attempts + 1, nosig = 0;
    int32_t att_start = attempts;                    // `attempts` when the current attempt began
    int status = -1;
    for (;;) {
        const int nb = (int)min((int64_t)ACQ_BLK, jb.end - pos);
        if (nb <= 0) break;                          // out of samples: still searching
        {
            // all of the block's loads in flight at once (a loop of dependent-looking
            // iterations issued them one latency at a time: the sequential walk below then
            // waited for 16 memory round trips per block)
            constexpr int R = ACQ_BLK / 64;
            float2 xs[R], os[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int i = lane + 64 * r;
                const int64_t p = pos + (i < nb ? i : 0);
                xs[r] = iq_at<FMT>(x, p);
                os[r] = osc[acq_lp(p, a, lpa, ph)];
            }
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int i = lane + 64 * r;
                float j = 0.0f, h = 0.0f;            // zeros past nb: a group's tail reads them
                if (i < nb) {
                    const float2 t = cmul_exact(xs[r], os[r]);
                    j = jan_abs(t);
                    h = hypotf(t.x, t.y);
                }
                ja[i] = j;
                hy[i] = h;
                pj[i] = 0.00001 * (double)j;
            }
        }
        __syncthreads();
        // The state machine runs on every lane alike (its state is the same in all 64);
        // only the two chains of a group run on lane 0 alone.
        int kind = 0, at = nb;                       // 0: block consumed, 1: restart after `at`, 2: found at `at`
        int i = 0;
        while (i < nb && kind == 0) {
            if (st == WARM) {                        // 20 T_s samples building sLevel (:280-282)
                const int e = min(nb, i + (ACQ_WARM - w));
                float sl = sLevel;
                int k = i;
                for (; k + 8 <= e; k += 8) {
#pragma unroll
                    for (int u = 0; u < 8; u++) sl = slevel_next(sl, pj[k + u]);
                }
                for (; k < e; k++) sl = slevel_next(sl, pj[k]);
                sLevel = sl;
                w += e - i;
                i = e;
                if (w == ACQ_WARM) { st = INIT; idx = 0; cur = 0.0f; }
            } else if (st == INIT) {                 // 50 samples filling the envelope (:286-292)
                const int e = min(nb, i + (ACQ_INIT - idx));
                if (lane < e - i) env[idx + lane] = ja[i + lane];
                float sl = sLevel, cs = cur;
                for (int k = i; k < e; k++) {
                    sl = slevel_next(sl, pj[k]);
                    cs += ja[k];
                }
                sLevel = sl;
                cur = cs;
                idx += e - i;
                i = e;
                if (idx == ACQ_INIT) { st = NULLS; counter = 0; }
                __syncthreads();
            } else {
                // SyncOnNull (:299-316) / SyncOnEndNull (:322-337) over a group of up to 64
                // samples: the reference tests the state, then consumes the sample (sLevel
                // and envelope step, ++counter, give up past the limit).  Lane u forms the
                // envelope's difference at sample u (the value leaving the window entered 50
                // samples earlier: the ring before the group, or this group's own sample
                // u - 50), lane 0 runs both chains over the group, then lane u tests the
                // state before sample u; the group keeps everything up to the first failure.
                const bool nulls = st == NULLS;
                const float *vs = nulls ? ja : hy;
                const int ng = min(64, nb - i);
                {
                    const float v = vs[i + lane];
                    const float old = lane >= 50 ? vs[i + lane - 50] : env[(idx + lane - 50) & 63];
                    dd[lane] = lane < ng ? v - old : 0.0f;
                }
                __syncthreads();
                if (lane == 0) {
                    float sl = sLevel, cs = cur;
#pragma unroll
                    for (int u = 0; u < 64; u++) {
                        sc[u] = make_float2(sl, cs);
                        sl = slevel_next(sl, pj[i + u]);
                        cs += dd[u];
                    }
                    sc[64] = make_float2(sl, cs);
                }
                __syncthreads();
                const float2 s = sc[lane];
                const bool pass = nulls ? q50_gt(s.y, 0.40 * (double)s.x)    // still above the dip threshold
                                        : q50_lt(s.y, 0.75 * (double)s.x);   // still inside the null
                const uint64_t fails = __ballot(!pass && lane < ng);
                const int f = fails ? (int)__builtin_ctzll(fails) : ng;
                const int lim = (nulls ? TF : TNULL + 50) - counter;        // consuming sample `lim` gives up
                int m;                                                       // samples consumed
                bool dip = false;
                if (f < ng && f <= lim) {
                    m = f;
                    if (nulls) {                     // the dip: SyncOnEndNull (:317-319)
                        dip = true;
                    } else {
                        kind = 2;                    // end of the null symbol: SyncOnPhase at sample i + f
                        at = i + f;
                    }
                } else if (lim < ng) {
                    m = lim + 1;                     // hopeless: notSynced
                    if (nulls && jb.scan && attempts > 5) { nosig++; attempts = 0; }
                    kind = 1;
                    at = i + m;
                } else {
                    m = ng;
                }
                if (lane < m) env[(idx + lane) & 63] = vs[i + lane];
                const float2 t = sc[m];
                sLevel = t.x;
                cur = t.y;
                idx += m;
                counter += m;
                i += m;
                if (dip) {
                    attempts = 0;
                    counter = 0;
                    st = ENDNULL;
                }
                __syncthreads();
            }
        }
        if (kind == 2) {
            pos += at;
            status = 0;
            break;
        }
        if (kind == 1) {                             // new attempt right after sample pos + at - 1
            const int64_t last = pos + at - 1;
            lpa = acq_lp(last, a, lpa, ph);
            a = pos = last + 1;
            st = WARM; w = 0; idx = 0; cur = 0.0f; sLevel = 0.0f; counter = 0;
            attempts++;
            att_start = attempts;
            continue;
        }
        pos += nb;
    }
    if (lane == 0) {
        AcqResult r;
        r.status = status;
        r.no_signal = nosig;
        if (status == 0) {
            r.window = pos;
            r.local_phase = acq_lp(pos - 1, a, lpa, ph);
            r.attempts = attempts;
        } else {
            // out of samples inside an attempt: the reference would block in getSample
            // until more arrive, with `attempts` counting this attempt; hand back the
            // attempt's start so that the next call, with more samples, repeats it exactly
            // (the host passes attempts - 1 in: it enters notSynced again)
            r.window = a;
            r.local_phase = lpa;
            r.attempts = att_start;
        }
        res[blockIdx.x] = r;
    }
}

// per-frame FreqCorr = sum of the chunk partials (fixed order: deterministic)
__global__ void k_fc_reduce(const float2 *__restrict__ part, int nchunks, int n, float2 *__restrict__ out) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n) return;
    float2 a = make_float2(0.0f, 0.0f);
    for (int c = 0; c < nchunks; c++) { a.x += part[f * nchunks + c].x; a.y += part[f * nchunks + c].y; }
    out[f] = a;
}

// k_fc_reduce for the pipeline's front pass, publishing what the host replay reads
// straight into its pinned buffers (startIndex, FreqCorr, SNR per frame, and the
// device error word, taken and cleared): the four small read-back copies were blit
// kernels queued between the demod and the next ACS (~45 us per step).
__global__ void k_front_publish(const float2 *__restrict__ part, int nchunks, int n, float2 *__restrict__ fc_d,
                                float2 *h_fc, const int32_t *__restrict__ si_d, int32_t *h_si,
                                const int16_t *__restrict__ snr_d, int16_t *h_snr, int32_t *err, int32_t *h_err) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f == 0) *h_err = atomicExch(err, 0);
    if (f >= n) return;
    float2 a = make_float2(0.0f, 0.0f);
    for (int c = 0; c < nchunks; c++) { a.x += part[f * nchunks + c].x; a.y += part[f * nchunks + c].y; }
    fc_d[f] = a;
    h_fc[f] = a;
    h_si[f] = si_d[f];
    h_snr[f] = snr_d[f];
}

// a back-end stream's error word, taken (cleared) and or-ed into its pinned host copy
__global__ void k_take_error(int32_t *err, int32_t *h_err) {
    if (threadIdx.x == 0) *h_err |= atomicExch(err, 0);
}

// ---- launchers -----------------------------------------------------------
hipError_t launch_take_error(hipStream_t st, int32_t *err, int32_t *h_err) {
    hipLaunchKernelGGL(k_take_error, dim3(1), dim3(64), 0, st, err, h_err);
    return hipGetLastError();
}
hipError_t launch_front_publish(hipStream_t st, const float *part, int nchunks, int n, float *fc_d, float *h_fc,
                                const int32_t *si_d, int32_t *h_si, const int16_t *snr_d, int16_t *h_snr,
                                int32_t *err, int32_t *h_err) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_front_publish, dim3((n + 63) / 64), dim3(64), 0, st, (const float2 *)part, nchunks, n,
                       (float2 *)fc_d, (float2 *)h_fc, si_d, h_si, snr_d, h_snr, err, h_err);
    return hipGetLastError();
}
hipError_t launch_fc_reduce(hipStream_t st, const float *part, int nchunks, int n, float *out) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fc_reduce, dim3((n + 63) / 64), dim3(64), 0, st, (const float2 *)part, nchunks, n, (float2 *)out);
    return hipGetLastError();
}
hipError_t launch_acquire(hipStream_t st, const void *iq, int fmt, const AcqJob *jobs, int n, const float2 *osc,
                          AcqResult *res) {
    if (n <= 0) return hipSuccess;
    if (fmt == DABGPU_IQ_F32) hipLaunchKernelGGL(k_acquire<DABGPU_IQ_F32>, dim3(n), dim3(64), 0, st, iq, jobs, n, osc, res);
    else if (fmt == DABGPU_IQ_S16) hipLaunchKernelGGL(k_acquire<DABGPU_IQ_S16>, dim3(n), dim3(64), 0, st, iq, jobs, n, osc, res);
    else if (fmt == DABGPU_IQ_U8) hipLaunchKernelGGL(k_acquire<DABGPU_IQ_U8>, dim3(n), dim3(64), 0, st, iq, jobs, n, osc, res);
    else return hipErrorInvalidValue;
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

// ---- device -> pinned host copy (dabgpu_pipe_fetch): a few waves stream 16-byte pieces
// from HBM straight into the mapped host buffer.  The runtime's copy of a device buffer
// into pinned memory runs as a blit kernel of many workgroups (rocprofv3:
// __amd_rocclr_copyBuffer) that take wave slots the next run's ACS holds
// (profiles/r04_delivered_ab.txt); this one needs `wgs` workgroups in all, and PCIe, not
// the SIMDs, paces it.  Each thread keeps 4 loads in flight before its stores.
__global__ __launch_bounds__(256) void k_to_host(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

hipError_t launch_to_host(hipStream_t st, const void *src, void *dst, size_t bytes, int wgs) {
    if (!bytes) return hipSuccess;
    if ((((uintptr_t)src | (uintptr_t)dst | bytes) & 15) || wgs <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_to_host, dim3(wgs), dim3(256), 0, st, (const uint4 *)src, (uint4 *)dst, (int64_t)(bytes / 16));
    return hipGetLastError();
}

}  // namespace dab
