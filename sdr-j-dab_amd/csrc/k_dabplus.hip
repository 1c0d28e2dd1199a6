// k_dabplus.hip -- DAB+ superframe layer for gfx950: mp4Processor::addtoFrame +
// processSuperframe (mp4processor.cpp:107-292) for every DAB+ subchannel of every
// stream, over the CIFs one pipeline run decoded.
//
// One wave per (stream, DAB+ subchannel) walks that subchannel's CIFs in order:
// packs the 24*bitRate decoded bits into the 5-CIF byte ring (kept in HBM between
// runs, in LDS while the wave works), runs the fire-code check at the oldest block
// (firecode-checker.cpp:76-94) and, when it passes, the RS(120,110) decode of the
// RSDims interleaved codewords -- one codeword per lane, GF(2^8) tables in LDS --
// followed by the AU table and the AU CRCs (one AU per lane).  The RS decoder is a
// restatement of the reference's Karn-style decoder (reed-solomon.cpp:143-399:
// syndromes, Berlekamp-Massey, Chien search over all 255 positions, Forney), so its
// return value (errors corrected, or -1) and corrections match it exactly.
#include "dab_device.h"
#include "dab_kernels.h"

namespace dab {

constexpr int RS_NN = 255, RS_PAD = 135, RS_ROW = 121;   // LDS row stride (odd: spreads banks)

__device__ __forceinline__ int mod255(int x) { return x % 255; }

struct GfTabs {
    uint8_t exp[256];
    uint8_t log[256];
    uint16_t fire[256];      // fire-code syndrome table
    uint8_t mul[10][256];    // s * alpha^i: one lookup per Horner step of syndrome i
    uint16_t crc[256];       // CRC-CCITT (0x1021, msb first) byte table
};
static_assert(sizeof(GfTabs) == DP_TAB_BYTES, "host table layout");

__device__ __forceinline__ int gmul(const GfTabs &g, int a, int b) {
    return (a && b) ? g.exp[mod255(g.log[a] + g.log[b])] : 0;
}
__device__ __forceinline__ int gdiv(const GfTabs &g, int a, int b) {
    return a ? g.exp[mod255(RS_NN + g.log[a] - g.log[b])] : 0;
}

// Syndrome i of a codeword whose byte m (m = 0..119, full-codeword position
// 135 + m; the 135 leading pad bytes are zero and leave the Horner sum at zero)
// is at src[m * step] (reed-solomon.cpp:231-266).
__device__ __forceinline__ int rs_syndrome(const uint8_t *src, int step, int wrap, int start, int i, const GfTabs &g) {
    int s = 0, o = start;
    for (int m = 0; m < 120; m++) {
        s = src[o] ^ g.mul[i][s];
        o += step;
        if (o >= wrap) o -= wrap;
    }
    return s;
}

// decode_rs after the syndromes (reed-solomon.cpp:268-399): Berlekamp-Massey,
// Chien search over all 255 positions, error evaluator, Forney.  Returns the
// number of corrected symbols or -1, and the corrections to apply: fix_pos[k]
// (full-codeword position) ^= fix_val[k] for k < *nfix.
__device__ int rs_solve(const int (&syn)[10], const GfTabs &g, uint8_t *roots, uint8_t *locs, uint8_t *fix_pos,
                        uint8_t *fix_val, int *nfix) {
    *nfix = 0;
    int any = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) any |= syn[i];
    if (!any) return 0;
    // Berlekamp-Massey (:268-318)
    int L[11], Cr[11];
#pragma unroll
    for (int i = 0; i < 11; i++) L[i] = Cr[i] = 0;
    L[0] = 1;
    Cr[1] = 1;
    int err = syn[0], Lr = 0;
#pragma unroll
    for (int K = 1; K <= 10; K++) {
        int old[11];
#pragma unroll
        for (int i = 0; i < 11; i++) old[i] = L[i];
#pragma unroll
        for (int i = 0; i < 11; i++) L[i] ^= gmul(g, err, Cr[i]);
        if (2 * Lr < K && err != 0) {
            Lr = K - Lr;
#pragma unroll
            for (int i = 0; i < 11; i++) Cr[i] = gdiv(g, old[i], err);
        }
#pragma unroll
        for (int i = 10; i >= 1; i--) Cr[i] = Cr[i - 1];
        Cr[0] = 0;
        if (K < 10) {
            err = syn[K];
#pragma unroll
            for (int i = 1; i <= K; i++) err ^= gmul(g, syn[K - i], L[i]);
        }
    }
    int deg = 0, LL[11];
#pragma unroll
    for (int i = 0; i < 11; i++) {
        if (L[i]) deg = i;
        LL[i] = g.log[L[i]];                              // log(0) = 255
    }
    // Chien search over every position (:323-360)
    int reg[11];
#pragma unroll
    for (int j = 0; j < 11; j++) reg[j] = LL[j];
    int count = 0;
    for (int i = 1; i <= RS_NN; i++) {
        int result = 1;
#pragma unroll
        for (int j = 10; j >= 1; j--) {
            if (j <= deg && reg[j] != RS_NN) {
                reg[j] = mod255(reg[j] + j);
                result ^= g.exp[reg[j]];
            }
        }
        if (result == 0) {
            if (count < 10) { roots[count] = (uint8_t)i; locs[count] = (uint8_t)(i - 1); }
            count++;
        }
    }
    if (count != deg) return -1;
    // error evaluator (:370-399)
    int om[10], deg_omega = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        int tmp = 0;
#pragma unroll
        for (int j = i; j >= 0; j--) {
            if (j <= deg) {
                const int a = g.log[syn[i - j]];
                if (a != RS_NN && LL[j] != RS_NN) tmp ^= g.exp[mod255(a + LL[j])];
            }
        }
        if (tmp) deg_omega = i;
        om[i] = g.log[tmp];
    }
    // Forney (:183-227)
    const int dmax = (deg < 9 ? deg : 9) & ~1;
    int nf = 0;
    for (int jj = count - 1; jj >= 0; jj--) {
        const int r = roots[jj], loc = locs[jj];
        int num1 = 0;
#pragma unroll
        for (int i = 0; i < 10; i++)
            if (i <= deg_omega && om[i] != RS_NN) num1 ^= g.exp[mod255(om[i] + (i ? (i * r) % RS_NN : 0))];
        const int num2 = g.exp[(r * 254) % RS_NN];
        int den = 0;
#pragma unroll
        for (int i = 0; i <= 8; i += 2)
            if (i <= dmax && LL[i + 1] != RS_NN) den ^= g.exp[mod255(LL[i + 1] + (i ? (i * r) % RS_NN : 0))];
        if (den == 0) {
            *nfix = nf;                                  // corrections made before the failure stay
            return -1;
        }
        if (num1 != 0) {
            if (loc >= RS_NN - 10) {
                count--;
            } else {
                int c = mod255(g.log[num1] + g.log[num2]);
                c = mod255(c + RS_NN - g.log[den]);
                fix_pos[nf] = (uint8_t)loc;
                fix_val[nf] = g.exp[c];
                nf++;
            }
        }
    }
    *nfix = nf;
    return count;
}

// firecode_checker::check (firecode-checker.cpp:76-94) on 11 bytes
__device__ bool fire_ok(const uint8_t *x, const GfTabs &g) {
    uint32_t st = ((uint32_t)x[2] << 8) | x[3];
    for (int i = 4; i < 13; i++) {
        const int b = i < 11 ? x[i] : x[i - 11];          // bytes 4..10 then 0..1
        const uint32_t is = g.fire[st >> 8];
        st = ((is & 0xffu) ^ (uint32_t)b) | ((is ^ (st << 8)) & 0xff00u);
    }
    return st == 0;
}

// dabPlus_crc (mp4processor.cpp:40-61)
__device__ bool au_crc_ok(const uint8_t *msg, int len, int limit, const GfTabs &g) {
    uint32_t acc = 0xFFFF;
    const int n = len < limit ? len : limit;
    for (int i = 0; i < n; i++) acc = ((acc << 8) ^ g.crc[((acc >> 8) ^ msg[i]) & 0xFFu]) & 0xFFFFu;
    for (int i = n; i < len; i++) acc = ((acc << 8) ^ g.crc[(acc >> 8) & 0xFFu]) & 0xFFFFu;
    const uint32_t hi = len < limit ? msg[len] : 0, lo = len + 1 < limit ? msg[len + 1] : 0;
    const uint32_t crc = ~((hi << 8) | lo) & 0xFFFFu;
    return (crc ^ acc) == 0;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(64) void k_dabplus(DpJob J) {
    __shared__ GfTabs g;
    __shared__ uint8_t ring[120 * DP_MAX_RS];
    __shared__ uint8_t outv[110 * DP_MAX_RS + 16];
    __shared__ int16_t syn_s[10 * DP_MAX_RS];
    __shared__ uint8_t rl[64 * 40];
    __shared__ int32_t red[64];
    const int lane = threadIdx.x;
    const int stream = blockIdx.x / J.ndp, dp = blockIdx.x % J.ndp;
    const int br = J.dp_br[dp], sub = J.dp_sub[dp];
    const int RS = br / 8, nbytes = 3 * br, fsz = 120 * RS;
    // tables + this subchannel's ring into LDS
    for (int i = lane; i < (int)sizeof(GfTabs); i += 64) ((uint8_t *)&g)[i] = J.tabs[i];
    uint8_t *gring = J.ring + ((int64_t)stream * J.ndp + dp) * (120 * DP_MAX_RS);
    for (int i = lane; i < fsz; i += 64) ring[i] = gring[i];
    DpState st = J.state[(int64_t)stream * J.ndp + dp];
    wave_sync();
    for (int cl = 0; cl < J.ncif; cl++) {
        const int64_t rec = ((int64_t)stream * J.ncif + cl) * J.ndp + dp;
        dabgpu_superframe info;
        info.status = -1;
        info.num_aus = 0;
        info.n_corrected = 0;
        for (int i = 0; i < 7; i++) info.au_start[i] = 0;
        info.au_crc_ok = 0;
        info.reserved = 0;
        if (J.cif0 + cl < 16) {                          // de-interleaver warm-up: nothing delivered
            if (lane == 0) J.info[rec] = info;
            continue;
        }
        // addtoFrame: pack 8 bits per byte, msb first, into block `fill` (:115-121)
        const uint8_t *bits = J.msc + (((int64_t)stream * J.ncif + cl) * J.nsub + sub) * J.msc_stride;
        for (int i = lane; i < nbytes; i += 64) {
            const uint2 w = *(const uint2 *)(bits + 8 * i);
            const uint64_t v = ((uint64_t)w.y << 32) | w.x;
            uint32_t t = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) t = (t << 1) | (uint32_t)((v >> (8 * j)) & 1u);
            ring[st.fill * nbytes + i] = (uint8_t)t;
        }
        wave_sync();
        st.blocks++;
        st.fill = (st.fill + 1) % 5;
        info.status = 0;
        if (st.blocks >= 5) {
            const int base = st.fill * nbytes;
            if (!fire_ok(ring + base, g)) {
                info.status = 1;
                st.blocks = 4;
            } else {
                // processSuperframe: RS over the RSDims interleaved columns (:165-179).
                // Byte k of column j is ring[(base + j + k*RS) % fsz], so the
                // uncorrected output outv[j + k*RS] is the ring rotated by base.
                for (int i = lane; i < 110 * RS; i += 64) {
                    const int o = base + i;
                    outv[i] = ring[o < fsz ? o : o - fsz];
                }
                // syndromes: every (column, root) pair is one Horner chain on one lane
                for (int p = lane; p < 10 * RS; p += 64) {
                    const int j = p / 10, i = p - 10 * j;
                    syn_s[p] = (int16_t)rs_syndrome(ring, RS, fsz, base + j < fsz ? base + j : base + j - fsz, i, g);
                }
                wave_sync();
                int ler = 0;
                if (lane < RS) {                                 // one column per lane
                    int sy[10];
#pragma unroll
                    for (int i = 0; i < 10; i++) sy[i] = syn_s[10 * lane + i];
                    uint8_t *w = rl + lane * 40;
                    int nf = 0;
                    ler = rs_solve(sy, g, w, w + 10, w + 20, w + 30, &nf);
                    for (int f = 0; f < nf; f++) {
                        const int m = w[20 + f] - RS_PAD;
                        if (m >= 0 && m < 110) outv[lane + m * RS] ^= w[30 + f];
                    }
                }
                red[lane] = ler;
                wave_sync();
                // the reference stops at the first failing column
                int nerr = 0, fail = 0;
                for (int j = 0; j < RS && !fail; j++) {
                    const int l = red[j];
                    if (l > 0) nerr += l;
                    if (l < 0) fail = 1;
                }
                info.n_corrected = (int16_t)nerr;
                bool ok = !fail;
                if (ok) {
                    // AU table (:181-233)
                    const int dac = (outv[2] >> 6) & 1, sbr = (outv[2] >> 5) & 1;
                    int n, a[7];
                    const int end = 110 * RS;
                    switch (2 * dac + sbr) {
                    default:
                    case 0: n = 4; a[0] = 8; a[1] = outv[3] * 16 + (outv[4] >> 4);
                        a[2] = (outv[4] & 0xf) * 256 + outv[5]; a[3] = outv[6] * 16 + (outv[7] >> 4); a[4] = end; break;
                    case 1: n = 2; a[0] = 5; a[1] = outv[3] * 16 + (outv[4] >> 4); a[2] = end; break;
                    case 2: n = 6; a[0] = 11; a[1] = outv[3] * 16 + (outv[4] >> 4);
                        a[2] = (outv[4] & 0xf) * 256 + outv[5]; a[3] = outv[6] * 16 + (outv[7] >> 4);
                        a[4] = (outv[7] & 0xf) * 256 + outv[8]; a[5] = outv[9] * 16 + (outv[10] >> 4); a[6] = end; break;
                    case 3: n = 3; a[0] = 6; a[1] = outv[3] * 16 + (outv[4] >> 4);
                        a[2] = (outv[4] & 0xf) * 256 + outv[5]; a[3] = end; break;
                    }
                    info.num_aus = (int8_t)n;
                    for (int i = 0; i < 7; i++) info.au_start[i] = (int16_t)(i <= n ? a[i] : 0);
                    int bad = n;                                  // first AU with an impossible layout
                    for (int i = 0; i < n; i++) {
                        const int len = a[i + 1] - a[i] - 2;
                        if (a[i + 1] < a[i] || len >= 960 || len < 0) { bad = i; break; }
                    }
                    // one AU per lane: CRC over [a[i], a[i+1])
                    int mine = 0;
                    if (lane < bad) {
                        int ai = 0, an = 0;
                        for (int i = 0; i < 7; i++) if (i == lane) { ai = a[i]; an = a[i + 1]; }
                        const int len = an - ai - 2;
                        mine = au_crc_ok(outv + ai, len, end - ai, g) ? 1 : 0;
                    }
                    const uint64_t crcmask = __ballot(mine);
                    info.au_crc_ok = (uint8_t)(crcmask & 0x3F);
                    ok = bad == n;
                }
                info.status = ok ? 3 : 2;
                st.blocks = ok ? 0 : 4;
                if (ok) {
                    uint8_t *o = J.sf_out + rec * J.sf_stride;
                    for (int i = lane; i < 110 * RS; i += 64) o[i] = outv[i];
                }
                wave_sync();
            }
        }
        if (lane == 0) J.info[rec] = info;
    }
    for (int i = lane; i < fsz; i += 64) gring[i] = ring[i];
    if (lane == 0) J.state[(int64_t)stream * J.ndp + dp] = st;
}

hipError_t launch_dabplus(hipStream_t st, const DpJob &job) {
    if (job.ndp <= 0 || job.nstreams <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dabplus, dim3(job.nstreams * job.ndp), dim3(64), 0, st, job);
    return hipGetLastError();
}

}  // namespace dab

namespace dab {

// reedSolomon::dec batched: one lane per codeword (the a19 operator on its own).
__global__ __launch_bounds__(64) void k_rs(const uint8_t *__restrict__ in, int n, const uint8_t *__restrict__ tabs,
                                          uint8_t *__restrict__ out, int16_t *__restrict__ ret) {
    __shared__ GfTabs g;
    __shared__ uint8_t rows[64 * RS_ROW];
    __shared__ uint8_t rl[64 * 40];
    const int lane = threadIdx.x, cw = blockIdx.x * 64 + lane;
    for (int i = lane; i < (int)sizeof(GfTabs); i += 64) ((uint8_t *)&g)[i] = tabs[i];
    wave_sync();
    if (cw >= n) return;
    uint8_t *row = rows + lane * RS_ROW;
    for (int k = 0; k < 120; k++) row[k] = in[(int64_t)cw * 120 + k];
    int sy[10];
#pragma unroll
    for (int i = 0; i < 10; i++) sy[i] = rs_syndrome(row, 1, 1 << 30, 0, i, g);
    uint8_t *w = rl + lane * 40;
    int nf = 0;
    const int r = rs_solve(sy, g, w, w + 10, w + 20, w + 30, &nf);
    for (int f = 0; f < nf; f++) {
        const int m = w[20 + f] - RS_PAD;
        if (m >= 0) row[m] ^= w[30 + f];
    }
    for (int k = 0; k < 110; k++) out[(int64_t)cw * 110 + k] = row[k];
    ret[cw] = (int16_t)r;
}

hipError_t launch_rs(hipStream_t st, const uint8_t *in, int n, const uint8_t *tabs, uint8_t *out, int16_t *ret) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rs, dim3((n + 63) / 64), dim3(64), 0, st, in, n, tabs, out, ret);
    return hipGetLastError();
}

}  // namespace dab
