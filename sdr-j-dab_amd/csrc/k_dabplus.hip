// k_dabplus.hip -- DAB+ superframe layer for gfx950: mp4Processor::addtoFrame +
// processSuperframe (mp4processor.cpp:107-292) for every DAB+ subchannel of every
// stream, over the CIFs one pipeline run decoded.
//
// Two kernels per run.  k_dp_superframe evaluates every superframe candidate of
// the run in parallel -- one wave per (stream, subchannel, CIF): the fire code at
// the oldest of the 5 blocks ending at that CIF and, where it holds, the RS(120,110)
// decode of the RSDims interleaved codewords, the AU table and the AU CRCs.
// k_dp_walk then runs the reference's sequential block counting (blocksInBuffer)
// over the candidates' verdicts, which decides which of them the reference would
// have evaluated, and carries the last 4 CIFs and the state to the next run.  The
// RS decoder is a restatement of the reference's Karn-style decoder
// (reed-solomon.cpp:143-399: syndromes, Berlekamp-Massey, Chien search over all 255
// positions, Forney), so its return value (errors corrected, or -1) and
// corrections match it exactly.
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
    uint16_t pow8[1024];     // x^(8d) mod the CRC polynomial
};
static_assert(sizeof(GfTabs) == FIBCRC_OFF, "host table layout (the FIB CRC table follows)");

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
__device__ __forceinline__ bool fire_ok(const uint32_t (&x)[11], const uint16_t *fire) {
    uint32_t st = (x[2] << 8) | x[3];
#pragma unroll
    for (int i = 4; i < 13; i++) {
        const uint32_t b = i < 11 ? x[i] : x[i - 11];     // bytes 4..10 then 0..1
        const uint32_t is = fire[st >> 8];
        st = ((is & 0xffu) ^ b) | ((is ^ (st << 8)) & 0xff00u);
    }
    return st == 0;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// byte i of one CIF's decoded bits, 8 bits msb first (addtoFrame, mp4processor.cpp:115-121)
__device__ __forceinline__ uint32_t pack_byte(const uint8_t *bits, int i) {
    const uint2 w = *(const uint2 *)(bits + 8 * i);
    uint32_t t = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) t = (t << 1) | ((w.x >> (8 * j)) & 1u);
#pragma unroll
    for (int j = 0; j < 4; j++) t = (t << 1) | ((w.y >> (8 * j)) & 1u);
    return t;
}

// Byte p of the superframe candidate ending at CIF cl of this run: the 5 blocks
// cl-4..cl in delivery order, i.e. the reference's ring read from its oldest block
// (mp4processor.cpp:128-140).  Blocks before the run come from the carry (the
// previous run's last 4 CIFs, oldest first).
__device__ __forceinline__ uint32_t window_byte(const DpJob &J, const uint8_t *carry, int stream, int sub,
                                                int nbytes, int cl, int p) {
    const int b = p / nbytes, w = p - b * nbytes, q = cl - 4 + b;
    if (q < 0) return carry[(q + 4) * nbytes + w];
    const uint8_t *src = J.msc + (((int64_t)stream * J.ncif + q) * J.nsub + sub) * J.msc_stride;
    return J.packed ? src[w] : pack_byte(src, w);
}

// Bytes 4d .. 4d+3 of the same window as one little-endian word (packed MSC with 4-byte
// aligned rows: a CIF block is 3 * bitRate bytes, a multiple of 24, so no word straddles two)
__device__ __forceinline__ uint32_t window_word(const DpJob &J, const uint8_t *carry, int stream, int sub,
                                                int nbytes, int cl, int d) {
    const int p = 4 * d, b = p / nbytes, w = p - b * nbytes, q = cl - 4 + b;
    if (q < 0) return *(const uint32_t *)(carry + (q + 4) * nbytes + w);
    return *(const uint32_t *)(J.msc + (((int64_t)stream * J.ncif + q) * J.nsub + sub) * J.msc_stride + w);
}
__device__ __forceinline__ bool words_ok(const DpJob &J) {
    return J.packed && (((uintptr_t)J.msc | (uintptr_t)J.msc_stride | (uintptr_t)J.ring) & 3) == 0;
}
// the window's fsz bytes into LDS: every load of a lane in flight before its first store
// (a load-store pair per byte would wait out one memory round trip per byte)
__device__ __forceinline__ void window_to_lds(const DpJob &J, const uint8_t *carry, int stream, int sub, int nbytes,
                                              int cl, int fsz, uint8_t *dst, int lane) {
    if (words_ok(J)) {
        const int nw = fsz >> 2;                         // fsz = 120 RS: a multiple of 4
        uint32_t *d32 = (uint32_t *)dst;
        for (int d0 = 0; d0 < nw; d0 += 8 * 64) {
            uint32_t v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int d = d0 + 64 * k + lane;
                v[k] = d < nw ? window_word(J, carry, stream, sub, nbytes, cl, d) : 0u;
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int d = d0 + 64 * k + lane;
                if (d < nw) d32[d] = v[k];
            }
        }
        return;
    }
    for (int p0 = 0; p0 < fsz; p0 += 8 * 64) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int p = p0 + 64 * k + lane;
            v[k] = p < fsz ? window_byte(J, carry, stream, sub, nbytes, cl, p) : 0u;
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int p = p0 + 64 * k + lane;
            if (p < fsz) dst[p] = (uint8_t)v[k];
        }
    }
}

// a * b in GF(2)[x] / (x^16 + x^12 + x^5 + 1)
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 15; k >= 0; k--) {
        r = ((r << 1) ^ ((r & 0x8000u) ? 0x1021u : 0u)) & 0xFFFFu;
        if ((b >> k) & 1u) r ^= a;
    }
    return r;
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

// Superframe candidates.  k_dp_fire, one wave per (stream, DAB+ subchannel), one lane
// per CIF of the run: the fire code at the oldest block of the 5-CIF window ending at
// that CIF (firecode-checker.cpp:76-94); a window that holds an undelivered CIF or
// fails is marked 0, a passing one is queued (about one CIF in five once the
// superframes are aligned).  k_dp_superframe then runs processSuperframe
// (mp4processor.cpp:146-292) on the queued candidates only -- RS(120,110) over the
// RSDims interleaved columns, AU table, AU CRCs -- as a grid of resident waves that load
// the GF tables once and take candidates from the queue (round 1 launched one wave per
// candidate, each copying the tables, four in five only to fail the fire code).  Which
// candidates the reference actually evaluates depends on the superframe state
// (blocksInBuffer), walked afterwards by k_dp_walk; the verdict of every candidate
// (0 fire code failed, 2 rejected, 3 decoded) goes to J.code, the record and the
// corrected bytes of a passing one to their slots.
// The work of one superframe is spread over the wave: syndromes as direct sums
// (lane = column x a slice of its rows), Berlekamp-Massey/Chien/Forney one column
// per lane, each AU CRC in 64 slices joined by x^(8d) shifts (the CRC is linear).
__global__ __launch_bounds__(64) void k_dp_fire(DpJob J) {
    __shared__ uint16_t fire[256];
    const int lane = threadIdx.x, sd = blockIdx.x;      // sd = stream * ndp + dp
    const int stream = sd / J.ndp, dp = sd - stream * J.ndp;
    const int br = J.dp_br[dp], sub = J.dp_sub[dp], nbytes = 3 * br;
    const uint16_t *tf = (const uint16_t *)(J.tabs + offsetof(GfTabs, fire));
    for (int i = lane; i < 256; i += 64) fire[i] = tf[i];
    wave_sync();
    const uint8_t *carry = J.ring + (int64_t)sd * (120 * DP_MAX_RS);
    for (int c0 = 0; c0 < J.ncif; c0 += 64) {              // wave-uniform trip count
        const int cl = c0 + lane;
        bool ok = false;
        if (cl < J.ncif) {
            // a window holding an undelivered CIF (de-interleaver warm-up, or a CIF slot the
            // stream did not fill in this run) is never evaluated
            ok = !(cl >= J.ncifs[stream] || J.cif0s[stream] + cl - 4 < 16);
            if (ok) {
                uint32_t x[11];
#pragma unroll
                for (int p = 0; p < 11; p++) x[p] = window_byte(J, carry, stream, sub, nbytes, cl, p);
                ok = fire_ok(x, fire);
            }
            J.code[(int64_t)sd * J.ncif + cl] = ok ? 1 : 0;
        }
        // one queue reservation per wave (same-address atomics serialise in L2)
        const uint64_t bal = __ballot(ok);
        int base = 0;
        if (lane == 0 && bal) base = atomicAdd(J.ncand, (int)__popcll(bal));
        base = __shfl(base, 0, 64);
        if (ok) J.cand[base + __popcll(bal & ((1ull << lane) - 1ull))] = sd * J.ncif + cl;
    }
}

// processSuperframe (mp4processor.cpp:146-292) of the candidate window ending at CIF cl of
// (stream, DAB+ subchannel) sd, by one wave: RS(120,110) over the RSDims columns, the AU
// table and AU CRCs; the verdict to J.code, the record and corrected bytes to their slots.
// LDS: sfb [120 * DP_MAX_RS], syn_s [10 * DP_MAX_RS], rl [64 * 40], red [64] of the wave.
__device__ void sf_decode(const DpJob &J, const GfTabs &g, int sd, int cl, uint8_t *sfb, uint32_t *syn_s,
                          uint8_t *rl, int32_t *red, int lane) {
    const int stream = sd / J.ndp, dp = sd - stream * J.ndp;
    const int br = J.dp_br[dp], sub = J.dp_sub[dp];
    const int RS = br / 8, nbytes = 3 * br, fsz = 120 * RS, end = 110 * RS;
    uint8_t *code = J.code + (int64_t)sd * J.ncif + cl;
    const uint8_t *carry = J.ring + (int64_t)sd * (120 * DP_MAX_RS);
    window_to_lds(J, carry, stream, sub, nbytes, cl, fsz, sfb, lane);
    for (int p = lane; p < 10 * RS; p += 64) syn_s[p] = 0;
    wave_sync();
    // syndromes S_i = sum_m r_m alpha^(i (119-m)) per column: the Horner sums of
    // reed-solomon.cpp:231-266 (roots alpha^0..alpha^9, the 135 zero pad bytes
    // contribute nothing).  Lane -> column lane % RS, rows lane / RS + k * (64 / RS).
    const int per = 64 / RS;
    if (lane < per * RS) {
        const int j = lane % RS;
        uint32_t acc[10];
#pragma unroll
        for (int i = 0; i < 10; i++) acc[i] = 0;
        for (int m = lane / RS; m < 120; m += per) {
            const int r = sfb[j + m * RS];
            if (r) {
                const int t = 119 - m;
                int e = g.log[r];
                acc[0] ^= g.exp[e];
#pragma unroll
                for (int i = 1; i < 10; i++) {
                    e += t;
                    if (e >= RS_NN) e -= RS_NN;
                    acc[i] ^= g.exp[e];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 10; i++)
            if (acc[i]) atomicXor(&syn_s[10 * j + i], acc[i]);
    }
    wave_sync();
    int ler = 0;
    if (lane < RS) {                                     // one column per lane
        int sy[10];
#pragma unroll
        for (int i = 0; i < 10; i++) sy[i] = (int)syn_s[10 * lane + i];
        uint8_t *w = rl + lane * 40;
        int nf = 0;
        ler = rs_solve(sy, g, w, w + 10, w + 20, w + 30, &nf);
        for (int f = 0; f < nf; f++) {
            const int m = w[20 + f] - RS_PAD;
            if (m >= 0 && m < 110) sfb[lane + m * RS] ^= w[30 + f];
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
    dabgpu_superframe info;
    info.status = 2;
    info.num_aus = 0;
    info.n_corrected = (int16_t)nerr;
    for (int i = 0; i < 7; i++) info.au_start[i] = 0;
    info.au_crc_ok = 0;
    info.reserved = 0;
    bool ok = !fail;
    if (ok) {
        // AU table (:181-233)
        const int dac = (sfb[2] >> 6) & 1, sbr = (sfb[2] >> 5) & 1;
        int n, a[7];
        switch (2 * dac + sbr) {
        default:
        case 0: n = 4; a[0] = 8; a[1] = sfb[3] * 16 + (sfb[4] >> 4);
            a[2] = (sfb[4] & 0xf) * 256 + sfb[5]; a[3] = sfb[6] * 16 + (sfb[7] >> 4); a[4] = end; break;
        case 1: n = 2; a[0] = 5; a[1] = sfb[3] * 16 + (sfb[4] >> 4); a[2] = end; break;
        case 2: n = 6; a[0] = 11; a[1] = sfb[3] * 16 + (sfb[4] >> 4);
            a[2] = (sfb[4] & 0xf) * 256 + sfb[5]; a[3] = sfb[6] * 16 + (sfb[7] >> 4);
            a[4] = (sfb[7] & 0xf) * 256 + sfb[8]; a[5] = sfb[9] * 16 + (sfb[10] >> 4); a[6] = end; break;
        case 3: n = 3; a[0] = 6; a[1] = sfb[3] * 16 + (sfb[4] >> 4);
            a[2] = (sfb[4] & 0xf) * 256 + sfb[5]; a[3] = end; break;
        }
        info.num_aus = (int8_t)n;
        for (int i = 0; i < 7; i++) info.au_start[i] = (int16_t)(i <= n ? a[i] : 0);
        int bad = n;                                     // first AU with an impossible layout
        for (int i = 0; i < n; i++) {
            const int len = a[i + 1] - a[i] - 2;
            if (a[i + 1] < a[i] || len >= 960 || len < 0) { bad = i; break; }
        }
        // dabPlus_crc (mp4processor.cpp:40-61) of AU i over [a[i], a[i+1]): lane l
        // runs the table CRC over its slice (lane 0 from the 0xFFFF preset, the others
        // from 0), shifts it past the bytes after the slice, and the slices XOR
        // together.  Bytes past the superframe read as zero.
        uint32_t mask = 0;
        for (int i = 0; i < bad; i++) {
            const int ai = a[i], len = a[i + 1] - ai - 2, limit = end - ai;
            const int cs = (len + 63) >> 6;
            const int k0 = min(len, lane * cs), k1 = min(len, k0 + cs);
            uint32_t acc = lane == 0 ? 0xFFFFu : 0u;
            for (int k = k0; k < k1; k++) {
                const uint32_t b = k < limit ? sfb[ai + k] : 0u;
                acc = ((acc << 8) ^ g.crc[((acc >> 8) ^ b) & 0xFFu]) & 0xFFFFu;
            }
            if (acc) acc = crc_mulmod(acc, g.pow8[len - k1]);
            acc = wave_xor(acc);
            const uint32_t hi = len < limit ? sfb[ai + len] : 0u, lo = len + 1 < limit ? sfb[ai + len + 1] : 0u;
            if (((~((hi << 8) | lo) & 0xFFFFu) ^ acc) == 0) mask |= 1u << i;
        }
        info.au_crc_ok = (uint8_t)(mask & 0x3F);
        ok = bad == n;
    }
    if (ok) {
        info.status = 3;
        uint8_t *o = J.sf_out + (((int64_t)stream * J.ncif + cl) * J.ndp + dp) * J.sf_stride;
        for (int i = lane; i < end; i += 64) o[i] = sfb[i];
    }
    if (lane == 0) {
        J.info[((int64_t)stream * J.ncif + cl) * J.ndp + dp] = info;
        *code = (uint8_t)info.status;
    }
}

__global__ __launch_bounds__(64) void k_dp_superframe(DpJob J) {
    __shared__ GfTabs g;
    __shared__ __attribute__((aligned(16))) uint8_t sfb[120 * DP_MAX_RS];
    __shared__ uint32_t syn_s[10 * DP_MAX_RS];
    __shared__ uint8_t rl[64 * 40];
    __shared__ int32_t red[64];
    const int lane = threadIdx.x;
    const uint32_t *tabs32 = (const uint32_t *)J.tabs;
    for (int i = lane; i < (int)sizeof(GfTabs) / 4; i += 64) ((uint32_t *)&g)[i] = tabs32[i];
    const int ncand = *J.ncand;                          // k_dp_fire's queue (same stream, before)
    for (int ci = blockIdx.x; ci < ncand; ci += gridDim.x) {
        wave_sync();                                         // the previous candidate's LDS reads are done
        const int id = J.cand[ci];
        sf_decode(J, g, id / J.ncif, id % J.ncif, sfb, syn_s, rl, red, lane);
    }
}

// The superframe state machine of addtoFrame (mp4processor.cpp:107-145) over the
// run's CIFs, one wave per (stream, DAB+ subchannel): blocksInBuffer decides which
// candidates are evaluated; their verdicts come from k_dp_superframe.  Writes the
// records of the CIFs without an evaluated superframe, the state, and the carry
// (the run's last 4 CIFs as bytes) for the next run.
// addtoFrame's block counting (mp4processor.cpp:107-145) over the run's CIFs of sd, by one
// wave, and the carry (the run's last 4 CIFs) for the next run; nc: LDS [4 * 3 * 384]
__device__ void dp_walk(const DpJob &J, int sd, uint8_t *nc, int lane) {
    const int stream = sd / J.ndp, dp = sd - stream * J.ndp;
    const int br = J.dp_br[dp], sub = J.dp_sub[dp], nbytes = 3 * br;
    DpState st = J.state[sd];
    const uint8_t *code = J.code + (int64_t)sd * J.ncif;
    const int nd = J.ncifs[stream];                     // CIFs this stream delivered
    const int64_t cif0 = J.cif0s[stream];
    for (int c0 = 0; c0 < J.ncif; c0 += 64) {
        const int cl = c0 + lane;
        const int v = cl < J.ncif ? code[cl] : 0;
        int fs = 0;
        const int nc = min(64, J.ncif - c0);
        for (int i = 0; i < nc; i++) {                  // uniform
            int s;
            if (c0 + i >= nd || cif0 + c0 + i < 16) {
                s = -1;                                  // not delivered (warm-up, or past the stream's CIFs)
            } else {
                st.blocks++;
                st.fill = (st.fill + 1) % 5;
                s = 0;
                if (st.blocks >= 5) {
                    const int cd = __builtin_amdgcn_readlane(v, i);
                    s = cd == 0 ? 1 : cd;
                    st.blocks = cd == 3 ? 0 : 4;
                }
            }
            if (lane == i) fs = s;
        }
        if (cl < J.ncif && fs < 2) {
            dabgpu_superframe info;
            info.status = (int8_t)fs;
            info.num_aus = 0;
            info.n_corrected = 0;
            for (int i = 0; i < 7; i++) info.au_start[i] = 0;
            info.au_crc_ok = 0;
            info.reserved = 0;
            J.info[((int64_t)stream * J.ncif + cl) * J.ndp + dp] = info;
        }
    }
    // carry = the stream's last 4 delivered CIFs (oldest first); with fewer than 4 new
    // ones the older part comes from the previous carry (staged: it is overwritten)
    uint8_t *carry = J.ring + (int64_t)sd * (120 * DP_MAX_RS);
    for (int p0 = 0; p0 < 4 * nbytes; p0 += 8 * 64) {    // a lane's loads in flight together
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int p = p0 + 64 * k + lane;
            v[k] = 0;
            if (p < 4 * nbytes) {
                const int b = p / nbytes, w = p - b * nbytes, q = nd - 4 + b;
                const uint8_t *src = J.msc + (((int64_t)stream * J.ncif + (q >= 0 ? q : 0)) * J.nsub + sub) * J.msc_stride;
                v[k] = q >= 0 ? (J.packed ? src[w] : pack_byte(src, w)) : carry[(q + 4) * nbytes + w];
            }
        }
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (p0 + 64 * k + lane < 4 * nbytes) nc[p0 + 64 * k + lane] = (uint8_t)v[k];
    }
    wave_sync();
    for (int p = lane; p < 4 * nbytes; p += 64) carry[p] = nc[p];
    if (lane == 0) J.state[sd] = st;
}

__global__ __launch_bounds__(64) void k_dp_walk(DpJob J) {
    __shared__ uint8_t nc[4 * 3 * 384];
    dp_walk(J, blockIdx.x, nc, threadIdx.x);
}

// The whole layer for one (stream, DAB+ subchannel) in one workgroup of DP_WAVES waves: the
// fire code of every CIF window (one thread per CIF), the passing candidates' superframes
// (the waves take them in turn), then the walk -- one launch instead of a queue reset and
// three dependent launches, the GF tables loaded once per workgroup.  The workgroup's own
// verdicts are all the walk reads, so no grid-wide step.
constexpr int DP_WAVES = 8;
__global__ __launch_bounds__(64 * DP_WAVES) void k_dp_layer(DpJob J) {
    __shared__ __attribute__((aligned(16))) GfTabs g;
    __shared__ __attribute__((aligned(16))) uint8_t sfb[DP_WAVES][120 * DP_MAX_RS];
    __shared__ uint32_t syn_s[DP_WAVES][10 * DP_MAX_RS];
    __shared__ uint8_t rl[DP_WAVES][64 * 40];
    __shared__ int32_t red[DP_WAVES][64];
    __shared__ int16_t cand[4 * 512];
    __shared__ int32_t ncand;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, sd = blockIdx.x;
    const int stream = sd / J.ndp, dp = sd - stream * J.ndp;
    const int br = J.dp_br[dp], sub = J.dp_sub[dp], nbytes = 3 * br;
    const uint32_t *tabs32 = (const uint32_t *)J.tabs;
    for (int i = t; i < (int)sizeof(GfTabs) / 4; i += 64 * DP_WAVES) ((uint32_t *)&g)[i] = tabs32[i];
    if (t == 0) ncand = 0;
    __syncthreads();
    const uint8_t *carry = J.ring + (int64_t)sd * (120 * DP_MAX_RS);
    for (int cl = t; cl < J.ncif; cl += 64 * DP_WAVES) {
        // a window holding an undelivered CIF (de-interleaver warm-up, or a CIF slot the
        // stream did not fill in this run) is never evaluated
        bool ok = !(cl >= J.ncifs[stream] || J.cif0s[stream] + cl - 4 < 16);
        if (ok) {
            uint32_t x[11];
#pragma unroll
            for (int p = 0; p < 11; p++) x[p] = window_byte(J, carry, stream, sub, nbytes, cl, p);
            ok = fire_ok(x, g.fire);
        }
        J.code[(int64_t)sd * J.ncif + cl] = ok ? 1 : 0;
        if (ok) cand[atomicAdd(&ncand, 1)] = (int16_t)cl;
    }
    __syncthreads();
    const int nc = ncand;
    for (int ci = w; ci < nc; ci += DP_WAVES) {
        sf_decode(J, g, sd, cand[ci], sfb[w], syn_s[w], rl[w], red[w], lane);
        wave_sync();                                     // this wave's LDS reads are done
    }
    __syncthreads();                                     // every verdict of sd written (J.code)
    if (w == 0) dp_walk(J, sd, sfb[1], lane);            // (the carry staging reuses an idle stage)
    if (!J.sf_compact) return;
    // compact output: the run's decoded superframes of sd in CIF order (after the walk,
    // status 3 marks exactly the ones the reference evaluated and decoded), slot k of the
    // k-th; the record's `reserved` byte carries k (0xFF: not stored)
    __syncthreads();                                     // the walk's records are written
    if (w == 0) {
        int k = 0;
        for (int c0 = 0; c0 < J.ncif; c0 += 64) {
            const int cl = c0 + lane;
            dabgpu_superframe *r = cl < J.ncif ? &J.info[((int64_t)stream * J.ncif + cl) * J.ndp + dp] : nullptr;
            const bool dec = r && r->status == 3;
            const uint64_t bal = __ballot(dec);
            const int kk = k + __popcll(bal & ((1ull << lane) - 1ull));
            if (dec) {
                r->reserved = (uint8_t)(kk < J.kmax ? kk : 0xFF);
                if (kk < J.kmax) cand[kk] = (int16_t)cl;
            } else if (r) {
                r->reserved = 0xFF;
            }
            k += __popcll(bal);
        }
        if (lane == 0) ncand = k < J.kmax ? k : J.kmax;
    }
    __syncthreads();
    const int nk = ncand, end = 110 * (br / 8);
    for (int q = w; q < nk; q += DP_WAVES) {             // a wave per superframe, a byte per lane
        const uint8_t *src = J.sf_out + (((int64_t)stream * J.ncif + cand[q]) * J.ndp + dp) * J.sf_stride;
        uint8_t *dst = J.sf_compact + ((int64_t)sd * J.kmax + q) * J.sf_stride;
        for (int i = lane; i < end; i += 64) dst[i] = src[i];
    }
}

hipError_t launch_dabplus(hipStream_t st, const DpJob &job) {
    if (job.ndp <= 0 || job.nstreams <= 0) return hipSuccess;
    if (job.ncif < 4) return hipErrorInvalidValue;       // the carry holds the last 4 CIFs
    static const bool split = [] { const char *e = getenv("DABGPU_DP_SPLIT"); return e && e[0] == '1'; }();   // A/B
    if (job.sf_compact && job.ncif > 4 * 512) return hipErrorInvalidValue;   // the fused layer only
    if (job.sf_compact || (!split && job.ncif <= 4 * 512)) {
        hipLaunchKernelGGL(k_dp_layer, dim3(job.nstreams * job.ndp), dim3(64 * DP_WAVES), 0, st, job);
        return hipGetLastError();
    }
    hipError_t e = hipMemsetAsync(job.ncand, 0, sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_dp_fire, dim3(job.nstreams * job.ndp), dim3(64), 0, st, job);
    // resident waves (about 9 per CU at 16.5 KB of LDS each) draining the queue
    const int nmax = job.nstreams * job.ndp * job.ncif;
    hipLaunchKernelGGL(k_dp_superframe, dim3(nmax < 256 * 8 ? nmax : 256 * 8), dim3(64), 0, st, job);
    hipLaunchKernelGGL(k_dp_walk, dim3(job.nstreams * job.ndp), dim3(64), 0, st, job);
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
