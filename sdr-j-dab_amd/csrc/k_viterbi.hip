// k_viterbi.hip -- k=7 R=1/4 Viterbi decoder for gfx950 and its callers.
//
// Reference semantics (viterbi.cpp:225-242 + FULL_SPIRAL spiral-sse.c:30-698):
//   sym = clamp(soft + 127, 0, 255); branch metric sum_j sym_j ^ B_j, B in {0,255};
//   uint32 path metrics without renormalisation, start 63 / state0 = 0;
//   strict ">" picks the upper predecessor; full chainback from state 0.
//
// gfx950 design
//   k_acs       one wave64 per codeword, one trellis state per lane.  States
//               are relabelled every step (lane L holds state rotl6(L, t mod 6))
//               so each ACS butterfly is a single lane-pair exchange at xor
//               distance 32,16,8,4,2,1 (permlane32/16_swap, DPP) instead of a
//               64-way shuffle.  Branch metrics for 48 steps are built in LDS by
//               48 lanes at once (depuncturing + 16-CIF time de-interleave fused
//               into that gather).  The 64 decisions of a step come straight
//               from two v_cmp masks and land in HBM as 48-step tiles.
//   k_traceback one LANE per codeword: 64 chainbacks per wave in lock-step,
//               reading the decision tiles; bits leave through 16-B stores
//               with the energy-dispersal PRBS xor-ed in.
#include "dab_device.h"
#include "dab_kernels.h"

namespace dab {

__device__ __forceinline__ int rotl6(int x, int r) { return ((x << r) | (x >> (6 - r))) & 63; }
__device__ __forceinline__ int delay16(int i) {         // dab-concurrent.cpp:42-43
    int b = i & 15;
    int rv = ((b & 1) << 3) | ((b & 2) << 1) | ((b & 4) >> 1) | ((b & 8) >> 3);
    return 15 - rv;
}

struct CwInfo {
    int prof;
    bool valid;
    // source addressing
    const int16_t *base;   // for SRC_MOTHER/FRAG/FIC
    int64_t stream_off;    // SRC_MSC: element offset of the stream's ring
    int64_t cif;           // SRC_MSC: global CIF index
    int32_t sub_start;
};

__device__ __forceinline__ CwInfo cw_info(const VitJob &J, int cw) {
    CwInfo c;
    c.prof = 0; c.valid = true; c.base = nullptr; c.stream_off = 0; c.cif = 0; c.sub_start = 0;
    switch (J.kind) {
    case SRC_MOTHER: c.base = J.src + (int64_t)cw * J.src_stride; break;
    case SRC_FRAG:   c.base = J.src + (int64_t)cw * J.src_stride; c.prof = J.cw_prof ? J.cw_prof[cw] : 0; break;
    case SRC_FIC:    c.base = J.src + (int64_t)J.slots[cw >> 2] * FRAME_SOFT + (cw & 3) * 2304; break;
    default: {
        const int sub = cw % J.nsub;
        const int rest = cw / J.nsub;
        const int cl = rest % J.ncif;
        const int stream = rest / J.ncif;
        c.prof = sub;
        c.cif = J.cif0 + cl;
        c.valid = c.cif >= 16;                       // dab-concurrent.cpp:172-175 warm-up
        c.stream_off = (int64_t)stream * J.ring * FRAME_SOFT;
        c.sub_start = J.sub_start[sub];
    }
    }
    if (J.valid && !J.valid[cw]) c.valid = false;
    return c;
}

// soft value of punctured-input element idx of codeword c
__device__ __forceinline__ int load_elem(const VitJob &J, const CwInfo &c, int idx) {
    int64_t off;
    if (J.kind != SRC_MSC) {
        off = (c.base - J.src) + idx;
    } else {
        const int64_t g = c.cif - delay16(idx);
        if (g < 0) return 0;                          // delay lines start at zero
        const int64_t frame = g >> 2;
        const int slot = (int)(frame % J.ring);
        const int64_t loc = ((int64_t)slot * NSYM + 3 + 18 * (int)(g & 3)) * SYMBITS + c.sub_start + idx;
        if (loc < 0 || loc >= (int64_t)J.ring * FRAME_SOFT) {   // stay inside this stream's ring
            atomicOr(J.err, KERR_VITERBI);
            return 0;
        }
        off = c.stream_off + loc;
    }
    if (off < 0 || off >= J.src_len) {               // never read outside the buffer
        atomicOr(J.err, KERR_VITERBI);
        return 0;
    }
    return J.src[off];
}

// the 4 mother-code soft values of trellis step t (positions 4t..4t+3)
__device__ __forceinline__ void fetch4(const VitJob &J, const CwInfo &c, const Profile *__restrict__ pp, int t, int (&x)[4]) {
    const Profile &P = *pp;
    const int p = 4 * t;
    if (P.nseg == 0) {
#pragma unroll
        for (int e = 0; e < 4; e++) x[e] = load_elem(J, c, p + e);
        return;
    }
    const int blk = p >> 7;
    uint32_t m;
    int base, b;
    if (blk < P.blk_end[P.nseg - 1]) {
        int s = 0;
        while (blk >= P.blk_end[s]) s++;
        const int bis = blk - (s ? P.blk_end[s - 1] : 0);
        m = P.mask[s];
        const int n1 = __popc(m);
        const int o = p & 127;
        b = o & 31;
        base = P.in_base[s] + bis * 4 * n1 + (o >> 5) * n1;
    } else {
        b = p - 128 * P.blk_end[P.nseg - 1];
        if (b >= 24) {                               // beyond PI_X: the memset zeros of the
#pragma unroll                                       // viterbiBlock (deconvolve.cpp:182)
            for (int e = 0; e < 4; e++) x[e] = 0;
            return;
        }
        m = P.tail_mask;
        base = P.in_base[P.nseg];
    }
    int idx = base + __popc(m & ((1u << b) - 1u));
#pragma unroll
    for (int e = 0; e < 4; e++) {
        if ((m >> (b + e)) & 1u) { x[e] = load_elem(J, c, idx); idx++; }
        else x[e] = 0;                               // "a real do not know" (fic-handler.cpp:259)
    }
}

__device__ __forceinline__ int parity(int v) { return __popc(v) & 1; }

template <int RHO>
struct LaneMask {            // lanes whose bit (5-RHO) is set = lanes holding an upper (msb=1) state
    static constexpr uint64_t v = RHO == 0 ? 0xFFFFFFFF00000000ull : RHO == 1 ? 0xFFFF0000FFFF0000ull
                                : RHO == 2 ? 0xFF00FF00FF00FF00ull : RHO == 3 ? 0xF0F0F0F0F0F0F0F0ull
                                : RHO == 4 ? 0xCCCCCCCCCCCCCCCCull : 0xAAAAAAAAAAAAAAAAull;
};

__global__ __launch_bounds__(64) void k_acs(VitJob J) {
    __shared__ uint32_t bm[8 * VCH];
    const int lane = threadIdx.x, cw = blockIdx.x;
    const CwInfo c = cw_info(J, cw);
    if (!c.valid) return;
    const Profile *pp = J.prof + c.prof;
    const int steps = pp->nbits + 6;
    uint32_t off[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        const int i = rotl6(lane, r) & 31;               // butterfly of the state this lane holds
        const int q = parity((2 * i) & 0155) | (parity((2 * i) & 0117) << 1) | (parity((2 * i) & 0123) << 2);
        off[r] = (uint32_t)(q * VCH);
    }
    uint32_t x = lane == 0 ? 0u : 63u;                   // viterbi.cpp:360-371
    uint64_t *dec = J.dec + (J.dec_off ? J.dec_off[cw] : (int64_t)cw * J.tiles_max * VCH);
    for (int t0 = 0; t0 < steps; t0 += VCH) {
        if (lane < VCH && t0 + lane < steps) {
            int s[4];
            fetch4(J, c, pp, t0 + lane, s);
#pragma unroll
            for (int e = 0; e < 4; e++) s[e] = min(max(s[e] + 127, 0), 255);
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const int m0 = (q & 1) ? 255 : 0, m1 = (q & 2) ? 255 : 0, m2 = (q & 4) ? 255 : 0;
                bm[q * VCH + lane] = (uint32_t)((s[0] ^ m0) + (s[1] ^ m1) + (s[2] ^ m2) + (s[3] ^ m0));
            }
        }
        const int nst = min(VCH, steps - t0);
        uint32_t dlo = 0, dhi = 0;
        sfor<0, VCH / 6>([&](auto gc) {
            sfor<0, 6>([&](auto rc) {
                constexpr int rho = decltype(rc)::value;
                constexpr int j = decltype(gc)::value * 6 + rho;
                if (j < nst) {
                    const uint32_t tb = bm[off[rho] + j];
                    const uint32_t a = x + tb;
                    const uint32_t xp = xchg<(32 >> rho)>(x, lane);
                    const uint32_t b = xp + (1020u - tb);
                    const uint64_t G = __ballot(a > b), Lt = __ballot(b > a);
                    constexpr uint64_t M = LaneMask<rho>::v;
                    const uint64_t D = (G & ~M) | (Lt & M);
                    dlo = (uint32_t)llvm_amdgcn_writelane((int)(uint32_t)D, j, (int)dlo);
                    dhi = (uint32_t)llvm_amdgcn_writelane((int)(uint32_t)(D >> 32), j, (int)dhi);
                    x = min(a, b);
                }
            });
        });
        if (lane < nst) dec[t0 + lane] = ((uint64_t)dhi << 32) | dlo;
    }
}

__global__ __launch_bounds__(64) void k_traceback(VitJob J) {
    const int lane = threadIdx.x, cw = blockIdx.x * 64 + lane;
    bool act = cw < J.n_cw;
    CwInfo c;
    int N = 0;
    if (act) {
        c = cw_info(J, cw);
        act = c.valid;
        if (act) N = J.prof[c.prof].nbits;
    }
    const int steps = act ? N + 6 : 0;
    int tmax = steps;
    for (int o = 32; o > 0; o >>= 1) tmax = max(tmax, __shfl_xor(tmax, o));
    const uint64_t *dec = J.dec + (act ? (J.dec_off ? J.dec_off[cw] : (int64_t)cw * J.tiles_max * VCH) : 0);
    uint8_t *out = J.out + (act ? (int64_t)cw * J.out_stride : 0);
    int lr = 0;                                          // lane index holding the traced state
    uint32_t w = 0;
    int rho = (tmax - 1) % 6;
    for (int t = tmax - 1; t >= 0; t--) {
        if (t < steps) {
            const int p = 5 - rho;
            const uint64_t D = dec[t];
            const int u = (lr >> p) & 1;                 // decoded bit of step t
            const int d = (int)((D >> lr) & 1ull);       // predecessor's msb
            lr = (lr & ~(1 << p)) | (d << p);
            if (t < N) {
                w |= (uint32_t)u << (t & 31);
                if ((t & 31) == 0) {
                    if (J.prbs) w ^= J.prbs_words[t >> 5];
                    if (t + 32 <= N) {
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            const uint32_t nib = (w >> (4 * k)) & 0xFu;
                            *(uint32_t *)(out + t + 4 * k) = (nib * 0x00204081u) & 0x01010101u;
                        }
                    } else {
                        for (int i = 0; t + i < N; i++) out[t + i] = (uint8_t)((w >> i) & 1u);
                    }
                    w = 0;
                }
            }
        }
        rho = rho == 0 ? 5 : rho - 1;
    }
}

// FIB CRC check (dab-constants.h:310-340): invert the 16 CRC bits in place, run
// CRC-CCITT from all-ones over 256 bits, pass iff the register ends at zero.
__global__ void k_fic_post(uint8_t *__restrict__ bits, uint8_t *__restrict__ ok, int n_fib) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_fib) return;
    uint8_t *b = bits + (int64_t)f * 256;
    for (int i = 240; i < 256; i++) b[i] ^= 1;
    uint32_t r = 0xFFFF;
    for (int i = 0; i < 256; i++) {
        const uint32_t top = (r >> 15) & 1u;
        r = (r << 1) & 0xFFFFu;
        if (top ^ b[i]) r ^= 0x1021u;
    }
    ok[f] = r == 0;
}

hipError_t launch_viterbi(hipStream_t st, const VitJob &job) {
    if (job.n_cw <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_acs, dim3(job.n_cw), dim3(64), 0, st, job);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_traceback, dim3((job.n_cw + 63) / 64), dim3(64), 0, st, job);
    return hipGetLastError();
}

hipError_t launch_acs(hipStream_t st, const VitJob &job) {
    if (job.n_cw <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_acs, dim3(job.n_cw), dim3(64), 0, st, job);
    return hipGetLastError();
}
hipError_t launch_traceback(hipStream_t st, const VitJob &job) {
    if (job.n_cw <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_traceback, dim3((job.n_cw + 63) / 64), dim3(64), 0, st, job);
    return hipGetLastError();
}

hipError_t launch_fic_post(hipStream_t st, uint8_t *bits, uint8_t *ok, int n_fib) {
    if (n_fib <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fic_post, dim3((n_fib + 63) / 64), dim3(64), 0, st, bits, ok, n_fib);
    return hipGetLastError();
}

}  // namespace dab
