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

// XCD-aware block order (cdna_hip_programming.md T1): blocks b with equal b % 8
// share an XCD's L2; give each such group a contiguous range of codewords so the
// 16 CIFs that read the same ring rows (time de-interleave) decode on one L2.
__device__ __forceinline__ int xcd_order(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// Per-codeword source, resolved once per wave.
struct Src {
    const int16_t *base;   // first input element (SRC_MSC: the stream's ring)
    int prof;              // profile index
    int row;               // output / decision row of this codeword
    bool valid;
};

// SRC_MSC logical order (stream, subchannel, CIF) -- consecutive CIFs of one
// subchannel share 15 of their 16 source rows; output rows stay
// ((stream * ncif) + cif) * nsub + sub.
template <int KIND>
__device__ __forceinline__ Src src_of(const VitJob &J, int logical, int32_t *rowoff, int lane) {
    Src c;
    c.prof = 0;
    c.valid = true;
    c.row = logical;
    if constexpr (KIND == SRC_MOTHER) {
        c.base = J.src + (int64_t)logical * J.src_stride;
    } else if constexpr (KIND == SRC_FRAG) {
        c.base = J.src + (int64_t)logical * J.src_stride;
        c.prof = J.cw_prof ? J.cw_prof[logical] : 0;
    } else if constexpr (KIND == SRC_FIC) {
        c.base = J.src + (int64_t)J.slots[logical >> 2] * FRAME_SOFT + (logical & 3) * 2304;
    } else {
        const int cl = logical % J.ncif;
        const int rest = logical / J.ncif;
        const int sub = rest % J.nsub;
        const int stream = rest / J.nsub;
        c.row = (stream * J.ncif + cl) * J.nsub + sub;
        c.prof = sub;
        const int64_t cif = J.cif0 + cl;
        c.valid = cif >= 16;                           // dab-concurrent.cpp:172-175 warm-up
        c.base = J.src + (int64_t)stream * J.ring * FRAME_SOFT;
        if (lane < 16) {
            // element idx of CIF n comes from CIF n - d[idx & 15] (dab-concurrent.cpp:42-43,162-169)
            const int b = lane;
            const int rv = ((b & 1) << 3) | ((b & 2) << 1) | ((b & 4) >> 1) | ((b & 8) >> 3);
            const int64_t g = cif - (15 - rv);
            int32_t ro = -1;                           // delay line still empty: zeros
            if (g >= 0) {
                const int slot = (int)((g >> 2) % J.ring);
                ro = (slot * NSYM + 3 + 18 * (int)(g & 3)) * SYMBITS + J.sub_start[sub];
                const Profile &P = J.prof[sub];
                if (ro < 0 || (int64_t)ro + P.frag > (int64_t)J.ring * FRAME_SOFT) {
                    atomicOr(J.err, KERR_VITERBI);     // never read outside the stream's ring
                    ro = -1;
                }
            }
            rowoff[lane] = ro;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (J.valid && !J.valid[c.row]) c.valid = false;
    if constexpr (KIND != SRC_MSC) {
        const Profile &P = J.prof[c.prof];
        const int64_t need = P.nseg ? P.frag : 4 * (int64_t)(P.nbits + 6);
        const int64_t o = c.base - J.src;
        if (c.valid && (o < 0 || o + need > J.src_len)) {   // never read outside the buffer
            if (lane == 0) atomicOr(J.err, KERR_VITERBI);
            c.valid = false;
        }
    }
    return c;
}

// Element offsets (from c.base) of the 4 mother-code soft values of trellis step t
// (positions 4t..4t+3) with the depuncturing of deconvolve.cpp:172-237 /
// fic-handler.cpp:241-270.  keep bit e = 0 marks an erasure ("a real do not know",
// fic-handler.cpp:259, or the zero tail of deconvolve.cpp:182); its offset is a
// safe in-bounds dummy so the 4 loads can be issued unconditionally.
// a Profile as wave-uniform registers: only constant indices below, so nothing
// spills to scratch and nothing goes through the vector memory queue
struct ProfR {
    int nbits, nseg, last_end, tail_base;
    uint32_t mask[4], tail_mask;
    int blk_end[4], in_base[4];
};
__device__ __forceinline__ ProfR prof_regs(const Profile *p) {
    ProfR r;
    r.nbits = __builtin_amdgcn_readfirstlane(p->nbits);
    r.nseg = __builtin_amdgcn_readfirstlane(p->nseg);
    r.tail_mask = __builtin_amdgcn_readfirstlane(p->tail_mask);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        r.mask[k] = __builtin_amdgcn_readfirstlane(p->mask[k]);
        r.blk_end[k] = __builtin_amdgcn_readfirstlane(p->blk_end[k]);
        r.in_base[k] = __builtin_amdgcn_readfirstlane(p->in_base[k]);
    }
    r.last_end = 0;
    r.tail_base = __builtin_amdgcn_readfirstlane(p->in_base[0]);
#pragma unroll
    for (int k = 1; k <= 4; k++) {
        if (r.nseg == k) {
            r.last_end = r.blk_end[k - 1];
            r.tail_base = __builtin_amdgcn_readfirstlane(p->in_base[k]);
        }
    }
    return r;
}

template <int KIND>
__device__ __forceinline__ uint32_t addr4(const int32_t *rowoff, const ProfR *__restrict__ pp, int t, int (&o)[4]) {
    const ProfR &P = *pp;
    const int p = 4 * t;
    uint32_t keep = 0;
    int idx[4] = {0, 0, 0, 0};
    if (P.nseg == 0) {
#pragma unroll
        for (int e = 0; e < 4; e++) idx[e] = p + e;
        keep = 0xF;
    } else {
        const int blk = p >> 7;
        uint32_t m = 0;
        int base = 0, b = 0;
        if (blk < P.last_end) {
            // segment of this block: selects over the (wave-uniform) profile words,
            // no per-lane indexing
            int bs = 0, ib = P.in_base[0];
            m = P.mask[0];
#pragma unroll
            for (int k = 1; k < 4; k++) {
                if (k < P.nseg && blk >= P.blk_end[k - 1]) { bs = P.blk_end[k - 1]; ib = P.in_base[k]; m = P.mask[k]; }
            }
            const int bis = blk - bs;
            const int n1 = __popc(m);
            const int oo = p & 127;
            b = oo & 31;
            base = ib + bis * 4 * n1 + (oo >> 5) * n1;
        } else {
            b = p - 128 * P.last_end;
            m = b < 24 ? P.tail_mask : 0u;
            base = P.tail_base;
            if (b >= 24) b = 0;
        }
        const uint32_t k4 = (m >> b) & 0xFu;
        int i = base + __popc(m & ((1u << b) - 1u));
#pragma unroll
        for (int e = 0; e < 4; e++) {
            idx[e] = i;
            i += (k4 >> e) & 1;
        }
        keep = k4;
    }
#pragma unroll
    for (int e = 0; e < 4; e++) {
        int off = idx[e];
        if constexpr (KIND == SRC_MSC) {
            const int ro = rowoff[idx[e] & 15];
            if (ro < 0) keep &= ~(1u << e);          // delay line still empty: zero
            off = ro + idx[e];
        }
        o[e] = ((keep >> e) & 1u) ? off : 0;
    }
    return keep;
}

__device__ __forceinline__ int parity(int v) { return __popc(v) & 1; }

template <int RHO>
struct LaneMask {            // lanes whose bit (5-RHO) is set = lanes holding an upper (msb=1) state
    static constexpr uint64_t v = RHO == 0 ? 0xFFFFFFFF00000000ull : RHO == 1 ? 0xFFFF0000FFFF0000ull
                                : RHO == 2 ? 0xFF00FF00FF00FF00ull : RHO == 3 ? 0xF0F0F0F0F0F0F0F0ull
                                : RHO == 4 ? 0xCCCCCCCCCCCCCCCCull : 0xAAAAAAAAAAAAAAAAull;
};

// Row stride of the branch-metric table: odd, so the 8 rows that one ACS step
// reads (8 distinct words, broadcast to 64 lanes) sit in 8 different LDS banks.
constexpr int BMS = VCH + 1;

// branch metrics of one step for the 8 (b0,b1,b2) output patterns
// (viterbi.cpp:159-164: metric = sum_j sym_j ^ B_j with b3 = b0)
__device__ __forceinline__ void put_bm(uint32_t *bm, const int16_t (&s)[4], uint32_t keep, int lane) {
    if (lane < VCH) {
        int y[4];
#pragma unroll
        for (int e = 0; e < 4; e++) y[e] = min(max(((keep >> e) & 1u ? (int)s[e] : 0) + 127, 0), 255);
        // y ^ 255 = 255 - y on [0, 255]: 4 partial sums instead of 8 x 4 xors
        const int a[2] = {y[0] + y[3], 510 - (y[0] + y[3])};
        const int bc[4] = {y[1] + y[2], 255 - y[1] + y[2], 255 + y[1] - y[2], 510 - (y[1] + y[2])};
#pragma unroll
        for (int q = 0; q < 8; q++) bm[q * BMS + lane] = (uint32_t)(a[q & 1] + bc[q >> 1]);
    }
}

// ACS over one tile of nst (<= VCH) trellis steps.  1020 - bm[q] = bm[q ^ 7].
// Returns the tile's decision word of step `lane` (lanes < nst).
template <bool FULL>
__device__ __forceinline__ uint64_t acs_tile(const uint32_t *bm, const uint32_t (&off)[6], const uint32_t (&offc)[6],
                                             uint32_t &x, int lane, int nst) {
    uint32_t dlo = 0, dhi = 0;
    sfor<0, VCH / 6>([&](auto gc) {
        sfor<0, 6>([&](auto rc) {
            constexpr int rho = decltype(rc)::value;
            constexpr int j = decltype(gc)::value * 6 + rho;
            if (FULL || j < nst) {
                const uint32_t a = x + bm[off[rho] + j];
                const uint32_t b = xchg<(32 >> rho)>(x, lane) + bm[offc[rho] + j];
                const uint64_t G = __ballot(a > b), Lt = __ballot(b > a);
                constexpr uint64_t M = LaneMask<rho>::v;
                const uint64_t D = (G & ~M) | (Lt & M);
                dlo = (uint32_t)llvm_amdgcn_writelane((int)(uint32_t)D, j, (int)dlo);
                dhi = (uint32_t)llvm_amdgcn_writelane((int)(uint32_t)(D >> 32), j, (int)dhi);
                x = min(a, b);
            }
        });
    });
    return ((uint64_t)dhi << 32) | dlo;
}

template <int KIND>
__global__ __launch_bounds__(64) void k_acs(VitJob J) {
    __shared__ uint32_t bm[8 * BMS];
    __shared__ int32_t rowoff[16];
    const int lane = threadIdx.x;
    const Src c = src_of<KIND>(J, xcd_order(blockIdx.x, gridDim.x), rowoff, lane);
    if (!c.valid) return;
    // the profile is wave-uniform: scalar loads, kept out of the vector memory queue
    const ProfR prof = prof_regs(J.prof + c.prof);       // in registers for the whole codeword
    const ProfR *pp = &prof;
    const int steps = prof.nbits + 6;
    uint32_t off[6], offc[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        const int i = rotl6(lane, r) & 31;               // butterfly of the state this lane holds
        const int q = parity((2 * i) & 0155) | (parity((2 * i) & 0117) << 1) | (parity((2 * i) & 0123) << 2);
        off[r] = (uint32_t)(q * BMS);
        offc[r] = (uint32_t)((q ^ 7) * BMS);
    }
    uint32_t x = lane == 0 ? 0u : 63u;                   // viterbi.cpp:360-371
    uint64_t *dec = J.dec + (int64_t)c.row * J.dec_stride;
    // inputs of the next tile are loaded while the current one runs its ACS
    int16_t s[4];
    uint32_t keep;
    auto fetch = [&](int t) {
        int o[4];
        keep = 0;
        if (lane < VCH && t < steps) keep = addr4<KIND>(rowoff, pp, t, o);
        else o[0] = o[1] = o[2] = o[3] = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) s[e] = c.base[o[e]];
    };
    // A tile's decisions are stored one tile late, just BEFORE the next prefetch:
    // vmcnt counts stores too, so the wait for the prefetched inputs then never
    // has to wait for a store issued after them.
    fetch(lane);
    uint64_t dprev = 0;
    int tprev = -1;
    int t0 = 0;
    for (; t0 + VCH <= steps; t0 += VCH) {
        put_bm(bm, s, keep, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (tprev >= 0 && lane < VCH) dec[tprev + lane] = dprev;
        fetch(t0 + VCH + lane);
        dprev = acs_tile<true>(bm, off, offc, x, lane, VCH);
        tprev = t0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (tprev >= 0 && lane < VCH) dec[tprev + lane] = dprev;
    if (t0 < steps) {
        put_bm(bm, s, keep, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t d = acs_tile<false>(bm, off, offc, x, lane, steps - t0);
        if (lane < steps - t0) dec[t0 + lane] = d;
    }
}

// Chainback (viterbi.cpp:333-357) from state 0, one lane per codeword.  The
// decision words of a lane are contiguous; TBC-step chunks stream through a
// 3-deep register ring (two chunks in flight while one is walked), so the
// dependent bit walk does not wait on memory.
template <bool CHECK>
__device__ __forceinline__ void tb_chunk(const uint4 (&c)[TBC / 2], int ch, int steps, int N, int &lr, int &rho,
                                         bool act, uint8_t *out, const VitJob &J) {
    uint32_t w = 0;
#pragma unroll
    for (int k = TBC - 1; k >= 0; k--) {
        const int t = ch * TBC + k;
        const uint32_t Dlo = (k & 1) ? c[k >> 1].z : c[k >> 1].x;
        const uint32_t Dhi = (k & 1) ? c[k >> 1].w : c[k >> 1].y;
        const int p = 5 - rho;
        const int u = (lr >> p) & 1;                                   // decoded bit of step t
        const uint32_t Dw = (lr & 32) ? Dhi : Dlo;
        const int d = (int)((Dw >> (lr & 31)) & 1u);                   // predecessor's msb
        const int nl = (lr & ~(1 << p)) | (d << p);
        if (!CHECK || t < steps) {
            lr = nl;
            w |= (uint32_t)u << k;
        }
        rho = rho == 0 ? 5 : rho - 1;
    }
    const int t0 = ch * TBC;
    if (act && t0 < N) {
        if (J.prbs) w ^= J.prbs_words[t0 >> 5];
        if (t0 + 32 <= N) {
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const uint32_t nib = (w >> (4 * e)) & 0xFu;
                *(uint32_t *)(out + t0 + 4 * e) = (nib * 0x00204081u) & 0x01010101u;
            }
        } else {
            for (int i = 0; t0 + i < N; i++) out[t0 + i] = (uint8_t)((w >> i) & 1u);
        }
    }
}

template <int KIND>
__global__ __launch_bounds__(64) void k_traceback(VitJob J) {
    static_assert(TBC == 32, "one 32-bit output word per chunk");
    const int lane = threadIdx.x, cw = blockIdx.x * 64 + lane;
    bool act = cw < J.n_cw;
    int N = 0, prof = 0;
    if (act) {
        // validity and profile by output row (inverse of src_of's mapping)
        if constexpr (KIND == SRC_MSC) {
            const int sub = cw % J.nsub;
            const int cl = (cw / J.nsub) % J.ncif;
            prof = sub;
            act = J.cif0 + cl >= 16;
        } else if constexpr (KIND == SRC_FRAG) {
            prof = J.cw_prof ? J.cw_prof[cw] : 0;
        }
        if (J.valid && !J.valid[cw]) act = false;
        if (act) N = J.prof[prof].nbits;
    }
    int tmax = act ? N + 6 : 0;
    for (int o = 32; o > 0; o >>= 1) tmax = max(tmax, __shfl_xor(tmax, o));
    if (tmax == 0) return;
    // inactive lanes walk codeword row 0's decisions (in bounds) and store nothing
    const int steps = act ? N + 6 : tmax;
    int smin = steps;
    for (int o = 32; o > 0; o >>= 1) smin = min(smin, __shfl_xor(smin, o));
    const uint4 *dq = (const uint4 *)(J.dec + (act ? (int64_t)cw * J.dec_stride : 0));
    uint8_t *out = J.out + (act ? (int64_t)cw * J.out_stride : 0);
    const int nch = (tmax + TBC - 1) / TBC;
    auto load = [&](uint4 (&c)[TBC / 2], int ch) {
        const bool ld = ch >= 0;
        const uint4 *q = dq + (ld ? ch : 0) * (TBC / 2);
#pragma unroll
        for (int k = 0; k < TBC / 2; k++) c[k] = q[k];
    };
    auto walk = [&](const uint4 (&c)[TBC / 2], int ch, int &lr, int &rho) {
        if ((ch + 1) * TBC <= smin) tb_chunk<false>(c, ch, steps, N, lr, rho, act, out, J);
        else tb_chunk<true>(c, ch, steps, N, lr, rho, act, out, J);
    };
    int lr = 0;                                          // lane index holding the traced state
    int rho = (nch * TBC - 1) % 6;                       // t mod 6 of the step being walked
    uint4 A[TBC / 2], B[TBC / 2], C[TBC / 2];
    load(A, nch - 1);
    load(B, nch - 2);
    for (int ch = nch - 1; ch >= 0; ch -= 3) {
        load(C, ch - 2);
        walk(A, ch, lr, rho);
        if (ch < 1) break;
        load(A, ch - 3);
        walk(B, ch - 1, lr, rho);
        if (ch < 2) break;
        load(B, ch - 4);
        walk(C, ch - 2, lr, rho);
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

template <template <int> class K>
static hipError_t launch_kind(hipStream_t st, const VitJob &job, dim3 grid) {
    switch (job.kind) {
    case SRC_MOTHER: hipLaunchKernelGGL(K<SRC_MOTHER>::fn(), grid, dim3(64), 0, st, job); break;
    case SRC_FRAG:   hipLaunchKernelGGL(K<SRC_FRAG>::fn(), grid, dim3(64), 0, st, job); break;
    case SRC_FIC:    hipLaunchKernelGGL(K<SRC_FIC>::fn(), grid, dim3(64), 0, st, job); break;
    case SRC_MSC:    hipLaunchKernelGGL(K<SRC_MSC>::fn(), grid, dim3(64), 0, st, job); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
template <int KIND> struct AcsK { static auto fn() { return k_acs<KIND>; } };
template <int KIND> struct TbK { static auto fn() { return k_traceback<KIND>; } };

hipError_t launch_acs(hipStream_t st, const VitJob &job) {
    if (job.n_cw <= 0) return hipSuccess;
    return launch_kind<AcsK>(st, job, dim3(job.n_cw));
}
hipError_t launch_traceback(hipStream_t st, const VitJob &job) {
    if (job.n_cw <= 0) return hipSuccess;
    return launch_kind<TbK>(st, job, dim3((job.n_cw + 63) / 64));
}
hipError_t launch_viterbi(hipStream_t st, const VitJob &job) {
    hipError_t e = launch_acs(st, job);
    return e != hipSuccess ? e : launch_traceback(st, job);
}

hipError_t launch_fic_post(hipStream_t st, uint8_t *bits, uint8_t *ok, int n_fib) {
    if (n_fib <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fic_post, dim3((n_fib + 63) / 64), dim3(64), 0, st, bits, ok, n_fib);
    return hipGetLastError();
}

}  // namespace dab
