// k_viterbi.hip -- k=7 R=1/4 Viterbi decoder for gfx950 and its callers.
//
// Reference semantics (viterbi.cpp:225-242 + FULL_SPIRAL spiral-sse.c:30-698):
//   sym = clamp(soft + 127, 0, 255); branch metric sum_j sym_j ^ B_j, B in {0,255};
//   uint32 path metrics without renormalisation, start 63 / state0 = 0;
//   strict ">" picks the upper predecessor; full chainback from state 0.
//
// gfx950 design
//   k_acs       one wave64 per PAIR of codewords, one trellis state per lane, the two
//               codewords' path metrics packed in the 16-bit halves of one VGPR
//               (v_pk_add_u16 / v_pk_min_u16 do both).  Exactness of 16 bits: metric
//               spread across states is <= 6 * 1020 (every state is reachable from the
//               best one in 6 steps, branch metrics are in [0, 1020]), so subtracting a
//               common offset every 30 steps keeps every metric in [0, 43860] and every
//               comparison equal to the reference's uint32 one.
//               States are relabelled every step (lane L holds state rotl6(L, t mod 6)),
//               so a butterfly pairs lanes at xor distance 32,16,8,4,2,1.  Each lane
//               forms its two candidates as (metric of the LOWER lane of its pair) +
//               row A and (metric of the UPPER lane) + row B, the rows chosen per lane
//               so that the decision is "A > B" in every lane.  The broadcasts are DPP
//               (quad_perm, row_shr/shl with bank masks) or one permlane16/32_swap.
//               Both codewords' decisions come from one packed subtract (sign bits of
//               B - A) and shift into one VGPR (dec_in); every 30 steps they are
//               unpacked into one 30-bit word per codeword and stored: decisions never
//               leave the VGPRs as scalar masks.  Branch metrics for 60 steps are built
//               in LDS by the lanes at once (depuncturing + 16-CIF time de-interleave
//               fused into that gather), both codewords packed per word.
//   k_traceback one LANE per codeword, 64 chainbacks per wave in lock-step.  Decision
//               words of a 30-step chunk for the wave's 64 codewords are staged in LDS
//               (16 KB, register-prefetched 2 chunks ahead); each step reads the word of
//               the lane that held the traced state, two steps per LDS round trip.
//               Bits leave through 2-B stores with the energy-dispersal PRBS xor-ed in.
//
// Decision layout (dab_kernels.h dec_word_index): 64-row blocks, each block's chunks
// contiguous (a codeword's words then lie within 1.7 MB instead of one per 14 MB stride,
// which cost the ACS its TLB reach), word [lane] of (row, chunk): bit dpos(k) = decision
// of `lane` at trellis step 30*chunk + k (k < 30; dpos below).
#include "dab_device.h"
#include "dab_kernels.h"
#include <algorithm>

namespace dab {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_pk(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

__device__ __forceinline__ int rotl6(int x, int r) { return ((x << r) | (x >> (6 - r))) & 63; }

// XCD-aware block order (cdna_hip_programming.md T1): blocks b with equal b % 8
// share an XCD's L2; give each such group a contiguous range of codewords so the
// 16 CIFs that read the same ring rows (time de-interleave) decode on one L2.
__device__ __forceinline__ int xcd_order(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-codeword source, resolved once per wave.
struct Src {
    const int16_t *base;   // first input element (SRC_MSC: the stream's ring)
    __amdgpu_buffer_rsrc_t rs;   // buffer over the readable elements: 32-bit offsets, and
                                 // reads past its end (erasures, empty delay line) return 0
    int prof;              // profile index
    int row;               // output / decision row of this codeword
    bool valid;
};

// SRC_MSC logical order (stream, subchannel, CIF) -- consecutive CIFs of one
// subchannel share 15 of their 16 source rows and their profile; output rows stay
// ((stream * ncif) + cif) * nsub + sub.
template <int KIND, bool B8 = false>
__device__ __forceinline__ Src src_of(const VitJob &J, int logical, int32_t *rowoff, int lane) {
    static_assert(!B8 || KIND == SRC_FIC || KIND == SRC_MSC, "RING8 bytes: the pipeline's ring only");
    constexpr int ESZ = B8 ? 1 : 2;                    // bytes per soft value
    Src c;
    c.prof = 0;
    c.valid = logical < J.n_cw;
    if (!c.valid) logical = 0;
    c.row = logical;
    if constexpr (KIND == SRC_MOTHER) {
        c.base = J.src + (int64_t)logical * J.src_stride;
    } else if constexpr (KIND == SRC_FRAG) {
        c.base = J.src + (int64_t)logical * J.src_stride;
        c.prof = J.cw_prof ? J.cw_prof[logical] : 0;
    } else if constexpr (KIND == SRC_FIC) {
        const int32_t slot = J.slots[logical >> 2];    // < 0: frame not committed
        c.valid = c.valid && slot >= 0;
        c.base = (const int16_t *)((const char *)J.src +
                                   ESZ * ((int64_t)(slot < 0 ? 0 : slot) * FRAME_SOFT + (logical & 3) * 2304));
    } else {
        const int cl = logical % J.ncif;
        const int rest = logical / J.ncif;
        const int sub = rest % J.nsub;
        const int stream = rest / J.nsub;
        c.row = (stream * J.ncif + cl) * J.nsub + sub;
        c.prof = sub;
        const int64_t cif = J.cif0s[stream] + cl;
        // CIFs the stream delivered in this batch; dab-concurrent.cpp:172-175 warm-up
        c.valid = c.valid && cl < J.ncifs[stream] && cif >= 16;
        c.base = (const int16_t *)((const char *)J.src + ESZ * (int64_t)stream * J.ring * FRAME_SOFT);
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
        wave_sync();
    }
    if (c.valid && J.valid && !J.valid[c.row]) c.valid = false;
    int64_t nrec = 0;                                  // readable bytes from base
    if constexpr (KIND != SRC_MSC) {
        if (c.valid) {
            const Profile &P = J.prof[c.prof];
            const int64_t need = P.nseg ? P.frag : 4 * (int64_t)(P.nbits + 6);
            const int64_t o = ((const char *)c.base - (const char *)J.src) / ESZ;   // in soft values
            if (o < 0 || o + need > J.src_len) {      // never read outside the buffer
                if (lane == 0) atomicOr(J.err, KERR_VITERBI);
                c.valid = false;
            }
            nrec = ESZ * need;
        }
    } else {
        nrec = ESZ * (int64_t)J.ring * FRAME_SOFT;      // the stream's ring (rowoff checked above)
    }
    // wave-uniform by construction; readfirstlane keeps the descriptor in SGPRs
    const uint64_t b = (uint64_t)(uintptr_t)c.base;
    // (readfirstlane returns int: widen through uint32_t, no sign extension)
    const uint64_t bu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
    const int nu = __builtin_amdgcn_readfirstlane(c.valid ? (int)nrec : 0);
    c.rs = __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)bu, (short)0, nu, 0x00020000);
    return c;
}

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

// Input indices (relative to the codeword's punctured fragment) of the 4 mother-code
// soft values of trellis step t (positions 4t..4t+3) with the depuncturing of
// deconvolve.cpp:172-237 / fic-handler.cpp:241-270.  keep bit e = 0 marks an erasure
// ("a real do not know", fic-handler.cpp:259, or the zero tail of deconvolve.cpp:182).
__device__ __forceinline__ uint32_t idx4(const ProfR &P, int t, int (&idx)[4]) {
    const int p = 4 * t;
    if (P.nseg == 0) {
#pragma unroll
        for (int e = 0; e < 4; e++) idx[e] = p + e;
        return 0xF;
    }
    const int blk = p >> 7;
    uint32_t m = 0;
    int base = 0, b = 0;
    if (blk < P.last_end) {
        // segment of this block: selects over the (wave-uniform) profile words
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
    return k4;
}

// idx4 when every lane of the tile lies in one depuncturing segment (the common case:
// segments span hundreds of steps): the segment's block start, input base and PI mask
// arrive wave-uniform instead of through per-lane selects
__device__ __forceinline__ uint32_t idx4_seg(int t, int bs, int ib, uint32_t m, int (&idx)[4]) {
    const int p = 4 * t, blk = p >> 7;
    const int n1 = __popc(m), oo = p & 127, b = oo & 31;
    const int base = ib + (blk - bs) * 4 * n1 + (oo >> 5) * n1;
    const uint32_t k4 = (m >> b) & 0xFu;
    int i = base + __popc(m & ((1u << b) - 1u));
#pragma unroll
    for (int e = 0; e < 4; e++) {
        idx[e] = i;
        i += (k4 >> e) & 1;
    }
    return k4;
}
// the 4 soft values of one step of one codeword into half H of s[] (erasures and
// steps past the codeword's end read as 0)
template <int KIND, int H>
__device__ __forceinline__ void load4(const Src &c, const int32_t *rowoff, const int (&idx)[4], uint32_t keep,
                                      u16x2 (&s)[4]) {
#pragma unroll
    for (int e = 0; e < 4; e++) {
        int off = idx[e];
        bool k = (keep >> e) & 1u;
        if constexpr (KIND == SRC_MSC) {
            const int ro = rowoff[idx[e] & 15];
            k = k && ro >= 0;                         // delay line still empty: zero
            off = ro + idx[e];
        }
        // erasures read past the buffer's end: the hardware returns 0
        s[e][H] = __builtin_amdgcn_raw_buffer_load_b16(c.rs, k ? 2 * off : 0x7FFFFFF0, 0, 0);
    }
}

__device__ __forceinline__ int parity(int v) { return __popc(v) & 1; }

// LDS branch-metric table for a tile of VT steps: 8 rows q (the (b0,b1,b2) output
// pattern); step j of row q holds the pair {bm[q], bm[q^7]} as two packed words
// (codeword A in the low, B in the high 16 bits).  The row stride puts the 8 rows one
// ds_read_b64 touches in 8 distinct bank pairs.
// branch-metric pairs are read ACS_PF steps ahead of their use (round 3: 3 steps ahead
// took k_acs2 1.31 -> 1.29 ms in the pipeline, profiles/r03_acs_pf_ab.txt; 2 and 4 no better)
#ifndef ACS_PF
#define ACS_PF 3
#endif
constexpr int WS = DEC_WORD_STEPS;         // 30 decisions per word: a multiple of 6, so
                                           // every word starts at relabelling phase 0
constexpr int VT = 2 * WS;                 // steps per branch-metric tile (lanes 0..59 build one each)
constexpr int BRS = 2 * VT + 2;            // 122: rows 0..7 start at banks 0,58,52,46,40,34,28,22
static_assert(WS % 6 == 0 && (BRS & 3) == 2, "bank-pair stride");
constexpr int RENORM = WS;                 // steps between metric renormalisations (see header)
constexpr uint32_t SPREAD = 6 * 1020;

// branch metrics of one step for the 8 (b0,b1,b2) output patterns, both codewords
// (viterbi.cpp:159-164: metric = sum_j sym_j ^ B_j with b3 = b0; y ^ 255 = 255 - y).
// Every partial sum stays inside its 16-bit half, so plain 32-bit adds work on pairs.
template <bool B8 = false>
__device__ __forceinline__ void put_bm(uint32_t *bm, int j, const u16x2 (&s)[4]) {
    typedef short i16x2 __attribute__((ext_vector_type(2)));
    uint32_t y[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        if constexpr (B8) {                 // RING8 bytes: already v + 127 in 0..254
            y[e] = as_u32(s[e]);
            continue;
        }
        // int16_t temp = input[i] + 127, clamped to 0..255 (viterbi.cpp:230-233): the sum
        // wraps in 16 bits like the reference's int16_t, so inputs above 32640 become 0
        const i16x2 t = __builtin_bit_cast(i16x2, as_u32(s[e] + (u16x2){127, 127}));
        const i16x2 v = __builtin_elementwise_min(__builtin_elementwise_max(t, (i16x2){0, 0}), (i16x2){255, 255});
        y[e] = __builtin_bit_cast(uint32_t, v);
    }
    const uint32_t a0 = y[0] + y[3], a1 = 0x01FE01FEu - a0;
    const uint32_t b0 = y[1] + y[2], b1 = 0x00FF00FFu - y[1] + y[2], b2 = 0x00FF00FFu + y[1] - y[2],
                   b3 = 0x01FE01FEu - b0;
    const uint32_t w[4] = {a0 + b0, a1 + b0, a0 + b1, a1 + b1};           // q = 0..3
    const uint32_t wc[4] = {a1 + b3, a0 + b3, a1 + b2, a0 + b2};          // q ^ 7 = 7..4
    // q = 0..3: {bm[q], bm[7-q]};  q = 4..7: {bm[q], bm[7-q]} = {wc[7-q], w[7-q]}
#pragma unroll
    for (int q = 0; q < 4; q++) *(uint2 *)&bm[q * BRS + 2 * j] = make_uint2(w[q], wc[q]);
#pragma unroll
    for (int q = 4; q < 8; q++) *(uint2 *)&bm[q * BRS + 2 * j] = make_uint2(wc[7 - q], w[7 - q]);
}

// Candidates of one step: A = P + ta, B = Q + tb with (P, Q) = metric of the lower /
// upper lane of this lane's butterfly pair (xor M).  The packed halves never carry
// (<= 42840 + 1020 < 2^16), so 32-bit adds serve both codewords and the lane moves
// fold into them as DPP operands: quad_perm for M = 1, 2; for M = 4, 8 the own-lane
// sum first, then a bank-masked DPP add over the lanes that take their partner's
// metric; M = 32 goes through one permlane swap (a copy, a hazard wait and a
// quarter-rate swap), M = 16 reads P and Q through the LDS crossbar (two ds_swizzle
// within 32 lanes), which leaves that step's VALU to the two adds.  Measured (round 2,
// profiles/r02_acs_core.txt, r02_acs_ab.txt): the crossbar for M = 32 is 8 % faster in the
// ACS alone but slower in the kernel, whose tile loader also lives on the LDS; for M = 16
// alone 1.5 % faster; for M = 4 / 8 no gain.
// DPP hazard: a DPP source written by the previous VALU instruction needs two wait
// states -- only the first quad_perm add follows the metric update directly (s_nop 1);
// the bank-masked adds come after the two plain adds that also read x.
#define DPP_ADD(ctl) "v_add_u32_dpp %0, %1, %2 " ctl
#define DPP_ADD_NOP(ctl) "s_nop 1\n\tv_add_u32_dpp %0, %1, %2 " ctl
template <int M>
__device__ __forceinline__ void cand(uint32_t x, uint32_t ta, uint32_t tb, uint32_t &A, uint32_t &B) {
    if constexpr (M == 1) {
        asm(DPP_ADD_NOP("quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf") : "=&v"(A) : "v"(x), "v"(ta));
        asm(DPP_ADD("quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf") : "=&v"(B) : "v"(x), "v"(tb));
    } else if constexpr (M == 2) {
        asm(DPP_ADD_NOP("quad_perm:[0,1,0,1] row_mask:0xf bank_mask:0xf") : "=&v"(A) : "v"(x), "v"(ta));
        asm(DPP_ADD("quad_perm:[2,3,2,3] row_mask:0xf bank_mask:0xf") : "=&v"(B) : "v"(x), "v"(tb));
    } else if constexpr (M == 16) {
        // swizzle bit mode: lane' = (lane & and) | or within 32 lanes (a permlane16 swap
        // instead measured no faster, round 3)
        A = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x0F) + ta;              // lane & ~16
        B = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (0x10 << 5)) + tb; // lane | 16
    } else if constexpr (M == 4) {
        // upper lanes (banks 1,3 of each row) take lane-4 as P; lower lanes (banks 0,2) lane+4 as Q
        // (one asm block: the two plain adds are the wait states before the DPP reads x)
        asm("v_add_u32 %0, %2, %3\n\tv_add_u32 %1, %2, %4\n\t"
            "v_add_u32_dpp %0, %2, %3 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
            "v_add_u32_dpp %1, %2, %4 row_shl:4 row_mask:0xf bank_mask:0x5"
            : "=&v"(A), "=&v"(B) : "v"(x), "v"(ta), "v"(tb));
    } else if constexpr (M == 8) {
        asm("v_add_u32 %0, %2, %3\n\tv_add_u32 %1, %2, %4\n\t"
            "v_add_u32_dpp %0, %2, %3 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
            "v_add_u32_dpp %1, %2, %4 row_shl:8 row_mask:0xf bank_mask:0x3"
            : "=&v"(A), "=&v"(B) : "v"(x), "v"(ta), "v"(tb));
    } else {
        static_assert(M == 32, "xor distance");
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        A = r[0] + ta;
        B = r[1] + tb;
    }
}
#undef DPP_ADD
#undef DPP_ADD_NOP

// w with the bits of e under mask m (one v_bfi)
__device__ __forceinline__ uint32_t bits_put(uint32_t m, uint32_t w, uint32_t e) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(e), "v"(w));
    return r;
}
// Decision bits in a stored word.  v_bfi and v_perm issue at half rate on gfx950
// (profiles/r02_valu_rate.txt): per pair of steps (2p, 2p+1) the v_perm selectors 8..11
// (a byte of copies of bit 15 / 31 of either source) turn the four decisions into four
// 0x00 / 0xFF bytes at once, and one v_bfi with the mask 0x01010101 << (p & 7) drops them
// into bit p & 7 of a collector's bytes -- 1 instruction per step (round 2 measured a
// shift-in per step and a v_perm + shift + v_bfi per pair slower, r02_acs_ab.txt).
// Collector a takes pairs 0..7, b pairs 8..14; the stored word of codeword 0 is
// {a.b0, a.b2, b.b0, b.b2}, of codeword 1 {a.b1, a.b3, b.b1, b.b3}.
// dpos(k) = bit of trellis step k (k < 30) of a chunk in its word.
__host__ __device__ constexpr int dpos(int k) { return k < 16 ? 8 * (k & 1) + (k >> 1) : 8 + 8 * (k & 1) + (k >> 1); }

// subtract a common offset from all states of each codeword (see header)
__device__ __forceinline__ uint32_t renorm(uint32_t x) {
    const uint32_t x0 = __builtin_amdgcn_readfirstlane(x);
    const uint32_t lo = x0 & 0xFFFFu, hi = x0 >> 16;
    const uint32_t c = (lo > SPREAD ? lo - SPREAD : 0u) | ((hi > SPREAD ? hi - SPREAD : 0u) << 16);
    return as_u32(as_pk(x) - as_pk(c));
}

// ACS over one decision word (WS trellis steps, or nst < WS for the last one) for NP
// codeword pairs (independent chains, interleaved step by step).  bm: this word's
// half of the tile table.  The words are stored at chunk `ch`; rb[k]: word offset of
// codeword k's chunk 0 in dec (wave-uniform; < 0: not stored).  One copy of this code
// serves every word (small hot loop: the instruction cache holds it).
// Decisions: d = B - A per 16-bit half has its sign bit set iff A > B (|A - B| <=
// spread + 1020 < 2^15), so one packed subtract yields both codewords' decisions;
// they shift down their half of w (dec_in), 15 steps per half-word, and are
// unpacked to one word per codeword (step k at bit k) at the end of the word.
// rp[r]: this lane's branch-metric row of relabelling phase r in the tile table (set once
// per kernel); U: the word's half of the tile -- each step's read is one ds_read_b64 at
// an immediate offset, no address arithmetic per word
template <int NP, bool FULL, int U>
__device__ __forceinline__ void acs_word_cw(const uint32_t *const (&rp)[6], uint32_t (&x)[NP], int nst,
                                            uint32_t (&cw)[2 * NP]) {
    static_assert(WS == 30, "two collectors of 8 and 7 step pairs per decision word");
    uint32_t w[NP], w0[NP], dp[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) w[p] = dp[p] = 0;
    // branch-metric pairs read ACS_PF steps ahead of their use (the LDS latency off the
    // metric chain)
    constexpr int PF = ACS_PF;
    uint2 tq[NP][PF + 1];
    auto ldt = [&](int jj, int p) { return *(const uint2 *)(rp[jj % 6] + U * 2 * WS + p * 8 * BRS + 2 * jj); };
    sfor<0, PF>([&](auto jc) {
        constexpr int jj = decltype(jc)::value;
#pragma unroll
        for (int p = 0; p < NP; p++) tq[p][jj % (PF + 1)] = ldt(jj, p);
    });
    sfor<0, WS>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int rho = j % 6;
        uint32_t d[NP];
        if constexpr (PF > 0 && j + PF < WS) {
#pragma unroll
            for (int p = 0; p < NP; p++) tq[p][(j + PF) % (PF + 1)] = ldt(j + PF, p);
        }
        if (FULL || j < nst) {
            sfor<0, NP>([&](auto pc) {
                constexpr int p = decltype(pc)::value;
                const uint2 t = PF > 0 ? tq[p][j % (PF + 1)] : ldt(j, p);
                uint32_t A, B;
                cand<(32 >> rho)>(x[p], t.x, t.y, A, B);
                d[p] = as_u32(as_pk(B) - as_pk(A));
                x[p] = as_u32(__builtin_elementwise_min(as_pk(A), as_pk(B)));
            });
        } else {
#pragma unroll
            for (int p = 0; p < NP; p++) d[p] = 0;        // past the codeword: keep the bit positions
        }
#pragma unroll
        for (int p = 0; p < NP; p++) {
            if constexpr ((j & 1) == 0) dp[p] = d[p];
            else w[p] = bits_put(0x01010101u << ((j >> 1) & 7), w[p], __builtin_amdgcn_perm(d[p], dp[p], 0x0B0A0908u));
        }
        if constexpr (j == 15) {
#pragma unroll
            for (int p = 0; p < NP; p++) {
                w0[p] = w[p];
                w[p] = 0;
            }
        }
    });
#pragma unroll
    for (int p = 0; p < NP; p++) {
        cw[2 * p] = __builtin_amdgcn_perm(w[p], w0[p], 0x06040200u);
        cw[2 * p + 1] = __builtin_amdgcn_perm(w[p], w0[p], 0x07050301u);
    }
#pragma unroll
    for (int p = 0; p < NP; p++) x[p] = renorm(x[p]);
}
// ... and its words stored at chunk offset o (rb[k] < 0: codeword k not stored)
// (through a buffer descriptor: the word's 32-bit offset is wave-uniform, so the store
// carries one lane offset register instead of a 64-bit address per lane)
template <int NP, bool FULL, int U>
__device__ __forceinline__ void acs_word(const uint32_t *const (&rp)[6], uint32_t (&x)[NP], int nst,
                                         __amdgpu_buffer_rsrc_t drs, const int64_t (&rb)[2 * NP], int64_t o, int lane) {
    uint32_t cw[2 * NP];
    acs_word_cw<NP, FULL, U>(rp, x, nst, cw);
#pragma unroll
    for (int k = 0; k < 2 * NP; k++)
        if (rb[k] >= 0)
            __builtin_amdgcn_raw_buffer_store_b32(cw[k], drs, 4 * lane, (int)(4 * (rb[k] + o)), 0);
}
// the two words of a tile [t0, t0 + VT)
template <int NP>
__device__ __forceinline__ void acs_tile(const uint32_t *const (&rp)[6], uint32_t (&x)[NP], int t0, int steps,
                                         __amdgpu_buffer_rsrc_t drs, const int64_t (&rb)[2 * NP], int lane) {
    const int64_t cstride = 64 * 64;                    // words per chunk of a 64-row block
    sfor<0, 2>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const int tw = t0 + u * WS;
        if (tw < steps) {
            const int64_t o = (int64_t)(tw / WS) * cstride;
            if (tw + WS <= steps) acs_word<NP, true, u>(rp, x, WS, drs, rb, o, lane);
            else acs_word<NP, false, u>(rp, x, steps - tw, drs, rb, o, lane);
        }
    });
}

// NP pairs of codewords per wave: codewords 2*NP*w .. 2*NP*w + 2*NP - 1 (logical order).
// LDS (kernel-owned, so two jobs in one launch share it): bm[NP*8*BRS], rowoff[2*NP][16]
template <int NP> struct AcsLds {
    uint32_t bm[NP * 8 * BRS];
    int32_t rowoff[2 * NP][16];
    int2 ro2[NP][16];               // SRC_MSC pair: both codewords' row byte offsets per idx & 15
};
constexpr int32_t RO_EMPTY = 0x40000000;   // byte offset past any ring: the buffer load returns 0
// Punctured inputs before mother-code position 4t (t wave-uniform: scalar arithmetic);
// the same depuncturing rule as idx4 (deconvolve.cpp:172-237, fic-handler.cpp:241-270)
__device__ __forceinline__ int in_index(const ProfR &P, int t) {
    const int p = 4 * t, blk = p >> 7;
    if (blk < P.last_end) {
        int bs = 0, ib = P.in_base[0];
        uint32_t m = P.mask[0];
#pragma unroll
        for (int k = 1; k < 4; k++) {
            if (k < P.nseg && blk >= P.blk_end[k - 1]) { bs = P.blk_end[k - 1]; ib = P.in_base[k]; m = P.mask[k]; }
        }
        const int n1 = __popc(m);
        return ib + (blk - bs) * 4 * n1 + ((p & 127) >> 5) * n1 + __popc(m & ((1u << (p & 31)) - 1u));
    }
    const int b = p - 128 * P.last_end;
    return P.tail_base + __popc(b >= 24 ? P.tail_mask : P.tail_mask & ((1u << b) - 1u));
}

// Input-major tile loader (SRC_MSC / SRC_FIC pairs of one profile).  The tile's steps
// [t0, t0 + VT) consume the punctured inputs [I0, I1); lane l loads inputs I0 + l + 64k.
// All of a lane's inputs share the residue (I0 + l) & 15, i.e. one time-interleaver
// delay-line row per lane and tile, so a soft value costs no address arithmetic (the
// 64k step is the load's constant offset).  The profile's inverse table (host-built,
// J.inv + Profile::inv_off: input -> mother-code position) scatters each value pair
// into an LDS staging table of the tile's 4 * VT mother positions (zero = erasure,
// deconvolve.cpp:182 / fic-handler.cpp:259), which the branch-metric builder then reads
// one step per lane.  The step-major loader below spends ~2.4 VALU instructions per
// trellis step on the depuncturing and delay-line selects of every value; this one 0.9.
constexpr int IN_K = 4;                    // <= 4 * VT inputs per tile: 4 rounds of 64 lanes
template <int KIND, bool B8>
__device__ __forceinline__ void acs_tiles_in(const VitJob &J, const Src (&c)[2], int prof, const ProfR &P, int steps,
                                             const uint32_t (&row)[6], uint32_t (&x)[1],
                                             __amdgpu_buffer_rsrc_t drs, const int64_t (&rb)[2], uint32_t *bm,
                                             const int2 *ro2, int lane) {
    const int frag = __builtin_amdgcn_readfirstlane(J.prof[prof].frag);
    const int ioff = __builtin_amdgcn_readfirstlane(J.prof[prof].inv_off);
    const __amdgpu_buffer_rsrc_t rinv =
        __builtin_amdgcn_make_buffer_rsrc((void *)(J.inv + ioff), (short)0, frag, 0x00020000);
    static_assert(4 * VT == VIT_TILE_POS, "inverse tables: positions within a tile");
    u16x2 vab[IN_K];                       // the pair's inputs, packed
    uint32_t vm[IN_K];                     // their mother-code positions
    int I0 = 0, I1 = 0;
    auto fetch = [&](int t0) {
        I0 = in_index(P, t0);
        I1 = in_index(P, min(t0 + VT, steps));
        const int i = I0 + lane;
        int2 ro;
        if constexpr (KIND == SRC_MSC) ro = ro2[i & 15];
        else ro = make_int2(c[0].valid ? 0 : RO_EMPTY, c[1].valid ? 0 : RO_EMPTY);
        constexpr int ESZ = B8 ? 1 : 2;
        const int oa = ro.x + ESZ * i, ob = ro.y + ESZ * i, oi = i;
#pragma unroll
        for (int k = 0; k < IN_K; k++) {
            if (64 * k < I1 - I0) {
                if constexpr (B8) {
                    // a refused or empty row (RO_EMPTY: the load is out of bounds and returns
                    // 0, which as a RING8 byte is soft value -127) reads the erasure byte 127,
                    // as the int16 form reads the erasure 0
                    const uint32_t a8 = __builtin_amdgcn_raw_buffer_load_b8(c[0].rs, oa, 64 * k, 0);
                    const uint32_t b8 = __builtin_amdgcn_raw_buffer_load_b8(c[1].rs, ob, 64 * k, 0);
                    vab[k][0] = ro.x == RO_EMPTY ? (uint16_t)RING8_BIAS : (uint16_t)a8;
                    vab[k][1] = ro.y == RO_EMPTY ? (uint16_t)RING8_BIAS : (uint16_t)b8;
                } else {
                    vab[k][0] = __builtin_amdgcn_raw_buffer_load_b16(c[0].rs, oa, 128 * k, 0);
                    vab[k][1] = __builtin_amdgcn_raw_buffer_load_b16(c[1].rs, ob, 128 * k, 0);
                }
                vm[k] = __builtin_amdgcn_raw_buffer_load_b8(rinv, oi, 64 * k, 0);
            }
        }
    };
    // the staging table (4 * VT words) aliases the bm rows: it is read before they are written
    auto put = [&](int t0) {
        // erasures (deconvolve.cpp:182 / fic-handler.cpp:259: soft value 0): 0, or 127 as RING8 bytes
        constexpr uint32_t E0 = B8 ? 0x007F007Fu : 0u;
        if (lane < VT) *(uint4 *)&bm[4 * lane] = make_uint4(E0, E0, E0, E0);
        wave_sync();
        const int n = I1 - I0;
#pragma unroll
        for (int k = 0; k < IN_K; k++) {
            if (64 * k < n && lane + 64 * k < n) bm[vm[k]] = as_u32(vab[k]);    // position in the tile
        }
        wave_sync();
        u16x2 sv[4];
        const uint4 q = *(const uint4 *)&bm[4 * (lane < VT ? lane : 0)];
        sv[0] = as_pk(q.x);
        sv[1] = as_pk(q.y);
        sv[2] = as_pk(q.z);
        sv[3] = as_pk(q.w);
        wave_sync();
        if (lane < VT) put_bm<B8>(bm, lane, sv);
    };
    const uint32_t *rp[6];
#pragma unroll
    for (int r = 0; r < 6; r++) rp[r] = bm + row[r];
    fetch(0);
    for (int t0 = 0; t0 < steps; t0 += VT) {
        put(t0);
        wave_sync();
        if (t0 + VT < steps) fetch(t0 + VT);
        acs_tile<1>(rp, x, t0, steps, drs, rb, lane);
        wave_sync();
    }
}

template <int KIND, int NP, bool B8 = false>
__device__ __forceinline__ void acs_body(const VitJob &J, int w, AcsLds<NP> &L) {
    uint32_t *bm = L.bm;
    int32_t (*rowoff)[16] = L.rowoff;
    const int lane = threadIdx.x;
    Src c[2 * NP];
    bool any = false;
#pragma unroll
    for (int k = 0; k < 2 * NP; k++) {
        c[k] = src_of<KIND, B8>(J, 2 * NP * w + k, rowoff[k], lane);
        any = any || c[k].valid;
    }
    if (!any) return;
    if constexpr (KIND == SRC_MSC) {
        // the pair's two delay-line row tables side by side, in bytes, an empty row (or
        // an invalid codeword's) as an offset past the buffer: one LDS read and no
        // compare per soft value pair in the tile loader
        if (lane < 16) {
#pragma unroll
            for (int p = 0; p < NP; p++) {
                const int32_t a = rowoff[2 * p][lane], b = rowoff[2 * p + 1][lane];
                constexpr int ESZ = B8 ? 1 : 2;
                L.ro2[p][lane] = make_int2(a >= 0 && c[2 * p].valid ? ESZ * a : RO_EMPTY,
                                           b >= 0 && c[2 * p + 1].valid ? ESZ * b : RO_EMPTY);
            }
        }
        wave_sync();
    }
    // profiles are wave-uniform: scalar loads, kept out of the vector memory queue
    const ProfR p0 = prof_regs(J.prof + c[0].prof);
    bool same = true;
    int stp[2 * NP], steps = 0;
#pragma unroll
    for (int k = 0; k < 2 * NP; k++) {
        same = same && c[k].prof == c[0].prof;
        // wave-uniform by construction; readfirstlane keeps the tile/word loops scalar
        // (a step count in a VGPR turns every loop exit into exec-mask juggling)
        stp[k] = __builtin_amdgcn_readfirstlane(c[k].valid ? J.prof[c[k].prof].nbits + 6 : 0);
        steps = max(steps, stp[k]);
    }
    same = __builtin_amdgcn_readfirstlane((int)same) != 0;
    // per-lane LDS row of each relabelling phase (see header): q = output pattern of
    // butterfly i = rotl6(lane, r) & 31; upper lanes of a pair swap the two rows
    uint32_t row[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
        const int i = rotl6(lane, r) & 31;
        const int q = parity((2 * i) & 0155) | (parity((2 * i) & 0117) << 1) | (parity((2 * i) & 0123) << 2);
        const bool upper = (lane >> (5 - r)) & 1;
        row[r] = (uint32_t)((upper ? q ^ 7 : q) * BRS);
    }
    uint32_t x[NP];
    int64_t rb[2 * NP];
#pragma unroll
    for (int p = 0; p < NP; p++) x[p] = lane == 0 ? 0u : 0x003F003Fu;   // viterbi.cpp:360-371
#pragma unroll
    for (int k = 0; k < 2 * NP; k++) {
        rb[k] = c[k].valid ? dec_word_index(c[k].row, J.dec_nch) : -1;
    }
    const int64_t cstride = 64 * 64;                    // words per chunk of a 64-row block
    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc((void *)J.dec, (short)0, -1, 0x00020000);
    if constexpr (KIND == SRC_MSC || KIND == SRC_FIC) {
        // a pair always shares its profile here: SRC_FIC has one, and an SRC_MSC pair is
        // two consecutive CIFs of one subchannel (ncif = 4F is even)
        static_assert(NP == 1, "input-major loader: one codeword pair per wave");
        acs_tiles_in<KIND, B8>(J, c, c[0].prof, p0, steps, row, x, drs, rb, bm, L.ro2[0], lane);
    } else {
    // step-major loader (SRC_MOTHER / SRC_FRAG: a pair may have two profiles)
    // inputs of the next tile are loaded while the current one runs its ACS;
    // lane < VT handles step t0 + lane
    u16x2 s[NP][4];                                      // packed {A, B} soft values, per pair
    // the depuncturing segments of profile 0 as plain scalars; the segment of a tile
    // is a sum of boundary flags
    // tb: first step of the tile (wave-uniform); t: this lane's step
    auto fetch = [&](int tb, int t) {
        int i0[4];
        uint32_t k0 = 0;
        // one depuncturing segment for the whole tile (wave-uniform, scalar): the
        // segment search of idx4 on the tile's first and last blocks
        const int blo = (4 * tb) >> 7, bhi = (4 * (tb + VT - 1) + 3) >> 7;
        int bs = 0, bs_hi = 0, ib = p0.in_base[0];
        uint32_t m = p0.mask[0];
#pragma unroll
        for (int k = 1; k < 4; k++) {
            if (k < p0.nseg && blo >= p0.blk_end[k - 1]) { bs = p0.blk_end[k - 1]; ib = p0.in_base[k]; m = p0.mask[k]; }
            if (k < p0.nseg && bhi >= p0.blk_end[k - 1]) bs_hi = p0.blk_end[k - 1];
        }
        const bool useg = p0.nseg > 0 && bhi < p0.last_end && bs == bs_hi;
        if (t < stp[0] || (same && t < steps)) {
            if (useg) {
                k0 = idx4_seg(t, bs, ib, m, i0);
            } else {
                k0 = idx4(p0, t, i0);
            }
        } else {
            i0[0] = i0[1] = i0[2] = i0[3] = 0;
        }
        if constexpr (KIND == SRC_MSC) {
            if (same) {
#pragma unroll
                for (int p = 0; p < NP; p++) {
                    const uint32_t ka = t < stp[2 * p] ? k0 : 0u, kb = t < stp[2 * p + 1] ? k0 : 0u;
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        const int2 r = L.ro2[p][i0[e] & 15];
                        const int32_t oa = ((ka >> e) & 1u) ? r.x + 2 * i0[e] : RO_EMPTY;
                        const int32_t ob = ((kb >> e) & 1u) ? r.y + 2 * i0[e] : RO_EMPTY;
                        s[p][e][0] = __builtin_amdgcn_raw_buffer_load_b16(c[2 * p].rs, oa, 0, 0);
                        s[p][e][1] = __builtin_amdgcn_raw_buffer_load_b16(c[2 * p + 1].rs, ob, 0, 0);
                    }
                }
                return;
            }
        }
        sfor<0, 2 * NP>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            int ik[4];
            uint32_t kk;
            if (same) {
                kk = t < stp[k] ? k0 : 0u;
#pragma unroll
                for (int e = 0; e < 4; e++) ik[e] = i0[e];
            } else {
                kk = 0;
                ik[0] = ik[1] = ik[2] = ik[3] = 0;
                if (t < stp[k]) kk = idx4(prof_regs(J.prof + c[k].prof), t, ik);
            }
            load4<KIND, k & 1>(c[k], rowoff[k], ik, kk, s[k >> 1]);
        });
    };
    auto put = [&]() {
#pragma unroll
        for (int p = 0; p < NP; p++) put_bm(bm + p * 8 * BRS, lane, s[p]);
    };
    const uint32_t *rp[6];
#pragma unroll
    for (int r = 0; r < 6; r++) rp[r] = bm + row[r];
    const bool mine = lane < VT;                         // lanes that build a step of the table
    fetch(0, mine ? lane : steps);
    for (int t0 = 0; t0 < steps; t0 += VT) {
        if (mine) put();
        wave_sync();
        fetch(t0 + VT, mine ? t0 + VT + lane : steps);
        acs_tile<NP>(rp, x, t0, steps, drs, rb, lane);
        wave_sync();
    }
    }
}

// Chainback (viterbi.cpp:333-357) from state 0, one lane per codeword.  The 64
// codewords' decision words of chunk c (16 KB, contiguous) are staged in LDS; lane l
// reads word [l][lr] where lr is the lane that held its traced state.  A chunk is
// one word of WS steps starting at relabelling phase 0, so the bit positions and the
// phase of every step are compile-time constants.
// LDS row per codeword: 64 words + 1 pad, so lanes tracing the same state (equal
// lr, common when the streams carry similar data) read 64 different banks
constexpr int TB_ROW = 65;
// codewords per traceback wave (32 would leave lanes 32..63 idle and halve each wave's
// chunk and register ring for two waves per SIMD: measured slower, 0.41 vs 0.37 ms)
constexpr int TB_CW = 64;
constexpr int TB_LD = TB_CW / 4;            // 16-byte loads per lane per chunk
#ifndef TB_RING_DEPTH
#define TB_RING_DEPTH 3
#endif
constexpr int TB_RING = TB_RING_DEPTH;      // decision chunks in the register ring (4 and 5 measured
                                           // no faster, profiles/r02_acs_ab.txt -- the compiler waits
                                           // vmcnt(0) at each staging anyway)
constexpr int TB_WORDS = TB_CW * TB_ROW;    // one chunk of a wave's codewords
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int TB_GROUP = 8;                 // chunks per output flush (240 bits per codeword)
constexpr int TB_PRBS = 1024;              // PRBS words (fic-handler.cpp:100-108: 32768 bits)
__device__ __forceinline__ void tb_load(u32x4 (&r)[TB_LD], const uint32_t *blk, int lane) {
    const u32x4 *q = (const u32x4 *)blk;
#pragma unroll
    for (int i = 0; i < TB_LD; i++) r[i] = q[i * 64 + lane];
}
__device__ __forceinline__ void tb_stage(uint32_t *lds, const u32x4 (&r)[TB_LD], int lane) {
    // r[i] = words 4q..4q+3 of the linear [TB_CW][64] block, q = i*64 + lane
#pragma unroll
    for (int i = 0; i < TB_LD; i++) {
        const int q = i * 64 + lane, row = q >> 4, col = (q & 15) * 4;
        uint32_t *d = lds + row * TB_ROW + col;
        d[0] = r[i].x;
        d[1] = r[i].y;
        d[2] = r[i].z;
        d[3] = r[i].w;
    }
}

// PRBS words a traceback of nch chunks reads (LDS sized by the launch)
__host__ __device__ inline int tb_prbs_words(int nch) { return min(TB_PRBS, (nch * WS + WS) / 32 + 2); }

template <int KIND>
__device__ __forceinline__ void tb_body(const VitJob &J, int blk, uint32_t *stage, uint32_t *prbs_l) {
    // a latency-bound chain that issues little: first pick on its SIMD, so it keeps
    // its pace next to throughput-bound waves of other kernels (the next run's demod)
    __builtin_amdgcn_s_setprio(3);
    const int lane = threadIdx.x, cw = blk * TB_CW + lane;
    bool act = lane < TB_CW && cw < J.n_cw;
    int N = 0, prof = 0;
    if (act) {
        // validity and profile by output row (inverse of src_of's mapping)
        if constexpr (KIND == SRC_MSC) {
            const int sub = cw % J.nsub;
            const int cl = (cw / J.nsub) % J.ncif;
            const int stream = cw / J.nsub / J.ncif;
            prof = sub;
            act = cl < J.ncifs[stream] && J.cif0s[stream] + cl >= 16;
        } else if constexpr (KIND == SRC_FRAG) {
            prof = J.cw_prof ? J.cw_prof[cw] : 0;
        } else if constexpr (KIND == SRC_FIC) {
            act = J.slots[cw >> 2] >= 0;
        }
        if (J.valid && !J.valid[cw]) act = false;
        if (act) N = J.prof[prof].nbits;
    }
    int tmax = act ? N + 6 : 0;
    for (int o = 32; o > 0; o >>= 1) tmax = max(tmax, __shfl_xor(tmax, o));
    tmax = __builtin_amdgcn_readfirstlane(tmax);         // uniform: the chunk loop stays scalar
    if (tmax == 0) return;
    const int steps = act ? N + 6 : 0;                   // inactive lanes walk garbage, store nothing
    int smin = act ? steps : tmax;                       // chunks below smin are whole in every lane
    for (int o = 32; o > 0; o >>= 1) smin = min(smin, __shfl_xor(smin, o));
    smin = __builtin_amdgcn_readfirstlane(smin);
    uint8_t *out = J.out + (act ? (int64_t)cw * J.out_stride : 0);
    const int nch = (tmax + WS - 1) / WS;
    // the energy-dispersal words in LDS: a vector load of them beside the decision
    // prefetches would wait for every outstanding load (vmcnt(0)) once per chunk
    if (J.prbs) {
        const int nw = tb_prbs_words(nch);
        for (int i = lane; i < nw; i += 64) prbs_l[i] = J.prbs_words[i];
        wave_sync();
    }
    static_assert(TB_CW == 64, "a traceback wave is one 64-row block of the decision layout");
    const uint32_t *blk0 = J.dec + dec_word_index((int64_t)blk * TB_CW, J.dec_nch);
    const int64_t cstride = 64 * 64;
    int lr = 0;                                          // lane index holding the traced state
    // decision chunks stream in through a TB_RING-deep register ring (TB_RING - 1
    // chunks of 16 KB per wave in flight while one is walked): the walk itself is short,
    // the loads are not
    u32x4 rr[TB_RING][TB_LD];
    auto ld = [&](u32x4 (&r)[TB_LD], int ch) { tb_load(r, blk0 + (int64_t)(ch > 0 ? ch : 0) * cstride, lane); };
    // Decoded bits leave in groups of TB_GROUP chunks (240 bytes per codeword, 16-byte
    // stores): vector-memory stores pending beside the decision prefetches make the
    // compiler wait for every outstanding load (vmcnt(0)), so they come rarely.
    uint32_t gb[TB_GROUP];
#pragma unroll
    for (int i = 0; i < TB_GROUP; i++) gb[i] = 0;
    const bool al16 = (((uintptr_t)J.out | (uintptr_t)J.out_stride) & 15) == 0;
    const bool al2 = (((uintptr_t)J.out | (uintptr_t)J.out_stride) & 1) == 0;
    // packed output: bits t .. t+15 as two bytes, msb first (mp4processor.cpp:115-121's
    // packing), in one 16-bit store (little-endian: byte t/8 in the low half)
    auto pk16 = [](uint32_t x) {                           // x: bit k = decoded bit t + k
        const uint32_t r = __builtin_bitreverse32(x) >> 16;   // bit 15 - k = bit t + k
        return (r >> 8) | ((r & 0xFFu) << 8);
    };
    auto flush = [&](int g) {
        const int tg = WS * TB_GROUP * g;
        if (!act || tg >= N) return;
        if (J.packed) {                                  // 240 bits = 30 bytes at byte tg / 8
            uint8_t *ob = out + tg / 8;
            if (al2 && tg + WS * TB_GROUP <= N) {
#pragma unroll
                for (int q = 0; q < WS * TB_GROUP / 16; q++) {
                    const int b = 16 * q, c = b / WS, r = b % WS;              // compile-time
                    uint32_t x = gb[c] >> r;
                    if (r > WS - 16) x |= gb[c + 1] << (WS - r);
                    *(uint16_t *)(ob + 2 * q) = (uint16_t)pk16(x & 0xFFFFu);
                }
            } else {                                     // N is a multiple of 8 (24 bitRate, 768)
                const int nb = min(WS * TB_GROUP, N - tg) / 8;
#pragma unroll
                for (int q = 0; q < WS * TB_GROUP / 8; q++) {
                    const int b = 8 * q, c = b / WS, r = b % WS;                // compile-time
                    if (q < nb) {
                        uint32_t x = gb[c] >> r;
                        if (r > WS - 8) x |= gb[c + 1] << (WS - r);
                        ob[q] = (uint8_t)(__builtin_bitreverse32(x & 0xFFu) >> 24);
                    }
                }
            }
            return;
        }
        if (al16 && tg + WS * TB_GROUP <= N) {
#pragma unroll
            for (int q = 0; q < WS * TB_GROUP / 16; q++) {
                uint32_t d[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int b = 16 * q + 4 * e, c = b / WS, r = b % WS;    // compile-time
                    uint32_t x = gb[c] >> r;
                    if (r > WS - 4) x |= gb[c + 1] << (WS - r);
                    d[e] = ((x & 0xFu) * 0x204081u) & 0x01010101u;           // 4 bits -> 4 bytes
                }
                *(uint4 *)(out + tg + 16 * q) = make_uint4(d[0], d[1], d[2], d[3]);
            }
        } else {                                         // the codeword's last group
#pragma unroll
            for (int k = 0; k < TB_GROUP; k++) {
                const int base = tg + WS * k, nk = min(WS, N - base);
                for (int i = 0; i < nk; i++) out[base + i] = (uint8_t)((gb[k] >> i) & 1u);
            }
        }
    };
    // the walk of chunk ch over its staged words
    auto walk = [&](int ch, const uint32_t *cur) {
        const uint32_t *mine = cur + (lane & (TB_CW - 1)) * TB_ROW;   // idle lanes walk a copy
        const int t0 = ch * WS;
        uint32_t w = 0;                                  // decoded bits of the chunk, step t0+k at bit k
        // two steps per LDS round trip: with the word of step k, read both candidate
        // words of step k-1 (the traced lane differs in bit p of step k only)
        static_assert(WS % 2 == 0, "step pairs");
        if (t0 + WS <= smin) {
            // every lane's chunk is whole: straight bit arithmetic, no per-step checks.
            // m = -(decision) as a 0 / all-ones mask: lr's bit p := d is one bfi, and
            // the candidate of step k-1 is picked bitwise by the same mask.
#pragma unroll
            for (int k = WS - 1; k >= 1; k -= 2) {
                const int p1 = 5 - (k % 6), p2 = 5 - ((k - 1) % 6);   // phase of step t0+k is k % 6
                const uint32_t b1 = 1u << p1, b2 = 1u << p2;
                const uint32_t w1 = mine[lr], c0 = mine[lr & ~b1], c1 = mine[lr | b1];
                const uint32_t m1 = (uint32_t)((int32_t)(w1 << (31 - dpos(k))) >> 31);     // -(decision k)
                w |= (k >= p1 ? ((uint32_t)lr << (k - p1)) : ((uint32_t)lr >> (p1 - k))) & (1u << k);
                lr = (int)((m1 & b1) | ((uint32_t)lr & ~b1));
                const uint32_t w2 = (m1 & c1) | (~m1 & c0);
                const uint32_t m2 = (uint32_t)((int32_t)(w2 << (31 - dpos(k - 1))) >> 31);
                w |= ((k - 1) >= p2 ? ((uint32_t)lr << (k - 1 - p2)) : ((uint32_t)lr >> (p2 - k + 1))) & (1u << (k - 1));
                lr = (int)((m2 & b2) | ((uint32_t)lr & ~b2));
            }
        } else {
            const bool full = t0 + WS <= steps;
#pragma unroll
            for (int k = WS - 1; k >= 1; k -= 2) {
                const int p1 = 5 - (k % 6), p2 = 5 - ((k - 1) % 6);
                const uint32_t w1 = mine[lr];
                const uint32_t c0 = mine[lr & ~(1 << p1)], c1 = mine[lr | (1 << p1)];
                {
                    const int d = (int)((w1 >> dpos(k)) & 1u);       // predecessor's msb
                    const int u = (lr >> p1) & 1;                     // decoded bit of step t0 + k
                    const int nl = (lr & ~(1 << p1)) | (d << p1);
                    if (full || t0 + k < steps) {
                        lr = nl;
                        w |= (uint32_t)u << k;
                    }
                }
                {
                    const uint32_t w2 = ((lr >> p1) & 1) ? c1 : c0;   // = mine[lr]
                    const int d = (int)((w2 >> dpos(k - 1)) & 1u);
                    const int u = (lr >> p2) & 1;
                    const int nl = (lr & ~(1 << p2)) | (d << p2);
                    if (full || t0 + k - 1 < steps) {
                        lr = nl;
                        w |= (uint32_t)u << (k - 1);
                    }
                }
            }
        }
        if (J.prbs) {                                    // energy dispersal bits t0 .. t0+29
            const int wi = t0 >> 5, sh = t0 & 31;
            const uint32_t lo = prbs_l[wi], hi = prbs_l[wi + 1];
            w ^= (sh ? (lo >> sh) | (hi << (32 - sh)) : lo) & 0x3FFFFFFFu;
        }
        // the chunk's 30 bits join the group buffer (gb[k] = chunk TB_GROUP*g + k once
        // the group's first chunk arrives; the walk runs downwards)
#pragma unroll
        for (int i = TB_GROUP - 1; i > 0; i--) gb[i] = gb[i - 1];
        gb[0] = w;
        if (ch % TB_GROUP == 0) {
            flush(ch / TB_GROUP);
            // no store left pending: the decision prefetches' waits stay exact
            __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0) expcnt(7) lgkmcnt(15)
        }
        wave_sync();
    };
    // the ring's register sets unrolled so every set is a fixed register range: the
    // wait before staging a set then covers only its own loads, not the chunks still in
    // flight behind it
    // one staging buffer: the walk's reads of chunk ch and the staging of ch - 1 are
    // ordered by the wave_sync that ends the walk (17 KB of LDS per wave, was 37 KB)
    auto chunk = [&](u32x4 (&r)[TB_LD], int ch) {
        tb_stage(stage, r, lane);
        wave_sync();
        ld(r, ch - TB_RING);
        walk(ch, stage);
    };
    sfor<0, TB_RING>([&](auto ic) { ld(rr[decltype(ic)::value], nch - 1 - decltype(ic)::value); });
    for (int ch = nch - 1; ch >= 0; ch -= TB_RING) {
        sfor<0, TB_RING>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if (ch - i >= 0) chunk(rr[i], ch - i);       // wave-uniform
        });
    }
}

template <int KIND, bool B8 = false>
__global__ __launch_bounds__(64, 8) void k_acs(VitJob J) {
    __shared__ AcsLds<1> L;
    acs_body<KIND, 1, B8>(J, xcd_order(blockIdx.x, gridDim.x), L);
}
// two jobs in one launch (the pipeline's MSC and FIC): blocks [0, nwa) run job A's waves
// wa0 .. wa0 + nwa - 1, the rest job B, so B's short waves fill the SIMDs A's last waves
// leave idle (wa0 > 0: a slice of A, DABGPU_VIT_SLICES)
template <int KA, int KB, bool B8 = false>
__global__ __launch_bounds__(64, 8) void k_acs2(VitJob A, VitJob B, int nwa, int wa0) {
    __shared__ AcsLds<1> L;
    const int b = blockIdx.x;
    if (b < nwa) acs_body<KA, 1, B8>(A, wa0 + xcd_order(b, nwa), L);
    else acs_body<KB, 1, B8>(B, xcd_order(b - nwa, gridDim.x - nwa), L);
}
// LDS (dynamic): the staging buffer, then tb_prbs_words(dec_nch) PRBS words
template <int KIND>
__global__ __launch_bounds__(64) void k_traceback(VitJob J) {
    extern __shared__ uint32_t tb_lds[];
    tb_body<KIND>(J, blockIdx.x, tb_lds, tb_lds + TB_WORDS);
}
template <int KA, int KB>
__global__ __launch_bounds__(64) void k_traceback2(VitJob A, VitJob B, int nba, int ba0) {
    extern __shared__ uint32_t tb_lds[];
    if ((int)blockIdx.x < nba) tb_body<KA>(A, ba0 + blockIdx.x, tb_lds, tb_lds + TB_WORDS);
    else tb_body<KB>(B, blockIdx.x - nba, tb_lds, tb_lds + TB_WORDS);
}
static size_t tb_lds_bytes(int nch) { return 4 * (size_t)(TB_WORDS + tb_prbs_words(nch)); }

// FIB CRC check (dab-constants.h:310-340): invert the 16 CRC bits in place, run
// CRC-CCITT from all-ones over 256 bits, pass iff the register ends at zero.  The CRC is
// linear, so one wave per FIB: lane l takes bits 4l..4l+3 (one coalesced 4-byte load),
// XORs the contributions of its 1 bits (host table, FIBCRC_OFF) and the wave XOR-reduces.
// No LDS allocation: the kernel runs beside the next run's demod, whose workgroups hold
// all of a CU's LDS (the 512-byte table is read through the caches instead).
// slots (optional): ring slot per frame (12 FIBs), < 0 = frame not committed: no check, ok = 0
// packed: the FIBs as 32 bytes each, msb first (dabgpu_pipe_set_packed DABGPU_PACK_FIC): lane l
// takes the nibble of bits 4l..4l+3 (the high nibble of byte l/2 for even l), the CRC bytes
// 30 and 31 are inverted by their even lanes
__global__ __launch_bounds__(256) void k_fic_post(uint8_t *__restrict__ bits, uint8_t *__restrict__ ok, int n_fib,
                                                  const int32_t *__restrict__ slots,
                                                  const uint16_t *__restrict__ tab, int packed) {
    const int lane = threadIdx.x & 63;
    const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= n_fib) return;
    if (slots && slots[f / 12] < 0) {
        if (lane == 0) ok[f] = 0;
        return;
    }
    uint32_t v;                                          // bit 4l + e of the FIB at bit 8e
    if (packed) {
        uint8_t *b = bits + (int64_t)f * 32 + (lane >> 1);
        uint32_t x = *b;
        if (lane >= 60) {                                // bytes 30, 31: the CRC, inverted
            x ^= 0xFFu;
            if (!(lane & 1)) *b = (uint8_t)x;
        }
        const uint32_t nib = (lane & 1) ? x & 0xFu : x >> 4;    // bit 4l + e at bit 3 - e
        v = ((nib >> 3) & 1u) | (((nib >> 2) & 1u) << 8) | (((nib >> 1) & 1u) << 16) | ((nib & 1u) << 24);
    } else {
        uint32_t *w = (uint32_t *)(bits + (int64_t)f * 256) + lane;
        v = *w;
        if (lane >= 60) {                                // bits 240..255: the CRC, inverted
            v ^= 0x01010101u;
            *w = v;
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int e = 0; e < 4; e++)
        if ((v >> (8 * e)) & 0xFFu) r ^= tab[4 * lane + e];
#pragma unroll
    for (int o = 32; o; o >>= 1) r ^= (uint32_t)__shfl_xor((int)r, o, 64);
    if (lane == 0) ok[f] = (r ^ tab[256]) == 0;
}

template <template <int> class K>
static hipError_t launch_kind(hipStream_t st, const VitJob &job, dim3 grid, size_t lds = 0) {
    switch (job.kind) {
    case SRC_MOTHER: hipLaunchKernelGGL(K<SRC_MOTHER>::fn(), grid, dim3(64), lds, st, job); break;
    case SRC_FRAG:   hipLaunchKernelGGL(K<SRC_FRAG>::fn(), grid, dim3(64), lds, st, job); break;
    case SRC_FIC:    hipLaunchKernelGGL(K<SRC_FIC>::fn(), grid, dim3(64), lds, st, job); break;
    case SRC_MSC:    hipLaunchKernelGGL(K<SRC_MSC>::fn(), grid, dim3(64), lds, st, job); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
template <int KIND> struct AcsK { static auto fn() { return k_acs<KIND>; } };
template <int KIND> struct TbK { static auto fn() { return k_traceback<KIND>; } };

// One codeword pair per wave (NP = 1).  NP > 1 (independent chains interleaved in one
// wave, fewer waves) measured slower on MI355X for the C3 batch: 0.81 ms (NP=2) and
// 1.14 ms (NP=3) vs 0.72 ms per launch -- thread-level parallelism hides the
// DPP hazards and LDS latency better than instruction-level parallelism here.
hipError_t launch_acs(hipStream_t st, const VitJob &job) {
    if (job.n_cw <= 0) return hipSuccess;
    if (job.dec_ncw < dec_rows(job.n_cw) || job.dec_nch <= 0) return hipErrorInvalidValue;
    if (job.ring8) {                                   // the pipeline's RING8 soft-bit ring
        const dim3 grid((job.n_cw + 1) / 2);
        if (job.kind == SRC_FIC) hipLaunchKernelGGL((k_acs<SRC_FIC, true>), grid, dim3(64), 0, st, job);
        else if (job.kind == SRC_MSC) hipLaunchKernelGGL((k_acs<SRC_MSC, true>), grid, dim3(64), 0, st, job);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    return launch_kind<AcsK>(st, job, dim3((job.n_cw + 1) / 2));
}
hipError_t launch_traceback(hipStream_t st, const VitJob &job) {
    if (job.n_cw <= 0) return hipSuccess;
    if (job.dec_ncw < dec_rows(job.n_cw) || job.dec_nch <= 0) return hipErrorInvalidValue;
    return launch_kind<TbK>(st, job, dim3((job.n_cw + TB_CW - 1) / TB_CW), tb_lds_bytes(job.dec_nch));
}
hipError_t launch_viterbi(hipStream_t st, const VitJob &job) {
    hipError_t e = launch_acs(st, job);
    return e != hipSuccess ? e : launch_traceback(st, job);
}
// MSC (a) and FIC (b) decoded by one ACS launch and one traceback launch.  The _range
// forms decode the MSC's traceback blocks [b0, b1) (64 codewords each; the ACS's waves
// 32 b0 .. 32 b1) and, with fic, the FIC: slices of the batch (DABGPU_VIT_SLICES A/B)
hipError_t launch_acs_msc_fic_range(hipStream_t st, const VitJob &a, const VitJob &b, int b0, int b1, bool fic) {
    if (a.kind != SRC_MSC || b.kind != SRC_FIC || a.n_cw <= 0 || b.n_cw <= 0) return hipErrorInvalidValue;
    if (a.dec_ncw < dec_rows(a.n_cw) || b.dec_ncw < dec_rows(b.n_cw) || a.dec_nch <= 0 || b.dec_nch <= 0)
        return hipErrorInvalidValue;
    if (a.ring8 != b.ring8) return hipErrorInvalidValue;
    const int nwa_all = (a.n_cw + 1) / 2, nwb = fic ? (b.n_cw + 1) / 2 : 0;
    const int w0 = b0 * (TB_CW / 2), w1 = min(nwa_all, b1 * (TB_CW / 2));
    if (b0 < 0 || w0 >= w1) return hipErrorInvalidValue;
    const int nwa = w1 - w0;
    if (a.ring8) hipLaunchKernelGGL((k_acs2<SRC_MSC, SRC_FIC, true>), dim3(nwa + nwb), dim3(64), 0, st, a, b, nwa, w0);
    else hipLaunchKernelGGL((k_acs2<SRC_MSC, SRC_FIC>), dim3(nwa + nwb), dim3(64), 0, st, a, b, nwa, w0);
    return hipGetLastError();
}
hipError_t launch_traceback_msc_fic_range(hipStream_t st, const VitJob &a, const VitJob &b, int b0, int b1, bool fic) {
    if (a.kind != SRC_MSC || b.kind != SRC_FIC || a.n_cw <= 0 || b.n_cw <= 0) return hipErrorInvalidValue;
    const int nba_all = (a.n_cw + TB_CW - 1) / TB_CW, nbb = fic ? (b.n_cw + TB_CW - 1) / TB_CW : 0;
    b1 = min(b1, nba_all);
    if (b0 < 0 || b0 >= b1) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_traceback2<SRC_MSC, SRC_FIC>), dim3(b1 - b0 + nbb), dim3(64),
                       tb_lds_bytes(max(a.dec_nch, b.dec_nch)), st, a, b, b1 - b0, b0);
    return hipGetLastError();
}
hipError_t launch_acs_msc_fic(hipStream_t st, const VitJob &a, const VitJob &b) {
    return launch_acs_msc_fic_range(st, a, b, 0, (a.n_cw + TB_CW - 1) / TB_CW, true);
}
hipError_t launch_traceback_msc_fic(hipStream_t st, const VitJob &a, const VitJob &b) {
    return launch_traceback_msc_fic_range(st, a, b, 0, (a.n_cw + TB_CW - 1) / TB_CW, true);
}

hipError_t launch_fic_post(hipStream_t st, uint8_t *bits, uint8_t *ok, int n_fib, const uint8_t *tabs,
                           const int32_t *slots, bool packed) {
    if (n_fib <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fic_post, dim3((n_fib + 3) / 4), dim3(256), 0, st, bits, ok, n_fib, slots,
                       (const uint16_t *)(tabs + FIBCRC_OFF), packed ? 1 : 0);
    return hipGetLastError();
}

}  // namespace dab
