/*
 * dab_oracle.c -- TEST INFRASTRUCTURE ONLY (see dab_oracle.h).
 *
 * Plain-C restatement of the sdr-j-dab v0.997 DAB Mode-I hot path.  Each
 * function names the reference lines it follows.  Float semantics follow
 * the reference's x86-64 -O2 build without -ffast-math: every complex<float>
 * product is two float products and one float add/sub (no FMA), std::abs on
 * a complex is hypotf, std::arg is atan2f.
 */
#include "dab_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

typedef struct { float re, im; } cf;

/* complex<float> a*b, a*conj(b) and a+=b, evaluated like GCC's inline
 * _Complex float multiply (two roundings for each product, one for the sum) */
static inline cf cmulf(cf a, cf b) {
    volatile float ac = a.re * b.re, bd = a.im * b.im, ad = a.re * b.im, bc = a.im * b.re;
    cf r; r.re = ac - bd; r.im = ad + bc; return r;
}
static inline cf cmul_conjf(cf a, cf b) {   /* a * conj(b) = (a.re,a.im)*(b.re,-b.im) */
    volatile float ac = a.re * b.re, bd = a.im * (-b.im), ad = a.re * (-b.im), bc = a.im * b.re;
    cf r; r.re = ac - bd; r.im = ad + bc; return r;
}
static inline float jan_abs(cf z) {          /* dab-constants.h:127-134 */
    float re = z.re < 0 ? -z.re : z.re;
    float im = z.im < 0 ? -z.im : z.im;
    return re + im;
}
static inline float cabs_f(cf z) { return hypotf(z.re, z.im); }   /* std::abs(complex<float>) */
static inline float carg_f(cf z) { return atan2f(z.im, z.re); }   /* std::arg(complex<float>) */

/* ------------------------------------------------------------------ tables */

/* Frequency-interleaving permutation, Mode I: V1 = 511, accept [256, 1792] \ {1024},
 * store value - 1024 (mapper.cpp:33-55 with the Mode-I arguments of mapper.cpp:84-86). */
void orc_mapper(int16_t *perm) {
    int16_t seq[ORC_TU];
    seq[0] = 0;
    for (int i = 1; i < ORC_TU; i++) seq[i] = (int16_t)((13 * seq[i - 1] + 511) % ORC_TU);
    int n = 0;
    for (int i = 0; i < ORC_TU; i++) {
        int v = seq[i];
        if (v == ORC_TU / 2) continue;
        if (v < 256 || v > 256 + ORC_K) continue;
        perm[n++] = (int16_t)(v - ORC_TU / 2);
    }
}

/* ETSI EN 300 401 Mode-I phase reference parameters, one row per 32 carriers:
 * (k_min, i, n) with k_max = k_min + 31 (phasetable.cpp:115-166, including the
 * 2014-09-03 fix of row k_min = 97). */
static const int16_t phi_rows[48][3] = {
    {-768,0,1},{-736,1,2},{-704,2,0},{-672,3,1},{-640,0,3},{-608,1,2},{-576,2,2},{-544,3,3},
    {-512,0,2},{-480,1,1},{-448,2,2},{-416,3,3},{-384,0,1},{-352,1,2},{-320,2,3},{-288,3,3},
    {-256,0,2},{-224,1,2},{-192,2,2},{-160,3,1},{-128,0,1},{ -96,1,3},{ -64,2,1},{ -32,3,2},
    {   1,0,3},{  33,3,1},{  65,2,1},{  97,1,1},{ 129,0,2},{ 161,3,2},{ 193,2,1},{ 225,1,0},
    { 257,0,2},{ 289,3,2},{ 321,2,3},{ 353,1,3},{ 385,0,0},{ 417,3,2},{ 449,2,1},{ 481,1,3},
    { 513,0,3},{ 545,3,3},{ 577,2,3},{ 609,1,0},{ 641,0,3},{ 673,3,0},{ 705,2,1},{ 737,1,1}};
/* h_{i,j} time-frequency phase parameter, 16-periodic (phasetable.cpp:234-259) */
static const int8_t h_par[4][16] = {
    {0,2,0,0,0,0,1,1,2,0,0,0,2,2,1,1},
    {0,3,2,3,0,1,3,0,2,1,2,3,2,3,3,0},
    {0,0,0,2,0,2,1,3,2,2,0,2,2,0,1,3},
    {0,1,2,1,0,3,3,2,2,3,2,1,2,1,3,2}};

float orc_get_phi(int32_t k) {               /* phasetable.cpp:261-274 */
    for (int r = 0; r < 48; r++) {
        int kmin = phi_rows[r][0];
        if (kmin <= k && k <= kmin + 31) {
            int i = phi_rows[r][1], n = phi_rows[r][2];
            return (float)(M_PI / 2 * (h_par[i][(k - kmin) & 15] + n));
        }
    }
    return 0.0f;
}

void orc_ref_table(float *ref) {              /* phasereference.cpp:40-47 */
    memset(ref, 0, sizeof(float) * 2 * ORC_TU);
    for (int i = 1; i <= ORC_K / 2; i++) {
        float phi = orc_get_phi(i);
        ref[2 * i] = cosf(phi);  ref[2 * i + 1] = sinf(phi);
        phi = orc_get_phi(-i);
        ref[2 * (ORC_TU - i)] = cosf(phi);  ref[2 * (ORC_TU - i) + 1] = sinf(phi);
    }
}

void orc_osc_entry(int32_t i, float *re, float *im) {   /* ofdm-processor.cpp:79-81 */
    *re = (float)cos(2.0 * M_PI * i / ORC_INPUT_RATE);
    *im = (float)sin(2.0 * M_PI * i / ORC_INPUT_RATE);
}

/* Energy-dispersal PRBS x^9 + x^5 + 1, all-ones start (fic-handler.cpp:100-108,
 * identical sequence in dab-concurrent.cpp:183-190). */
void orc_prbs(int n, uint8_t *out) {
    uint8_t sr[9];
    memset(sr, 1, 9);
    for (int i = 0; i < n; i++) {
        uint8_t b = sr[8] ^ sr[4];
        for (int j = 8; j > 0; j--) sr[j] = sr[j - 1];
        sr[0] = b;
        out[i] = b;
    }
}

/* Puncturing vectors PI_1..PI_24 (protTables.cpp:28-58 = ETSI EN 300 401 Table 29).
 * PI_k keeps 8+k of 32 bits; per 4-bit group g the kept count is
 * 1 + (k-1)/8 plus one for group 0 and for the first (k-1)%8 groups of the
 * fill order {4,2,6,1,5,3,7}; kept bits are the leading bits of each group. */
void orc_pcode(int idx, int8_t *out) {
    static const int order[7] = {4, 2, 6, 1, 5, 3, 7};
    int base = 1 + (idx - 1) / 8, extra = (idx - 1) % 8;
    int cnt[8];
    for (int g = 0; g < 8; g++) cnt[g] = base;
    cnt[0] += 1;
    for (int e = 0; e < extra; e++) cnt[order[e]] += 1;
    for (int g = 0; g < 8; g++)
        for (int b = 0; b < 4; b++) out[4 * g + b] = (int8_t)(b < cnt[g] ? 1 : 0);
}

/* UEP protection profiles (deconvolve.cpp:39-114 = ETSI EN 300 401 Table 8):
 * bitRate, level, L1..L4, PI1..PI4 */
static const int16_t uep_tab[][10] = {
    {32,5,3,4,17,0,5,3,2,-1},{32,4,3,3,18,0,11,6,5,-1},{32,3,3,4,14,3,15,9,6,8},
    {32,2,3,4,14,3,22,13,8,13},{32,1,3,5,13,3,24,17,12,17},
    {48,5,4,3,26,3,5,4,2,3},{48,4,3,4,26,3,9,6,4,6},{48,3,3,4,26,3,15,10,6,9},
    {48,2,3,4,26,3,24,14,8,15},{48,1,3,5,25,3,24,18,13,18},
    {64,5,6,9,31,2,5,3,2,3},{64,4,6,9,33,0,11,6,6,-1},{64,3,6,12,27,3,16,8,6,9},
    {64,2,6,10,29,3,23,13,8,13},{64,1,6,11,28,3,24,18,12,18},
    {80,5,6,10,41,3,6,3,2,3},{80,4,6,10,41,3,11,6,5,6},{80,3,6,11,40,3,16,8,6,7},
    {80,2,6,10,41,3,23,13,8,13},{80,1,6,10,41,3,24,7,12,18},
    {96,5,7,9,53,3,5,4,2,4},{96,4,7,10,52,3,9,6,4,6},{96,3,6,12,51,3,16,9,6,10},
    {96,2,6,10,53,3,22,12,9,12},{96,1,6,13,50,3,24,18,13,19},
    {112,5,14,17,50,3,5,4,2,5},{112,4,11,21,49,3,9,6,4,8},{112,3,11,23,47,3,16,8,6,9},
    {112,2,11,21,49,3,23,12,9,14},
    {128,5,12,19,62,3,5,3,2,4},{128,4,11,21,61,3,11,6,5,7},{128,3,11,22,60,3,16,9,6,10},
    {128,2,11,21,61,3,22,12,9,14},{128,1,11,20,62,3,24,17,13,19},
    {160,5,11,19,87,3,5,4,2,4},{160,4,11,23,83,3,11,6,5,9},{160,3,11,24,82,3,16,8,6,11},
    {160,2,11,21,85,3,22,11,9,13},{160,1,11,22,84,3,24,18,12,19},
    {192,5,11,20,110,3,6,4,2,5},{192,4,11,22,108,3,10,6,4,9},{192,3,11,24,106,3,16,10,6,11},
    {192,2,11,20,110,3,22,13,9,13},{192,1,11,21,109,3,24,20,13,24},
    {224,5,12,22,131,3,8,6,2,6},{224,4,12,26,127,3,12,8,4,11},{224,3,11,20,134,3,16,10,7,9},
    {224,2,11,22,132,3,24,16,10,15},{224,1,11,24,130,3,24,20,12,20},
    {256,5,11,24,154,3,6,5,2,5},{256,4,11,24,154,3,12,9,5,10},{256,3,11,27,151,3,16,10,7,10},
    {256,2,11,22,156,3,24,14,10,13},{256,1,11,26,152,3,24,19,14,18},
    {320,5,11,26,200,3,8,5,2,6},{320,4,11,25,201,3,13,9,5,10},{320,2,11,26,200,3,24,17,9,17},
    {384,5,11,27,247,3,8,6,2,7},{384,3,11,24,250,3,16,9,7,10},{384,1,12,28,245,3,24,20,14,23}};

int orc_uep_profile(int bitRate, int protLevel, int16_t *L, int16_t *PI) {
    int n = (int)(sizeof(uep_tab) / sizeof(uep_tab[0]));
    int idx = -1;
    for (int i = 0; i < n; i++)
        if (uep_tab[i][0] == bitRate && uep_tab[i][1] == protLevel) { idx = i; break; }
    int found = idx >= 0;
    if (!found) idx = 1;      /* deconvolve.cpp:150-153: unknown profile falls back to row 1 */
    for (int j = 0; j < 4; j++) { L[j] = uep_tab[idx][2 + j]; PI[j] = uep_tab[idx][6 + j]; }
    return found;
}

/* EEP A/B profiles (deconvolve.cpp:244-314 = ETSI EN 300 401 §11.3.2).
 * protLevel carries 0100 (A) or 0200 (B) plus the level 1..4. Returns 0 when
 * neither flag is set (the reference leaves its fields uninitialised then). */
int orc_eep_profile(int bitRate, int protLevel, int16_t *L, int16_t *PI) {
    int lvl = protLevel & 07;
    if (protLevel & 0100) {
        switch (lvl) {
        case 1: L[0] = 6 * bitRate / 8 - 3; L[1] = 3; PI[0] = 24; PI[1] = 23; return 1;
        case 2:
            if (bitRate == 8) { L[0] = 5; L[1] = 1; PI[0] = 13; PI[1] = 12; }
            else { L[0] = 2 * bitRate / 8 - 3; L[1] = 4 * bitRate / 8 + 3; PI[0] = 14; PI[1] = 13; }
            return 1;
        case 3: L[0] = 6 * bitRate / 8 - 3; L[1] = 3; PI[0] = 8; PI[1] = 7; return 1;
        case 4: L[0] = 4 * bitRate / 8 - 3; L[1] = 2 * bitRate / 8 + 3; PI[0] = 3; PI[1] = 2; return 1;
        }
        return 0;
    }
    if (protLevel & 0200) {
        int l1 = 24 * bitRate / 32 - 3;
        switch (lvl) {
        case 4: L[0] = l1; L[1] = 3; PI[0] = 2; PI[1] = 1; return 1;
        case 3: L[0] = l1; L[1] = 3; PI[0] = 4; PI[1] = 3; return 1;
        case 2: L[0] = l1; L[1] = 3; PI[0] = 6; PI[1] = 5; return 1;
        case 1: L[0] = l1; L[1] = 3; PI[0] = 10; PI[1] = 9; return 1;
        }
    }
    return 0;
}

/* time-interleaving delay of branch i&15: 15 - bitreverse4(i) (dab-concurrent.cpp:42-43) */
int orc_interleave_delay(int i) {
    int b = i & 15;
    int r = ((b & 1) << 3) | ((b & 2) << 1) | ((b & 4) >> 1) | ((b & 8) >> 3);
    return 15 - r;
}

/* -------------------------------------------------------------------- FFT */

/* 2048-point DFT, forward e^{-j}, unscaled; inverse e^{+j} then x 1/N
 * (fft.cpp:53 / fft.cpp:109-121).  Computed in double, rounded to float:
 * the "ideal" fp32 FFT that stands in for the un-vendored FFTW3f. */
void orc_fft2048(const float *in, float *out, int inverse) {
    static double tw_re[ORC_TU / 2], tw_im[ORC_TU / 2];
    static int init = 0;
    if (!init) {
        for (int k = 0; k < ORC_TU / 2; k++) {
            tw_re[k] = cos(2.0 * M_PI * k / ORC_TU);
            tw_im[k] = -sin(2.0 * M_PI * k / ORC_TU);
        }
        init = 1;
    }
    double re[ORC_TU], im[ORC_TU];
    for (int n = 0; n < ORC_TU; n++) {       /* bit-reversed load */
        int r = 0, x = n;
        for (int b = 0; b < 11; b++) { r = (r << 1) | (x & 1); x >>= 1; }
        re[r] = in[2 * n]; im[r] = in[2 * n + 1];
    }
    double sgn = inverse ? -1.0 : 1.0;
    for (int len = 2; len <= ORC_TU; len <<= 1) {
        int half = len >> 1, step = ORC_TU / len;
        for (int s = 0; s < ORC_TU; s += len)
            for (int j = 0; j < half; j++) {
                double wr = tw_re[j * step], wi = sgn * tw_im[j * step];
                double xr = re[s + j + half], xi = im[s + j + half];
                double tr = xr * wr - xi * wi, ti = xr * wi + xi * wr;
                re[s + j + half] = re[s + j] - tr; im[s + j + half] = im[s + j] - ti;
                re[s + j] += tr; im[s + j] += ti;
            }
    }
    const float factor = (float)(1.0 / (float)ORC_TU);
    for (int k = 0; k < ORC_TU; k++) {
        float fr = (float)re[k], fi = (float)im[k];
        if (inverse) { fr *= factor; fi *= factor; }
        out[2 * k] = fr; out[2 * k + 1] = fi;
    }
}

/* 2048-point FFT in fp32 (round 5): the precision class of the reference's FFTW3f
 * (fft.cpp:31-121 links libfftw3f with FFTW_ESTIMATE plans; FFTW is an un-vendored
 * dependency absent from this image).  A Stockham radix-4 transform --
 * five radix-4 DIF passes (n = 2048, 512, 128, 32, 8) and one radix-2 pass, natural
 * order in and out -- with every butterfly and twiddle product in float (two rounded
 * products and a rounded sum per real part, no FMA) and the twiddles computed in
 * double and rounded once, as FFTW precomputes its twiddles.  Forward unscaled;
 * inverse = conj(FFT(conj(x))) x 1/N (fft.cpp:109-121).  Split re/im arrays so the
 * passes vectorise.  Used (1) for the fp32 floor of the soft values
 * (tests/test_gpu_parity.py, test_demod_nco_matches_oracle) and (2) as the CPU
 * baseline's FFT (bench.py cpu_baseline). */
static float g_w32r[ORC_TU], g_w32i[ORC_TU];
static void w32_init(void) {
    static int init = 0;
    if (init) return;
    for (int k = 0; k < ORC_TU; k++) {
        g_w32r[k] = (float)cos(2.0 * M_PI * k / ORC_TU);
        g_w32i[k] = (float)-sin(2.0 * M_PI * k / ORC_TU);
    }
    init = 1;
}
/* one radix-4 DIF pass of the Stockham transform: sequences of length n = 4m at
 * stride s (x) -> y */
__attribute__((optimize("O3", "tree-vectorize")))
static void r4pass(const float *restrict xr, const float *restrict xi, float *restrict yr, float *restrict yi,
                   int m, int s) {
    for (int p = 0; p < m; p++) {
        const float w1r = g_w32r[p * s], w1i = g_w32i[p * s];
        const float w2r = g_w32r[2 * p * s], w2i = g_w32i[2 * p * s];
        const float w3r = g_w32r[3 * p * s], w3i = g_w32i[3 * p * s];
        const float *ar = xr + s * p, *ai = xi + s * p;
        float *or_ = yr + s * 4 * p, *oi = yi + s * 4 * p;
        for (int q = 0; q < s; q++) {
            const float a_r = ar[q], a_i = ai[q];
            const float b_r = ar[q + s * m], b_i = ai[q + s * m];
            const float c_r = ar[q + 2 * s * m], c_i = ai[q + 2 * s * m];
            const float d_r = ar[q + 3 * s * m], d_i = ai[q + 3 * s * m];
            const float apc_r = a_r + c_r, apc_i = a_i + c_i;
            const float amc_r = a_r - c_r, amc_i = a_i - c_i;
            const float bpd_r = b_r + d_r, bpd_i = b_i + d_i;
            const float jbmd_r = -(b_i - d_i), jbmd_i = b_r - d_r;      /* j (b - d) */
            or_[q] = apc_r + bpd_r; oi[q] = apc_i + bpd_i;
            const float t1r = amc_r - jbmd_r, t1i = amc_i - jbmd_i;
            const float t2r = apc_r - bpd_r, t2i = apc_i - bpd_i;
            const float t3r = amc_r + jbmd_r, t3i = amc_i + jbmd_i;
            /* two rounded products and one rounded sum per part (no FMA: -ffp-contract=off) */
            or_[q + s] = w1r * t1r - w1i * t1i; oi[q + s] = w1r * t1i + w1i * t1r;
            or_[q + 2 * s] = w2r * t2r - w2i * t2i; oi[q + 2 * s] = w2r * t2i + w2i * t2r;
            or_[q + 3 * s] = w3r * t3r - w3i * t3i; oi[q + 3 * s] = w3r * t3i + w3i * t3r;
        }
    }
}
/* the first pass (s = 1), vectorised over p: the same butterflies */
__attribute__((optimize("O3", "tree-vectorize")))
static void r4pass_first(const float *restrict xr, const float *restrict xi, float *restrict yr, float *restrict yi) {
    const int m = ORC_TU / 4;
    for (int p = 0; p < m; p++) {
        const float w1r = g_w32r[p], w1i = g_w32i[p], w2r = g_w32r[2 * p], w2i = g_w32i[2 * p];
        const float w3r = g_w32r[3 * p], w3i = g_w32i[3 * p];
        const float a_r = xr[p], a_i = xi[p], b_r = xr[p + m], b_i = xi[p + m];
        const float c_r = xr[p + 2 * m], c_i = xi[p + 2 * m], d_r = xr[p + 3 * m], d_i = xi[p + 3 * m];
        const float apc_r = a_r + c_r, apc_i = a_i + c_i;
        const float amc_r = a_r - c_r, amc_i = a_i - c_i;
        const float bpd_r = b_r + d_r, bpd_i = b_i + d_i;
        const float jbmd_r = -(b_i - d_i), jbmd_i = b_r - d_r;
        const float t1r = amc_r - jbmd_r, t1i = amc_i - jbmd_i;
        const float t2r = apc_r - bpd_r, t2i = apc_i - bpd_i;
        const float t3r = amc_r + jbmd_r, t3i = amc_i + jbmd_i;
        yr[4 * p] = apc_r + bpd_r; yi[4 * p] = apc_i + bpd_i;
        yr[4 * p + 1] = w1r * t1r - w1i * t1i; yi[4 * p + 1] = w1r * t1i + w1i * t1r;
        yr[4 * p + 2] = w2r * t2r - w2i * t2i; yi[4 * p + 2] = w2r * t2i + w2i * t2r;
        yr[4 * p + 3] = w3r * t3r - w3i * t3i; yi[4 * p + 3] = w3r * t3i + w3i * t3r;
    }
}
__attribute__((optimize("O3", "tree-vectorize")))
static void r2pass_last(const float *restrict xr, const float *restrict xi, float *restrict yr, float *restrict yi) {
    const int s = ORC_TU / 2;
    for (int q = 0; q < s; q++) {
        const float a_r = xr[q], a_i = xi[q], b_r = xr[q + s], b_i = xi[q + s];
        yr[q] = a_r + b_r; yi[q] = a_i + b_i;
        yr[q + s] = a_r - b_r; yi[q + s] = a_i - b_i;
    }
}
/* x -> y (pass 1), y -> x, x -> y, y -> x, x -> y (n = 8), y -> x (radix-2): result in x */
static void fft2048_f32_fwd(float *xr, float *xi, float *yr, float *yi) {
    r4pass_first(xr, xi, yr, yi);
    r4pass(yr, yi, xr, xi, 128, 4);
    r4pass(xr, xi, yr, yi, 32, 16);
    r4pass(yr, yi, xr, xi, 8, 64);
    r4pass(xr, xi, yr, yi, 2, 256);
    r2pass_last(yr, yi, xr, xi);
}
void orc_fft2048_f32(const float *in, float *out, int inverse) {
    w32_init();
    float xr[ORC_TU], xi[ORC_TU], yr[ORC_TU], yi[ORC_TU];
    const float sg = inverse ? -1.0f : 1.0f;          /* inverse: conj in, conj out */
    for (int k = 0; k < ORC_TU; k++) { xr[k] = in[2 * k]; xi[k] = sg * in[2 * k + 1]; }
    fft2048_f32_fwd(xr, xi, yr, yi);          /* 5 radix-4 passes + the radix-2 pass end in xr/xi */
    const float factor = (float)(1.0 / (float)ORC_TU);
    for (int k = 0; k < ORC_TU; k++) {
        float fr = xr[k], fi = sg * xi[k];
        if (inverse) { fr *= factor; fi *= factor; }
        out[2 * k] = fr; out[2 * k + 1] = fi;
    }
}

/* two more fp32 transforms of FFTW3f's precision class, for the spread of fp32 FFT
 * rounding (the soft values' fp32 floor, tests/test_gpu_parity.py): the radix-2
 * decimation-in-time transform of orc_fft2048 carried out in float (bit-reversed load),
 * and the radix-2 decimation-in-frequency (Gentleman-Sande) transform (bit-reversed
 * store); float butterflies, twiddles rounded once from double, no FMA */
static void fft2048_f32_r2(const float *in, float *out, int inverse, int dif) {
    w32_init();
    float re[ORC_TU], im[ORC_TU];
    const float sg = inverse ? -1.0f : 1.0f;
    for (int n = 0; n < ORC_TU; n++) {
        int r = n;
        if (!dif) { r = 0; int x = n; for (int b = 0; b < 11; b++) { r = (r << 1) | (x & 1); x >>= 1; } }
        re[r] = in[2 * n]; im[r] = sg * in[2 * n + 1];
    }
    if (!dif) {
        for (int len = 2; len <= ORC_TU; len <<= 1) {
            const int half = len >> 1, step = ORC_TU / len;
            for (int s0 = 0; s0 < ORC_TU; s0 += len)
                for (int j = 0; j < half; j++) {
                    const float wr = g_w32r[j * step], wi = g_w32i[j * step];
                    const float xr = re[s0 + j + half], xi = im[s0 + j + half];
                    const float tr = xr * wr - xi * wi, ti = xr * wi + xi * wr;
                    re[s0 + j + half] = re[s0 + j] - tr; im[s0 + j + half] = im[s0 + j] - ti;
                    re[s0 + j] += tr; im[s0 + j] += ti;
                }
        }
    } else {
        for (int len = ORC_TU; len >= 2; len >>= 1) {
            const int half = len >> 1, step = ORC_TU / len;
            for (int s0 = 0; s0 < ORC_TU; s0 += len)
                for (int j = 0; j < half; j++) {
                    const float wr = g_w32r[j * step], wi = g_w32i[j * step];
                    const float ar = re[s0 + j], ai = im[s0 + j], br = re[s0 + j + half], bi = im[s0 + j + half];
                    re[s0 + j] = ar + br; im[s0 + j] = ai + bi;
                    const float dr = ar - br, di = ai - bi;
                    re[s0 + j + half] = dr * wr - di * wi; im[s0 + j + half] = dr * wi + di * wr;
                }
        }
    }
    const float factor = (float)(1.0 / (float)ORC_TU);
    for (int k = 0; k < ORC_TU; k++) {
        int r = k;
        if (dif) { r = 0; int x = k; for (int b = 0; b < 11; b++) { r = (r << 1) | (x & 1); x >>= 1; } }
        float fr = re[r], fi = sg * im[r];
        if (inverse) { fr *= factor; fi *= factor; }
        out[2 * k] = fr; out[2 * k + 1] = fi;
    }
}
static void fft2048_f32_dit(const float *in, float *out, int inverse) { fft2048_f32_r2(in, out, inverse, 0); }
static void fft2048_f32_dif(const float *in, float *out, int inverse) { fft2048_f32_r2(in, out, inverse, 1); }
void orc_fft2048_kind(const float *in, float *out, int inverse, int kind) {
    if (kind == 2) fft2048_f32_dit(in, out, inverse);
    else if (kind == 3) fft2048_f32_dif(in, out, inverse);
    else if (kind == 1) orc_fft2048_f32(in, out, inverse);
    else orc_fft2048(in, out, inverse);
}

/* the front end's FFT: 0 = the double-precision "ideal" transform (the parity
 * oracle), 1 = the fp32 radix-4 (FFTW3f's precision class, CPU baseline), 2 / 3 = the
 * fp32 radix-2 DIT / DIF */
typedef void (*orc_fft_fn)(const float *, float *, int);
static orc_fft_fn fft_of(int kind) {
    return kind == 1 ? orc_fft2048_f32 : kind == 2 ? fft2048_f32_dit : kind == 3 ? fft2048_f32_dif : orc_fft2048;
}

/* ------------------------------------------------------------ OFDM front */

static float g_ref[2 * ORC_TU];
static int16_t g_perm[ORC_K];
static float g_refarg[18];
static int g_tables = 0;
/* oscillatorTable (ofdm-processor.cpp:76-81): 2,048,000 cf32, as the reference keeps it */
static float *g_osc = NULL;
static void tables_init(void) {
    if (g_tables) return;
    orc_ref_table(g_ref);
    orc_mapper(g_perm);
    float *osc = (float *)malloc(sizeof(float) * 2 * ORC_INPUT_RATE);
    for (int32_t i = 0; i < ORC_INPUT_RATE; i++) orc_osc_entry(i, &osc[2 * i], &osc[2 * i + 1]);
    g_osc = osc;
    for (int i = 0; i < 18; i++) {           /* ofdm-decoder.cpp:71-74 */
        cf a = {g_ref[2 * ((ORC_TU + i) % ORC_TU)], g_ref[2 * ((ORC_TU + i) % ORC_TU) + 1]};
        cf b = {g_ref[2 * ((ORC_TU + i + 1) % ORC_TU)], g_ref[2 * ((ORC_TU + i + 1) % ORC_TU) + 1]};
        g_refarg[i] = carg_f(cmul_conjf(a, b));
    }
    g_tables = 1;
}

static int32_t find_index_(const float *v, int16_t level, float *maxv, float *sumv, orc_fft_fn fft) {
    tables_init();
    float X[2 * ORC_TU], R[2 * ORC_TU];
    fft(v, X, 0);
    for (int i = 0; i < ORC_TU; i++) {
        cf a = {X[2 * i], X[2 * i + 1]}, b = {g_ref[2 * i], g_ref[2 * i + 1]};
        cf r = cmul_conjf(a, b);
        R[2 * i] = r.re; R[2 * i + 1] = r.im;
    }
    fft(R, X, 1);
    float sum = 0;
    for (int i = 0; i < ORC_TU; i++) { cf z = {X[2 * i], X[2 * i + 1]}; sum += cabs_f(z); }
    float Max = -10000;
    int32_t maxIndex = -1;
    for (int i = 0; i < ORC_TU; i++) {
        cf z = {X[2 * i], X[2 * i + 1]};
        if (cabs_f(z) > Max) { maxIndex = i; Max = cabs_f(z); }
    }
    if (maxv) *maxv = Max;
    if (sumv) *sumv = sum;
    if (Max < (float)level * sum / (float)ORC_TU)
        return (int32_t)(-fabsf(Max / (sum / (float)ORC_TU)) - 1);
    return maxIndex;
}
int32_t orc_find_index(const float *v, int16_t level, float *maxv, float *sumv) {   /* phasereference.cpp:60-88 */
    return find_index_(v, level, maxv, sumv, orc_fft2048);
}

static int16_t get_middle(const float *X) {  /* ofdm-decoder.cpp:233-258 (incl. its "sum = oldMax") */
    float sum = 0, oldMax = 0;
    int16_t maxIndex = 0;
    for (int i = 40; i < 1536 + 40; i++) { cf z = {X[2 * ((ORC_TU / 2 + i) % ORC_TU)], X[2 * ((ORC_TU / 2 + i) % ORC_TU) + 1]}; sum += cabs_f(z); }
    for (int i = 40; i < ORC_TU - (1536 - 40); i++) {
        cf a = {X[2 * ((ORC_TU / 2 + i) % ORC_TU)], X[2 * ((ORC_TU / 2 + i) % ORC_TU) + 1]};
        cf b = {X[2 * ((ORC_TU / 2 + i + 1536) % ORC_TU)], X[2 * ((ORC_TU / 2 + i + 1536) % ORC_TU) + 1]};
        sum -= cabs_f(a);
        sum += cabs_f(b);
        if (sum > oldMax) { sum = oldMax; maxIndex = (int16_t)i; }
    }
    return (int16_t)(maxIndex - (ORC_TU - 1536) / 2);
}

/* get_snr (ofdm-decoder.cpp:212-230) of a T_u spectrum, sums in bin order as the
 * reference; get_db(x) = 20 log10((x + 1) / 256) in float (dab-constants.h:107-109) */
static float get_db(float x) { return 20 * log10f((x + 1) / (float)256); }
int16_t orc_get_snr(const float *X) {
    const int low = ORC_TU / 2 - ORC_K / 2, high = low + ORC_K;
    float noise = 0, signal = 0;
    for (int i = 10; i < low - 20; i++) { cf z = {X[2 * ((ORC_TU / 2 + i) % ORC_TU)], X[2 * ((ORC_TU / 2 + i) % ORC_TU) + 1]}; noise += cabs_f(z); }
    for (int i = high + 20; i < ORC_TU - 10; i++) { cf z = {X[2 * ((ORC_TU / 2 + i) % ORC_TU)], X[2 * ((ORC_TU / 2 + i) % ORC_TU) + 1]}; noise += cabs_f(z); }
    noise /= (low - 30 + ORC_TU - high - 30);
    for (int i = ORC_TU / 2 - ORC_K / 4; i < ORC_TU / 2 + ORC_K / 4; i++) { cf z = {X[2 * ((ORC_TU / 2 + i) % ORC_TU)], X[2 * ((ORC_TU / 2 + i) % ORC_TU) + 1]}; signal += cabs_f(z); }
    return (int16_t)(get_db(signal / (ORC_K / 2)) - get_db(noise));
}

static inline float arg_pair(const float *X, int a, int b) {
    cf x = {X[2 * (a % ORC_TU)], X[2 * (a % ORC_TU) + 1]}, y = {X[2 * (b % ORC_TU)], X[2 * (b % ORC_TU) + 1]};
    return carg_f(cmul_conjf(x, y));
}

static int16_t process_block0_(const float *v, float *phase_ref, int flag, int method, orc_fft_fn fft) {
    tables_init();
    float X[2 * ORC_TU];
    fft(v, X, 0);
    if (phase_ref) memcpy(phase_ref, X, sizeof X);
    if (!flag) return 0;
    if (method == 0) return get_middle(X);
    if (method == 1) {
        float corr[72 + 18];
        for (int i = 0; i < 72 + 18; i++) {
            int base = ORC_TU - 36 + i;
            corr[i] = arg_pair(X, base, base + 1);
        }
        float MMax = 0;
        int16_t index_1 = 100;
        for (int i = 0; i < 72; i++) {
            float sum = 0;
            for (int j = 1; j < 18; j++) sum += fabsf(g_refarg[j] * corr[i + j]);
            if (sum > MMax) { MMax = sum; index_1 = (int16_t)i; }
        }
        return (int16_t)(ORC_TU - 36 + index_1 - ORC_TU);
    }
    float Mmin = 1000;
    int16_t index_1 = 100;
    for (int i = ORC_TU - 36; i < ORC_TU + 36; i++) {
        float a1 = (float)fabs(fabs(arg_pair(X, i + 1, i + 2) / M_PI) - 1);
        float a2 = (float)fabs(fabs(arg_pair(X, i + 2, i + 3) / M_PI) - 1);
        float a3 = fabsf(arg_pair(X, i + 3, i + 4));
        float a4 = fabsf(arg_pair(X, i + 4, i + 5));
        float a5 = fabsf(arg_pair(X, i + 5, i + 6));
        float b1 = (float)fabs(fabs(arg_pair(X, i + 17, i + 19) / M_PI) - 1);
        float b2 = fabsf(arg_pair(X, i + 19, i + 20));
        float b3 = fabsf(arg_pair(X, i + 20, i + 21));
        float b4 = fabsf(arg_pair(X, i + 21, i + 22));
        float sum = a1 + a2 + a3 + a4 + a5 + b1 + b2 + b3 + b4;
        if (sum < Mmin) { Mmin = sum; index_1 = (int16_t)i; }
    }
    return (int16_t)(index_1 - ORC_TU);
}
int16_t orc_process_block0(const float *v, float *phase_ref, int flag, int method) {   /* ofdm-decoder.cpp:85-162 */
    return process_block0_(v, phase_ref, flag, method, orc_fft2048);
}

static void process_token_(const float *v, float *phase_ref, int16_t *ibits, float *softf, float *X, orc_fft_fn fft) {
    fft(v + 2 * ORC_TG, X, 0);
    for (int i = 0; i < ORC_K; i++) {
        int index = g_perm[i];
        if (index < 0) index += ORC_TU;
        cf x = {X[2 * index], X[2 * index + 1]}, p = {phase_ref[2 * index], phase_ref[2 * index + 1]};
        cf r1 = cmul_conjf(x, p);
        phase_ref[2 * index] = x.re; phase_ref[2 * index + 1] = x.im;
        float ab1 = jan_abs(r1);
        float qr = -r1.re / ab1, qi = -r1.im / ab1;
        ibits[i] = (int16_t)((double)qr * 127.0);
        ibits[ORC_K + i] = (int16_t)((double)qi * 127.0);
        if (softf) { softf[i] = qr; softf[ORC_K + i] = qi; }
    }
}
void orc_process_token(const float *v, float *phase_ref, int16_t *ibits, float *softf) {   /* ofdm-decoder.cpp:167-190 */
    tables_init();
    float X[2 * ORC_TU];
    process_token_(v, phase_ref, ibits, softf, X, orc_fft2048);
}
void orc_process_token_fft(const float *v, float *phase_ref, int16_t *ibits, float *softf, int fft_kind) {
    tables_init();
    float X[2 * ORC_TU];
    process_token_(v, phase_ref, ibits, softf, X, fft_of(fft_kind));
}
int16_t orc_process_block0_fft(const float *v, float *phase_ref, int flag, int method, int fft_kind) {
    return process_block0_(v, phase_ref, flag, method, fft_of(fft_kind));
}

void orc_freqcorr(const float *v, double *acc_re, double *acc_im, float *facc) {   /* ofdm-processor.cpp:424-425 */
    for (int i = ORC_TU; i < ORC_TS; i++) {
        cf a = {v[2 * i], v[2 * i + 1]}, b = {v[2 * (i - ORC_TU)], v[2 * (i - ORC_TU) + 1]};
        cf p = cmul_conjf(a, b);
        if (acc_re) { *acc_re += p.re; *acc_im += p.im; }
        if (facc) { facc[0] += p.re; facc[1] += p.im; }
    }
}

/* ---- ofdmProcessor::run restated over an in-memory stream ---- */
typedef struct {
    const float *iq; int64_t n, pos;
    int32_t localPhase; float sLevel;
    /* the spectrum feed (HAVE_SPECTRUM, ofdm-processor.cpp:161-180,220-238): sampleCnt
     * counts the samples of every getSample / getSamples call; at the end of the call that
     * takes it past INPUT_RATE / 7 the first 32768 raw samples read since the previous
     * emission (localBuffer) go to spectrumBuffer */
    int64_t spec_cnt, spec_start;
    orc_display *disp;
} orc_src;

static void spec_tick(orc_src *s, int n) {                          /* ofdm-processor.cpp:170-180,229-238 */
    s->spec_cnt += n;
    if (s->spec_cnt > ORC_INPUT_RATE / 7) {
        if (s->disp && s->disp->n_spec < s->disp->max_spec) s->disp->spec_start[s->disp->n_spec] = s->spec_start;
        if (s->disp) s->disp->n_spec++;
        s->spec_cnt = 0;
        s->spec_start = s->pos;          /* localCounter = 0: the next sample read starts the buffer */
    }
}

static int get_sample_(orc_src *s, int32_t phase, cf *out) {
    if (s->pos >= s->n) return 0;
    cf t = {s->iq[2 * s->pos], s->iq[2 * s->pos + 1]};
    s->pos++;
    s->localPhase -= phase;
    s->localPhase = (s->localPhase + ORC_INPUT_RATE) % ORC_INPUT_RATE;
    cf o = {g_osc[2 * s->localPhase], g_osc[2 * s->localPhase + 1]};
    t = cmulf(t, o);
    s->sLevel = (float)(0.00001 * jan_abs(t) + (1 - 0.00001) * s->sLevel);
    *out = t;
    return 1;
}
static int get_sample(orc_src *s, int32_t phase, cf *out) {        /* ofdm-processor.cpp:133-183 */
    if (!get_sample_(s, phase, out)) return 0;
    spec_tick(s, 1);
    return 1;
}
static int get_samples(orc_src *s, cf *v, int n, int32_t phase) {  /* ofdm-processor.cpp:186-240 */
    for (int i = 0; i < n; i++) if (!get_sample_(s, phase, &v[i])) return 0;
    spec_tick(s, n);
    return 1;
}

/* ofdmProcessor::run's null search with scanMode (ofdm-processor.cpp:259-338): attempts
 * counted at notSynced (:274), reset when a dip is found (:318); a search that gives up
 * after T_F samples emits No_Signal_Found and restarts the count when scanMode and
 * attempts > 5 (:310-315).  Runs over iq[0, n) until the samples run out (the
 * reference's getSample blocks there: *attempts / *no_signal are its state at that
 * point) or the end of a null is found (returns 1, *pos = the sample after it: where
 * SyncOnPhase starts).  coarse + fine = 0. */
int orc_null_scan(const float *iq, int64_t n, int scan, int32_t *attempts, int32_t *no_signal, int64_t *pos) {
    tables_init();
    orc_src s = {iq, n, 0, 0, 0.0f, 0, 0, NULL};
    float *envBuffer = (float *)malloc(sizeof(float) * 32768);
    const int mask = 32768 - 1;
    int idx, ret = 0;
    float cur;
    int32_t counter, att = 0, ns = 0;
    cf smp;
notSynced:
    att++;
    s.sLevel = 0;
    for (int i = 0; i < 20 * ORC_TS; i++) if (!get_sample(&s, 0, &smp)) goto done;
    idx = 0; cur = 0;
    for (int i = 0; i < 50; i++) {
        if (!get_sample(&s, 0, &smp)) goto done;
        envBuffer[idx] = jan_abs(smp); cur += envBuffer[idx]; idx++;
    }
    counter = 0;
    while (cur / 50 > 0.40 * s.sLevel) {
        if (!get_sample(&s, 0, &smp)) goto done;
        envBuffer[idx] = jan_abs(smp);
        cur += envBuffer[idx] - envBuffer[(idx - 50) & mask];
        idx = (idx + 1) & mask;
        if (++counter > ORC_TF) {
            if (scan && att > 5) { ns++; att = 0; }
            goto notSynced;
        }
    }
    att = 0;
    counter = 0;
    while (cur / 50 < 0.75 * s.sLevel) {
        if (!get_sample(&s, 0, &smp)) goto done;
        envBuffer[idx] = cabs_f(smp);
        cur += envBuffer[idx] - envBuffer[(idx - 50) & mask];
        idx = (idx + 1) & mask;
        if (++counter > ORC_TNULL + 50) goto notSynced;
    }
    ret = 1;
done:
    free(envBuffer);
    *attempts = att;
    *no_signal = ns;
    if (pos) *pos = s.pos;
    return ret;
}

static int orc_ofdm_run_(const float *iq, int64_t n, int16_t threshold, int method, int max_frames,
                         orc_frame_info *info, int16_t *softbits, float *envBuffer, cf *buf, orc_display *disp,
                         int fftk);
int orc_ofdm_run_display(const float *iq, int64_t n, int16_t threshold, int method, int max_frames,
                         orc_frame_info *info, int16_t *softbits, orc_display *disp) {
    /* per call (reentrant: tests run the oracle on several streams from threads) */
    float *envBuffer = (float *)malloc(sizeof(float) * 32768);
    cf *buf = (cf *)malloc(sizeof(cf) * ORC_L * ORC_TS);
    if (disp) { disp->n_disp = 0; disp->n_spec = 0; }
    int ret = orc_ofdm_run_(iq, n, threshold, method, max_frames, info, softbits, envBuffer, buf, disp, 0);
    free(envBuffer);
    free(buf);
    return ret;
}
int orc_ofdm_run_fft(const float *iq, int64_t n, int16_t threshold, int method, int max_frames,
                     orc_frame_info *info, int16_t *softbits, int fft_kind) {
    float *envBuffer = (float *)malloc(sizeof(float) * 32768);
    cf *buf = (cf *)malloc(sizeof(cf) * ORC_L * ORC_TS);
    int ret = orc_ofdm_run_(iq, n, threshold, method, max_frames, info, softbits, envBuffer, buf, NULL, fft_kind);
    free(envBuffer);
    free(buf);
    return ret;
}
int orc_ofdm_run(const float *iq, int64_t n, int16_t threshold, int method,
                 int max_frames, orc_frame_info *info, int16_t *softbits) {
    return orc_ofdm_run_display(iq, n, threshold, method, max_frames, info, softbits, NULL);
}

static int orc_ofdm_run_(const float *iq, int64_t n, int16_t threshold, int method, int max_frames,
                         orc_frame_info *info, int16_t *softbits, float *envBuffer, cf *buf, orc_display *disp,
                         int fftk) {
    tables_init();
    orc_src s = {iq, n, 0, 0, 0.0f, 0, 0, disp};
    orc_fft_fn fft = fft_of(fftk);
    int iq_cnt = 0;                      /* processToken's static cnt (ofdm-decoder.cpp:171) */
    const int mask = 32768 - 1;
    float phase_ref[2 * ORC_TU];
    int16_t fine = 0; int32_t coarse = 0; int f2 = 1;
    int16_t prev1 = 1000, prev2 = 999;
    int frames = 0;
    int idx; float cur; int32_t counter;
    cf smp;

notSynced:
    s.sLevel = 0;
    for (int i = 0; i < 20 * ORC_TS; i++) if (!get_sample(&s, 0, &smp)) return frames;
    idx = 0; cur = 0;
    for (int i = 0; i < 50; i++) {
        if (!get_sample(&s, 0, &smp)) return frames;
        envBuffer[idx] = jan_abs(smp); cur += envBuffer[idx]; idx++;
    }
    counter = 0;
    while (cur / 50 > 0.40 * s.sLevel) {                   /* SyncOnNull :298-317 */
        if (!get_sample(&s, coarse + fine, &smp)) return frames;
        envBuffer[idx] = jan_abs(smp);
        cur += envBuffer[idx] - envBuffer[(idx - 50) & mask];
        idx = (idx + 1) & mask;
        if (++counter > ORC_TF) goto notSynced;
    }
    counter = 0;
    while (cur / 50 < 0.75 * s.sLevel) {                   /* SyncOnEndNull :322-338 */
        if (!get_sample(&s, coarse + fine, &smp)) return frames;
        envBuffer[idx] = cabs_f(smp);
        cur += envBuffer[idx] - envBuffer[(idx - 50) & mask];
        idx = (idx + 1) & mask;
        if (++counter > ORC_TNULL + 50) goto notSynced;
    }
    for (;;) {
        /* SyncOnPhase :344-357 */
        int64_t wstart = s.pos;
        int32_t lpw = s.localPhase;
        for (int i = 0; i < ORC_TU; i++)                  /* getSample, one at a time (:346-347) */
            if (!get_sample(&s, coarse + fine, &buf[i])) return frames;
        int32_t startIndex = find_index_((const float *)buf, threshold, NULL, NULL, fft);
        if (startIndex < 0) goto notSynced;
        memmove(buf, &buf[startIndex], (size_t)(ORC_TU - startIndex) * sizeof(cf));
        int bidx = ORC_TU - startIndex;
        /* OFDM_PRS :383-406 */
        if (!get_samples(&s, &buf[bidx], ORC_TU - bidx, coarse + fine)) return frames;
        int16_t correction = process_block0_((const float *)buf, phase_ref, f2, method, fft);
        if (f2) {
            if (correction == 0 && prev1 == 0 && prev2 == 0) f2 = 0;
            else if (correction != 100) {
                coarse += correction * ORC_CARRIER_DIFF;
                if (abs(coarse) > 35000) coarse = 0;
                prev2 = prev1; prev1 = correction;
            }
        }
        /* OFDM_SYMBOLS :414-446 */
        float fc[2] = {0, 0};
        int16_t *dst = (softbits && frames < max_frames) ? softbits + (int64_t)frames * 75 * 2 * ORC_K : NULL;
        int32_t used_coarse = coarse; int16_t used_fine = fine;
        for (int l = 1; l < ORC_L; l++) {
            int16_t ibits[2 * ORC_K];
            if (!get_samples(&s, buf, ORC_TS, coarse + fine)) return frames;
            orc_freqcorr((const float *)buf, NULL, NULL, fc);
            float X[2 * ORC_TU];
            process_token_((const float *)buf, phase_ref, ibits, NULL, X, fft);
            if (dst) memcpy(dst + (l - 1) * 2 * ORC_K, ibits, sizeof ibits);
            /* the IQ display (ofdm-decoder.cpp:192-206): every 8th displayToken (2) the
             * carriers fft_buffer[0, K/2) and [T_u - 1 - K/2, T_u - 1) into iqBuffer */
            if (l == (disp && disp->token ? disp->token : 2) && ++iq_cnt > 7) {
                if (disp && disp->n_disp < disp->max_disp) {
                    float *o = disp->iq_disp + (int64_t)disp->n_disp * 2 * ORC_K;
                    memcpy(o, X, sizeof(float) * ORC_K);
                    memcpy(o + ORC_K, X + 2 * (ORC_TU - 1 - ORC_K / 2), sizeof(float) * ORC_K);
                    disp->disp_frame[disp->n_disp] = frames;
                }
                if (disp) disp->n_disp++;
                iq_cnt = 0;
            }
        }
        cf fcc = {fc[0], fc[1]};
        fine = (int16_t)(fine + 0.1 * carg_f(fcc) / M_PI * (ORC_CARRIER_DIFF / 2));
        if (!get_samples(&s, buf, ORC_TNULL, coarse + fine)) {
            if (frames < max_frames && info) {
                info[frames].window_start = wstart; info[frames].start_index = startIndex;
                info[frames].coarse = used_coarse; info[frames].fine = used_fine;
                info[frames].correction = correction; info[frames].lp_window = lpw;
            }
            return frames + 1;
        }
        if (fine > ORC_CARRIER_DIFF / 2) { coarse += ORC_CARRIER_DIFF; fine -= ORC_CARRIER_DIFF; }
        else if (fine < -ORC_CARRIER_DIFF / 2) { coarse -= ORC_CARRIER_DIFF; fine += ORC_CARRIER_DIFF; }
        if (frames < max_frames && info) {
            info[frames].window_start = wstart; info[frames].start_index = startIndex;
            info[frames].coarse = used_coarse; info[frames].fine = used_fine;
            info[frames].correction = correction; info[frames].lp_window = lpw;
        }
        frames++;
        if (frames >= max_frames) return frames;
    }
}

/* --------------------------------------------------------------- Viterbi */

static int parity8(int x) { x ^= x >> 4; x ^= x >> 2; x ^= x >> 1; return x & 1; }

/* k = 7, rate 1/4, polynomials {0155, 0117, 0123, 0155} (viterbi.cpp:62-63).
 * Soft input x in [-127,127] (punctured = 0) becomes sym = clamp((int16_t)(x+127),0,255)
 * (viterbi.cpp:229-235). Branch metric sum_j sym_j ^ B_j with B in {0,255}
 * (viterbi.cpp:159-164); ACS as FULL_SPIRAL (spiral-no-sse.c:193-223):
 * uint32 metrics, no renormalisation, strict ">" picks the upper
 * predecessor; start metrics 63 except state 0 = 0 (viterbi.cpp:360-371);
 * full chainback from state 0 after nbits+6 steps (viterbi.cpp:333-357). */
void orc_viterbi(const int16_t *in, int nbits, uint8_t *out) {
    static const int polys[4] = {0155, 0117, 0123, 0155};
    uint32_t B[4][32];
    for (int st = 0; st < 32; st++)
        for (int j = 0; j < 4; j++) B[j][st] = parity8((2 * st) & polys[j]) ? 255u : 0u;
    int steps = nbits + 6;
    uint64_t *dec = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)steps);
    uint32_t m[2][64];
    for (int i = 0; i < 64; i++) m[0][i] = 63;
    m[0][0] = 0;
    int cur = 0;
    for (int s = 0; s < steps; s++) {
        uint32_t sym[4];
        for (int j = 0; j < 4; j++) {
            int16_t t = (int16_t)(in[4 * s + j] + 127);   /* int16_t temp: wraps above 32640 */
            if (t < 0) t = 0;
            if (t > 255) t = 255;
            sym[j] = (uint32_t)t;
        }
        uint64_t d = 0;
        uint32_t *X = m[cur], *Y = m[cur ^ 1];
        for (int i = 0; i < 32; i++) {
            uint32_t t = (sym[0] ^ B[0][i]) + (sym[1] ^ B[1][i]) + (sym[2] ^ B[2][i]) + (sym[3] ^ B[3][i]);
            uint32_t m0 = X[i] + t, m1 = X[i + 32] + (1020 - t);
            uint32_t m2 = X[i] + (1020 - t), m3 = X[i + 32] + t;
            int d0 = m0 > m1, d1 = m2 > m3;
            Y[2 * i] = d0 ? m1 : m0;
            Y[2 * i + 1] = d1 ? m3 : m2;
            d |= ((uint64_t)d0 << (2 * i)) | ((uint64_t)d1 << (2 * i + 1));
        }
        dec[s] = d;
        cur ^= 1;
    }
    uint32_t state = 0;
    for (int s = steps - 1; s >= 0; s--) {
        uint32_t bit = (uint32_t)((dec[s] >> state) & 1u);
        if (s < nbits) out[s] = (uint8_t)(state & 1u);
        state = (state >> 1) | (bit << 5);
    }
    free(dec);
}

/* ------------------------------------------------------------------- FIC */

void orc_fic_depuncture(const int16_t *in, int16_t *out) {      /* fic-handler.cpp:254-288 */
    int8_t pi16[32], pi15[32];
    static const uint8_t pix[24] = {1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0};
    orc_pcode(16, pi16); orc_pcode(15, pi15);
    int ic = 0, o = 0;
    for (int b = 0; b < 21; b++)
        for (int k = 0; k < 128; k++) out[o++] = pi16[k % 32] ? in[ic++] : 0;
    for (int b = 0; b < 3; b++)
        for (int k = 0; k < 128; k++) out[o++] = pi15[k % 32] ? in[ic++] : 0;
    for (int k = 0; k < 24; k++) out[o++] = pix[k] ? in[ic++] : 0;
}

int orc_check_crc_bits(uint8_t *in, int16_t size) {             /* dab-constants.h:310-340 */
    static const uint8_t poly[15] = {0,0,0,1,0,0,0,0,0,0,1,0,0,0,0};
    uint8_t b[16];
    memset(b, 1, 16);
    for (int i = size - 16; i < size; i++) in[i] ^= 1;
    for (int i = 0; i < size; i++) {
        if ((b[0] ^ in[i]) == 1) {
            for (int f = 0; f < 15; f++) b[f] = poly[f] ^ b[f + 1];
            b[15] = 1;
        } else {
            memmove(&b[0], &b[1], 15);
            b[15] = 0;
        }
    }
    int sum = 0;
    for (int i = 0; i < 16; i++) sum += b[i];
    return sum == 0;
}

void orc_fic_process(const int16_t *in, uint8_t *bits, uint8_t *crc_ok) {  /* fic-handler.cpp:241-321 */
    int16_t vb[3072 + 24];
    uint8_t prbs[768];
    orc_fic_depuncture(in, vb);
    orc_viterbi(vb, 768, bits);
    orc_prbs(768, prbs);
    for (int i = 0; i < 768; i++) bits[i] ^= prbs[i];
    for (int f = 0; f < 3; f++) crc_ok[f] = (uint8_t)orc_check_crc_bits(bits + 256 * f, 256);
}

/* ------------------------------------------------------------------- MSC */

int orc_msc_depuncture(int uep, int bitRate, int protLevel, const int16_t *in, int16_t *out) {
    int16_t L[4] = {0, 0, 0, 0}, PI[4] = {0, 0, 0, 0};
    int nseg;
    if (uep) { orc_uep_profile(bitRate, protLevel, L, PI); nseg = 4; }   /* deconvolve.cpp:142-237 */
    else { if (!orc_eep_profile(bitRate, protLevel, L, PI)) return -1; nseg = 2; }  /* :325-366 */
    static const uint8_t pix[24] = {1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0};
    int outSize = 24 * bitRate;
    memset(out, 0, sizeof(int16_t) * (size_t)(outSize * 4 + 24));
    int ic = 0, vc = 0;
    for (int sgi = 0; sgi < nseg; sgi++) {
        if (L[sgi] <= 0) continue;
        int8_t pc[32];
        orc_pcode(PI[sgi], pc);
        for (int b = 0; b < L[sgi]; b++)
            for (int j = 0; j < 128; j++) { if (pc[j % 32]) out[vc] = in[ic++]; vc++; }
    }
    for (int j = 0; j < 24; j++) { if (pix[j]) out[vc] = in[ic++]; vc++; }
    return ic;
}

int orc_msc_stream(int uep, int bitRate, int protLevel, int fragmentSize, int ncif,
                   const int16_t *cif_frag, uint8_t *out) {       /* dab-concurrent.cpp:144-193 */
    int nbits = 24 * bitRate;
    int16_t *data = (int16_t *)malloc(sizeof(int16_t) * (size_t)fragmentSize);
    int16_t *vb = (int16_t *)malloc(sizeof(int16_t) * (size_t)(4 * nbits + 24));
    uint8_t *prbs = (uint8_t *)malloc((size_t)nbits);
    orc_prbs(nbits, prbs);
    memset(out, 0, (size_t)ncif * (size_t)nbits);
    for (int c = 0; c < ncif; c++) {
        for (int i = 0; i < fragmentSize; i++) {
            int d = orc_interleave_delay(i);
            data[i] = (c - d >= 0) ? cif_frag[(size_t)(c - d) * fragmentSize + i] : 0;
        }
        if (c <= 15) continue;                                       /* :172-175 warm-up */
        if (orc_msc_depuncture(uep, bitRate, protLevel, data, vb) < 0) { free(data); free(vb); free(prbs); return -1; }
        uint8_t *o = out + (size_t)c * nbits;
        orc_viterbi(vb, nbits, o);
        for (int i = 0; i < nbits; i++) o[i] ^= prbs[i];
    }
    free(data); free(vb); free(prbs);
    return 0;
}

/* ------------------------------------------------------------------ DAB+ */
/* GF(2^8), poly 0435, Reed-Solomon (255,245) fcr 0 prim 1 nroots 10, shortened
 * by 135 (mp4processor.cpp:74; galois.cpp:33-126; reed-solomon.cpp:32-399). */
#define NN 255
#define NROOTS 10
static uint16_t gf_exp[256], gf_log[256];
static uint8_t rs_gen[NROOTS + 1];
static int gf_init_done = 0;
static int modnn(int x) { while (x >= NN) { x -= NN; x = (x >> 8) + (x & NN); } return x; }
static int pow_pw(int a, int n) { return a == 0 ? 0 : (a * n) % NN; }
static void gf_init(void) {
    if (gf_init_done) return;
    gf_log[0] = NN; gf_exp[NN] = 0;
    int sr = 1;
    for (int i = 0; i < NN; i++) {
        gf_log[sr] = (uint16_t)i; gf_exp[i] = (uint16_t)sr;
        sr <<= 1;
        if (sr & 256) sr ^= 0435;
        sr &= NN;
    }
    memset(rs_gen, 0, sizeof rs_gen);
    rs_gen[0] = 1;
    for (int i = 0, root = 0; i < NROOTS; i++, root++) {
        rs_gen[i + 1] = 1;
        for (int j = i; j > 0; j--) {
            if (rs_gen[j]) rs_gen[j] = (uint8_t)(rs_gen[j - 1] ^ gf_exp[modnn(gf_log[rs_gen[j]] + root)]);
            else rs_gen[j] = rs_gen[j - 1];
        }
        rs_gen[0] = (uint8_t)gf_exp[modnn(root + gf_log[rs_gen[0]])];
    }
    for (int i = 0; i <= NROOTS; i++) rs_gen[i] = (uint8_t)gf_log[rs_gen[i]];
    gf_init_done = 1;
}
static uint8_t gmul(uint8_t a, uint8_t b) { return (a == 0 || b == 0) ? 0 : (uint8_t)gf_exp[modnn(gf_log[a] + gf_log[b])]; }
static uint8_t gdiv(uint8_t a, uint8_t b) { return a == 0 ? 0 : (uint8_t)gf_exp[modnn(256 - 1 + gf_log[a] - gf_log[b])]; }

static int rs_decode_full(uint8_t *data) {                          /* reed-solomon.cpp:143-229 */
    uint8_t syn[NROOTS], Lambda[NROOTS + 1], Corr[NROOTS + 1], omega[NROOTS + 1];
    uint8_t roots[NROOTS], locs[NROOTS];
    int syn_error = 0;
    for (int i = 0; i < NROOTS; i++) {                               /* :231-266 */
        uint8_t s = data[0];
        for (int j = 1; j < NN; j++) {
            if (s == 0) s = data[j];
            else s = (uint8_t)(data[j] ^ gf_exp[modnn(gf_log[s] + pow_pw(i, 1))]);
        }
        syn[i] = s; syn_error |= s;
    }
    if (syn_error == 0) return 0;
    /* Berlekamp-Massey :268-318 */
    for (int i = 0; i < NROOTS + 1; i++) Corr[i] = Lambda[i] = 0;
    uint8_t err = syn[0];
    Lambda[0] = 1; Corr[1] = 1;
    int K = 1, Lr = 0;
    while (K <= NROOTS) {
        uint8_t old[NROOTS + 1];
        memcpy(old, Lambda, sizeof old);
        for (int i = 0; i < NROOTS + 1; i++) Lambda[i] ^= gmul(err, Corr[i]);
        if (2 * Lr < K && err != 0) {
            Lr = K - Lr;
            for (int i = 0; i < NROOTS + 1; i++) Corr[i] = gdiv(old[i], err);
        }
        for (int i = NROOTS; i >= 1; i--) Corr[i] = Corr[i - 1];
        Corr[0] = 0;
        if (K < NROOTS) {
            err = syn[K];
            for (int i = 1; i <= K; i++) err ^= gmul(syn[K - i], Lambda[i]);
        }
        K++;
    }
    int deg = 0;
    for (int i = 0; i < NROOTS + 1; i++) { if (Lambda[i]) deg = i; Lambda[i] = (uint8_t)gf_log[Lambda[i]]; }
    /* Chien search :323-360 */
    uint8_t reg[NROOTS + 1];
    memcpy(reg, Lambda, sizeof reg);
    int count = 0;
    for (int i = 1, k = 0; i <= NN; i++, k++) {
        int result = 1;
        for (int j = deg; j > 0; j--)
            if (reg[j] != NN) { reg[j] = (uint8_t)modnn(reg[j] + j); result ^= gf_exp[reg[j]]; }
        if (result != 0) continue;
        if (count < NROOTS) { roots[count] = (uint8_t)i; locs[count] = (uint8_t)k; }
        count++;
    }
    if (count != deg) return -1;
    /* omega :370-399 */
    int deg_omega = 0;
    for (int i = 0; i < NROOTS; i++) {
        int tmp = 0;
        for (int j = (deg < i) ? deg : i; j >= 0; j--)
            if (gf_log[syn[i - j]] != NN && Lambda[j] != NN)
                tmp ^= gf_exp[modnn(gf_log[syn[i - j]] + Lambda[j])];
        if (tmp) deg_omega = i;
        omega[i] = (uint8_t)gf_log[tmp];
    }
    omega[NROOTS] = NN;
    /* Forney :183-227 */
    for (int j = count - 1; j >= 0; j--) {
        int num1 = 0;
        for (int i = deg_omega; i >= 0; i--)
            if (omega[i] != NN) num1 ^= gf_exp[modnn(omega[i] + pow_pw(i, roots[j]))];
        int num2 = gf_exp[modnn(pow_pw(roots[j], modnn(256 - 1 + 0 - 1)) + NN)];
        int den = 0;
        for (int i = ((deg < NROOTS - 1) ? deg : NROOTS - 1) & ~1; i >= 0; i -= 2)
            if (Lambda[i + 1] != NN) den ^= gf_exp[modnn(Lambda[i + 1] + pow_pw(i, roots[j]))];
        if (den == 0) return -1;
        if (num1 != 0) {
            if (locs[j] >= (uint8_t)(NN - NROOTS)) count--;
            else {
                int c = modnn(gf_log[num1] + gf_log[num2]);
                c = modnn(c + (NN - gf_log[den]));
                data[locs[j]] ^= (uint8_t)gf_exp[c];
            }
        }
    }
    return count;
}

int16_t orc_rs_dec(const uint8_t *in, uint8_t *out) {               /* reed-solomon.cpp:129-141, cutlen 135 */
    gf_init();
    uint8_t rf[NN];
    memset(rf, 0, 135);
    for (int i = 135; i < NN; i++) rf[i] = in[i - 135];
    int r = rs_decode_full(rf);
    for (int i = 135; i < NN - NROOTS; i++) out[i - 135] = rf[i];
    return (int16_t)r;
}

void orc_rs_enc(const uint8_t *in, uint8_t *out) {                   /* reed-solomon.cpp:72-126 */
    gf_init();
    uint8_t rf[NN], bb[NROOTS];
    memset(rf, 0, 135);
    for (int i = 135; i < NN; i++) rf[i] = (i < NN - NROOTS) ? in[i - 135] : 0;
    memset(bb, 0, sizeof bb);
    for (int i = 0; i < NN - NROOTS; i++) {
        int fb = gf_log[rf[i] ^ bb[0]];
        if (fb != NN)
            for (int j = 1; j < NROOTS; j++) bb[j] ^= (uint8_t)gf_exp[modnn(fb + rs_gen[NROOTS - j])];
        memmove(&bb[0], &bb[1], NROOTS - 1);
        bb[NROOTS - 1] = (fb != NN) ? (uint8_t)gf_exp[modnn(fb + rs_gen[0])] : 0;
    }
    for (int i = 135; i < NN - NROOTS; i++) out[i - 135] = rf[i];
    for (int i = 0; i < NROOTS; i++) out[NN - 135 - NROOTS + i] = bb[i];
}

/* fire code g(x) = (x^11+1)(x^5+x^3+x^2+x+1) over bytes 2..10 then 0..1
 * (firecode-checker.cpp:31-94) */
int orc_firecode_check(const uint8_t *x) {
    static uint16_t tab[256];
    static int init = 0;
    if (!init) {
        static const uint8_t g[16] = {1,1,1,1,0,1,0,0,0,0,0,1,1,1,1,0};
        uint16_t itab[8];
        for (int i = 0; i < 8; i++) {
            uint8_t regs[16];
            memset(regs, 0, 16);
            regs[8 + i] = 1;
            for (int r = 0; r < 8; r++) {
                uint8_t z = regs[15];
                for (int j = 15; j > 0; j--) regs[j] = regs[j - 1] ^ (z & g[j]);
                regs[0] = z;
            }
            uint16_t v = 0;
            for (int j = 15; j >= 0; j--) v = (uint16_t)((v << 1) | regs[j]);
            itab[i] = v;
        }
        for (int i = 0; i < 256; i++) {
            tab[i] = 0;
            for (int j = 0; j < 8; j++) if (i & (1 << j)) tab[i] ^= itab[j];
        }
        init = 1;
    }
    uint16_t state = (uint16_t)((x[2] << 8) | x[3]);
    for (int i = 4; i < 11; i++) {
        uint16_t is = tab[state >> 8];
        state = (uint16_t)(((is & 0x00ff) ^ x[i]) | ((is ^ state << 8) & 0xff00));
    }
    for (int i = 0; i < 2; i++) {
        uint16_t is = tab[state >> 8];
        state = (uint16_t)(((is & 0x00ff) ^ x[i]) | ((is ^ state << 8) & 0xff00));
    }
    return state == 0;
}

int orc_dabplus_crc(const uint8_t *msg, int16_t len) {            /* mp4processor.cpp:40-61 */
    uint16_t acc = 0xFFFF;
    for (int i = 0; i < len; i++) {
        int16_t data = (int16_t)(msg[i] << 8);
        for (int j = 8; j > 0; j--) {
            if ((data ^ acc) & 0x8000) acc = (uint16_t)(((acc << 1) ^ 0x1021) & 0xFFFF);
            else acc = (uint16_t)((acc << 1) & 0xFFFF);
            data = (int16_t)((data << 1) & 0xFFFF);
        }
    }
    uint16_t crc = (uint16_t)(~((msg[len] << 8) | msg[len + 1]) & 0xFFFF);
    return (crc ^ acc) == 0;
}

int orc_superframe(const uint8_t *frame, int base, int bitRate, uint8_t *out, int16_t *n_corrected,
                   int *num_aus, int16_t *au_start, uint8_t *au_crc) {   /* mp4processor.cpp:146-230 */
    int RS = bitRate / 8;
    int16_t nerr = 0;
    *num_aus = 0;
    for (int j = 0; j < RS; j++) {
        uint8_t rin[120], rout[110];
        for (int k = 0; k < 120; k++) rin[k] = frame[(base + j + k * RS) % (RS * 120)];
        int16_t ler = orc_rs_dec(rin, rout);
        if (ler > 0) nerr = (int16_t)(nerr + ler);
        if (ler < 0) { *n_corrected = nerr; return 0; }
        for (int k = 0; k < 110; k++) out[j + k * RS] = rout[k];
    }
    *n_corrected = nerr;
    int dacRate = (out[2] >> 6) & 1, sbr = (out[2] >> 5) & 1;
    int n;
    switch (2 * dacRate + sbr) {
    default:
    case 0: n = 4; au_start[0] = 8; au_start[1] = (int16_t)(out[3] * 16 + (out[4] >> 4));
        au_start[2] = (int16_t)((out[4] & 0xf) * 256 + out[5]); au_start[3] = (int16_t)(out[6] * 16 + (out[7] >> 4));
        au_start[4] = (int16_t)(110 * RS); break;
    case 1: n = 2; au_start[0] = 5; au_start[1] = (int16_t)(out[3] * 16 + (out[4] >> 4));
        au_start[2] = (int16_t)(110 * RS); break;
    case 2: n = 6; au_start[0] = 11; au_start[1] = (int16_t)(out[3] * 16 + (out[4] >> 4));
        au_start[2] = (int16_t)((out[4] & 0xf) * 256 + out[5]); au_start[3] = (int16_t)(out[6] * 16 + (out[7] >> 4));
        au_start[4] = (int16_t)((out[7] & 0xf) * 256 + out[8]); au_start[5] = (int16_t)(out[9] * 16 + (out[10] >> 4));
        au_start[6] = (int16_t)(110 * RS); break;
    case 3: n = 3; au_start[0] = 6; au_start[1] = (int16_t)(out[3] * 16 + (out[4] >> 4));
        au_start[2] = (int16_t)((out[4] & 0xf) * 256 + out[5]); au_start[3] = (int16_t)(110 * RS); break;
    }
    *num_aus = n;
    for (int i = 0; i < n; i++) {
        au_crc[i] = 0;
        if (au_start[i + 1] < au_start[i]) return 0;
        int len = au_start[i + 1] - au_start[i] - 2;
        if (len >= 960 || len < 0) return 0;
        au_crc[i] = (uint8_t)orc_dabplus_crc(&out[au_start[i]], (int16_t)len);
    }
    return 1;
}

void orc_mp4_init(orc_mp4 *m, int bitRate) {                       /* mp4processor.cpp:71-95 */
    memset(m, 0, sizeof *m);
    m->bitRate = bitRate;
}

int orc_mp4_add(orc_mp4 *m, const uint8_t *bits, uint8_t *out, int16_t *n_corrected, int *num_aus,
                int16_t *au_start, uint8_t *au_crc) {               /* mp4processor.cpp:107-145 */
    const int nbytes = 3 * m->bitRate;                               /* nbits / 8, nbits = 24 * bitRate */
    for (int i = 0; i < nbytes; i++) {
        uint8_t t = 0;
        for (int j = 0; j < 8; j++) t = (uint8_t)((t << 1) | (bits[8 * i + j] & 1));
        m->ring[m->fill * nbytes + i] = t;
    }
    m->blocks++;
    m->fill = (m->fill + 1) % 5;
    *num_aus = 0;
    *n_corrected = 0;
    if (m->blocks < 5) return 0;
    const int base = m->fill * nbytes;
    if (!orc_firecode_check(&m->ring[base])) { m->blocks = 4; return 1; }
    if (orc_superframe(m->ring, base, m->bitRate, out, n_corrected, num_aus, au_start, au_crc)) {
        m->blocks = 0;
        return 3;
    }
    m->blocks = 4;
    return 2;
}

/* build every lazily initialised table once (call before using the oracle from threads) */
void orc_init(void) {
    float x[2 * ORC_TU], y[2 * ORC_TU];
    memset(x, 0, sizeof x);
    tables_init();
    orc_fft2048(x, y, 0);
    gf_init();
    uint8_t b[11] = {0};
    (void)orc_firecode_check(b);
}
