// dabsynth.cpp -- synthetic DAB Mode-I transmitter (see dabsynth.h).
// Input generator for tests/bench; not on the decode path.
#include "dabsynth.h"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <thread>
#include <algorithm>

namespace {

constexpr int TU = 2048, TS = 2552, TG = 504, TNULL = 2656, TF = 196608, K = 1536, L = 76;
constexpr int CIF_BITS = 55296;

// ---------------------------------------------------------------- random
struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0xD1B54A32D192ED03ull) {}
    uint64_t next() {           // splitmix64
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint8_t bit() { return (uint8_t)(next() >> 63); }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    double gauss() {            // Box-Muller
        double u1 = uni(), u2 = uni();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
    }
};

// ---------------------------------------------------------------- tables
// ETSI EN 300 401 Mode-I phase reference: rows of 32 carriers (k_min, i, n)
const int16_t kPhiRows[48][3] = {
    {-768,0,1},{-736,1,2},{-704,2,0},{-672,3,1},{-640,0,3},{-608,1,2},{-576,2,2},{-544,3,3},
    {-512,0,2},{-480,1,1},{-448,2,2},{-416,3,3},{-384,0,1},{-352,1,2},{-320,2,3},{-288,3,3},
    {-256,0,2},{-224,1,2},{-192,2,2},{-160,3,1},{-128,0,1},{ -96,1,3},{ -64,2,1},{ -32,3,2},
    {   1,0,3},{  33,3,1},{  65,2,1},{  97,1,1},{ 129,0,2},{ 161,3,2},{ 193,2,1},{ 225,1,0},
    { 257,0,2},{ 289,3,2},{ 321,2,3},{ 353,1,3},{ 385,0,0},{ 417,3,2},{ 449,2,1},{ 481,1,3},
    { 513,0,3},{ 545,3,3},{ 577,2,3},{ 609,1,0},{ 641,0,3},{ 673,3,0},{ 705,2,1},{ 737,1,1}};
const int8_t kH[4][16] = {
    {0,2,0,0,0,0,1,1,2,0,0,0,2,2,1,1},
    {0,3,2,3,0,1,3,0,2,1,2,3,2,3,3,0},
    {0,0,0,2,0,2,1,3,2,2,0,2,2,0,1,3},
    {0,1,2,1,0,3,3,2,2,3,2,1,2,1,3,2}};

// PRS phase of carrier k in units of pi/2 (0..3)
int prs_quarter(int k) {
    for (auto &r : kPhiRows)
        if (r[0] <= k && k <= r[0] + 31) return (kH[r[1]][(k - r[0]) & 15] + r[2]) & 3;
    return 0;
}

struct Tables {
    int16_t perm[K];          // carrier i -> signed carrier -768..768
    int prs_q8[TU];           // PRS phase in pi/4 units per FFT bin (or -1 unused)
    int8_t pcode[25][32];
    uint8_t prbs[9216 * 4];
    double tw_re[TU / 2], tw_im[TU / 2];
    Tables() {
        int16_t seq[TU]; seq[0] = 0;
        for (int i = 1; i < TU; i++) seq[i] = (int16_t)((13 * seq[i - 1] + 511) % TU);
        int n = 0;
        for (int i = 0; i < TU; i++) {
            int v = seq[i];
            if (v == TU / 2 || v < 256 || v > 256 + K) continue;
            perm[n++] = (int16_t)(v - TU / 2);
        }
        for (int b = 0; b < TU; b++) prs_q8[b] = -1;
        for (int k = 1; k <= K / 2; k++) {
            prs_q8[k] = 2 * prs_quarter(k);
            prs_q8[TU - k] = 2 * prs_quarter(-k);
        }
        static const int order[7] = {4, 2, 6, 1, 5, 3, 7};
        for (int idx = 1; idx <= 24; idx++) {
            int cnt[8], base = 1 + (idx - 1) / 8;
            for (int g = 0; g < 8; g++) cnt[g] = base;
            cnt[0]++;
            for (int e = 0; e < (idx - 1) % 8; e++) cnt[order[e]]++;
            for (int g = 0; g < 8; g++)
                for (int b = 0; b < 4; b++) pcode[idx][4 * g + b] = (int8_t)(b < cnt[g]);
        }
        uint8_t sr[9]; std::memset(sr, 1, 9);
        for (int i = 0; i < (int)sizeof(prbs); i++) {
            uint8_t b = sr[8] ^ sr[4];
            for (int j = 8; j > 0; j--) sr[j] = sr[j - 1];
            sr[0] = b; prbs[i] = b;
        }
        for (int k = 0; k < TU / 2; k++) { tw_re[k] = std::cos(2 * M_PI * k / TU); tw_im[k] = std::sin(2 * M_PI * k / TU); }
    }
};
const Tables &T() { static Tables t; return t; }

// inverse DFT without 1/N: x[n] = sum_k Z[k] e^{+j 2pi kn/N}
void idft2048(const double *zr, const double *zi, double *xr, double *xi) {
    const Tables &t = T();
    for (int n = 0; n < TU; n++) {
        int r = 0, x = n;
        for (int b = 0; b < 11; b++) { r = (r << 1) | (x & 1); x >>= 1; }
        xr[r] = zr[n]; xi[r] = zi[n];
    }
    for (int len = 2; len <= TU; len <<= 1) {
        int half = len >> 1, step = TU / len;
        for (int s = 0; s < TU; s += len)
            for (int j = 0; j < half; j++) {
                double wr = t.tw_re[j * step], wi = t.tw_im[j * step];
                double ar = xr[s + j + half], ai = xi[s + j + half];
                double tr = ar * wr - ai * wi, ti = ar * wi + ai * wr;
                xr[s + j + half] = xr[s + j] - tr; xi[s + j + half] = xi[s + j] - ti;
                xr[s + j] += tr; xi[s + j] += ti;
            }
    }
}

// UEP profiles (ETSI EN 300 401 Table 8): bitRate, level, L1..L4, PI1..PI4
const int16_t kUep[][10] = {
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

int profile(int uep, int br, int pl, int *Ls, int *PIs) {
    if (uep) {
        for (auto &r : kUep)
            if (r[0] == br && r[1] == pl) {
                for (int j = 0; j < 4; j++) { Ls[j] = r[2 + j]; PIs[j] = r[6 + j]; }
                return 4;
            }
        return 0;
    }
    int lvl = pl & 7;
    Ls[2] = Ls[3] = 0;
    if (pl & 0100) {
        switch (lvl) {
        case 1: Ls[0] = 6 * br / 8 - 3; Ls[1] = 3; PIs[0] = 24; PIs[1] = 23; return 2;
        case 2: if (br == 8) { Ls[0] = 5; Ls[1] = 1; PIs[0] = 13; PIs[1] = 12; }
                else { Ls[0] = 2 * br / 8 - 3; Ls[1] = 4 * br / 8 + 3; PIs[0] = 14; PIs[1] = 13; } return 2;
        case 3: Ls[0] = 6 * br / 8 - 3; Ls[1] = 3; PIs[0] = 8; PIs[1] = 7; return 2;
        case 4: Ls[0] = 4 * br / 8 - 3; Ls[1] = 2 * br / 8 + 3; PIs[0] = 3; PIs[1] = 2; return 2;
        }
    } else if (pl & 0200) {
        Ls[0] = 24 * br / 32 - 3; Ls[1] = 3;
        switch (lvl) {
        case 4: PIs[0] = 2; PIs[1] = 1; return 2;
        case 3: PIs[0] = 4; PIs[1] = 3; return 2;
        case 2: PIs[0] = 6; PIs[1] = 5; return 2;
        case 1: PIs[0] = 10; PIs[1] = 9; return 2;
        }
    }
    return 0;
}

const uint8_t kPIX[24] = {1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0,1,1,0,0};

// ----------------------------------------------------------------- GF/RS
struct GF {
    uint16_t exp_[512], log_[256];
    uint8_t gen[11];
    GF() {
        log_[0] = 255;
        int sr = 1;
        for (int i = 0; i < 255; i++) { log_[sr] = (uint16_t)i; exp_[i] = (uint16_t)sr; sr <<= 1; if (sr & 256) sr ^= 0435; sr &= 255; }
        for (int i = 255; i < 512; i++) exp_[i] = exp_[i - 255];
        // g(x) = prod_{i=0}^{9} (x - a^i), coefficients gen[0..10] (gen[10] = 1, monic)
        uint8_t g[11] = {1};
        int deg = 0;
        for (int i = 0; i < 10; i++) {
            uint8_t ng[11] = {0};
            for (int j = 0; j <= deg; j++) {
                ng[j + 1] ^= g[j];                              // x * g
                ng[j] ^= mul(g[j], (uint8_t)exp_[i]);           // a^i * g
            }
            deg++;
            std::memcpy(g, ng, sizeof g);
        }
        std::memcpy(gen, g, sizeof g);
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? (uint8_t)exp_[log_[a] + log_[b]] : 0; }
};
const GF &G() { static GF g; return g; }

// systematic RS(255,245) shortened to (120,110): data d[0..109] at the high-order end
void rs_encode(const uint8_t *d, uint8_t *cw) {
    const GF &gf = G();
    uint8_t rem[10] = {0};                  // remainder of x^10 * m(x) mod g(x)
    for (int i = 0; i < 110; i++) {
        uint8_t fb = d[i] ^ rem[9];
        for (int j = 9; j > 0; j--) rem[j] = rem[j - 1] ^ gf.mul(fb, gf.gen[j]);
        rem[0] = gf.mul(fb, gf.gen[0]);
    }
    std::memcpy(cw, d, 110);
    for (int j = 0; j < 10; j++) cw[110 + j] = rem[9 - j];
}

uint16_t crc_ccitt(const uint8_t *m, int n) {
    uint16_t acc = 0xFFFF;
    for (int i = 0; i < n; i++) {
        acc ^= (uint16_t)(m[i] << 8);
        for (int b = 0; b < 8; b++) acc = (acc & 0x8000) ? (uint16_t)((acc << 1) ^ 0x1021) : (uint16_t)(acc << 1);
    }
    return acc;
}

// fire code parity (g(x) = (x^11+1)(x^5+x^3+x^2+x+1)) computed as the CRC-16
// remainder that makes the receiver's check (bytes 2..10 then 0..1) return 0
uint16_t fire_parity(const uint8_t *x) {
    // polynomial 1+x+x^2+x^3+x^5+x^11+x^12+x^13+x^14+x^16 -> 0x782F (without x^16)
    uint16_t st = 0;
    auto feed = [&](uint8_t byte) {
        for (int b = 7; b >= 0; b--) {
            int in = (byte >> b) & 1, top = (st >> 15) & 1;
            st = (uint16_t)(st << 1);
            if (in ^ top) st ^= 0x782F;
        }
    };
    for (int i = 2; i < 11; i++) feed(x[i]);
    return st;
}

static const int kAuCount[4] = {4, 2, 6, 3}, kAuFirst[4] = {8, 5, 11, 6};
// an even split of a superframe into layout's AUs passes the reference's checks
// (mp4processor.cpp:197-205: length < 960; start addresses fit 12 bits)
static bool superframe_layout_ok(int rsdims, int layout) {
    const int n = 110 * rsdims, nau = kAuCount[layout], first = kAuFirst[layout], span = n - first;
    return span / nau + 1 < 960 - 2 && first + span * (nau - 1) / nau < 4096;
}

// one DAB+ superframe of rsdims RS columns; layout = 2 * dacRate + sbr: 4, 2, 6 or 3
// access units whose start addresses the header carries (12 bits each after byte 3,
// the first one implicit: mp4processor.cpp:163-195)
void make_superframe(Rng &rng, int rsdims, uint8_t *sf /*[120*rsdims]*/, int layout = 0) {
    int n = 110 * rsdims;
    std::vector<uint8_t> d(n);
    for (auto &b : d) b = (uint8_t)rng.next();
    const int nau = kAuCount[layout & 3], first = kAuFirst[layout & 3];
    d[2] = (uint8_t)((d[2] & 0x80) | ((layout & 3) << 5));   // dacRate, sbr; ch=0 ps=0 surround=0
    int au[7];
    au[0] = first;
    au[nau] = n;
    const int span = n - first;
    for (int i = 1; i < nau; i++) au[i] = first + span * i / nau;
    for (int i = 1; i < nau; i++) {                   // 12-bit start addresses, MSB first from byte 3
        const int bit = 24 + 12 * (i - 1);
        for (int b = 0; b < 12; b++) {
            const int pos = bit + b, v = (au[i] >> (11 - b)) & 1;
            d[pos >> 3] = (uint8_t)((d[pos >> 3] & ~(0x80 >> (pos & 7))) | (v << (7 - (pos & 7))));
        }
    }
    for (int i = 0; i < nau; i++) {
        int len = au[i + 1] - au[i] - 2;
        uint16_t c = (uint16_t)~crc_ccitt(&d[au[i]], len);
        d[au[i] + len] = (uint8_t)(c >> 8);
        d[au[i] + len + 1] = (uint8_t)(c & 0xff);
    }
    uint16_t fp = fire_parity(d.data());
    d[0] = (uint8_t)(fp >> 8); d[1] = (uint8_t)(fp & 0xff);
    std::memcpy(sf, d.data(), n);
    for (int j = 0; j < rsdims; j++) {
        uint8_t dat[110], cw[120];
        for (int k = 0; k < 110; k++) dat[k] = d[j + k * rsdims];
        rs_encode(dat, cw);
        for (int t = 0; t < 10; t++) sf[n + j + t * rsdims] = cw[110 + t];
    }
}

// one MPEG-1 layer II frame (24 ms at 48 kHz = 24 * bitRate bits): sync 0xFFF, ID 1,
// layer II, no CRC, the bit-rate index, 48 kHz; payload bytes below 0x80, so runs of
// ones stay shorter than the 12 a receiver syncs on (mp2processor.cpp:594-603)
void make_mp2_frame(Rng &rng, int bitRate, uint8_t *info /*[24 * bitRate] bits*/) {
    static const int rates[15] = {0, 32, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384};
    int idx = 8;
    for (int i = 1; i < 15; i++)
        if (rates[i] == bitRate) idx = i;
    const int nbytes = 3 * bitRate;
    for (int b = 0; b < nbytes; b++) {
        uint8_t v = (uint8_t)(rng.next() & 0x7F);
        if (b == 0) v = 0xFF;
        else if (b == 1) v = 0xFD;                       // sync tail, ID 1, layer II, no CRC
        else if (b == 2) v = (uint8_t)((idx << 4) | 0x04);   // bit rate, 48 kHz, no padding
        else if (b == 3) v = 0x04;
        for (int k = 0; k < 8; k++) info[8 * b + k] = (uint8_t)((v >> (7 - k)) & 1);
    }
}

// packet mode (EN 300 401 5.3.2): per CIF 3 * bitRate bytes of packets (24, 48, 72 or 96
// bytes: length index, continuity, first/last, address, command, useful length, data,
// CRC-16); the packets of address `addr` carry MSC data groups of random length, split
// over packets, with padding packets (address 0) in between now and then
struct PacketState {
    std::vector<uint8_t> group;    // rest of the data group in flight
    bool started = false;          // its first packet went out
    int cont = 0;
};
void make_packet_cif(Rng &rng, PacketState &st, int bitRate, int addr, uint8_t *info) {
    const int nbytes = 3 * bitRate;
    std::vector<uint8_t> out(nbytes, 0);
    int pos = 0;
    while (pos + 24 <= nbytes) {
        int li = (int)(rng.next() % 4);
        while (pos + 24 * (li + 1) > nbytes) li--;
        const int L = 24 * (li + 1), room = L - 5;
        uint8_t *p = &out[pos];
        std::memset(p, 0, L);
        const bool padding = rng.next() % 8 == 0;
        int fl = 0, useful = 0, a = 0;
        if (!padding) {
            if (st.group.empty()) {
                st.group.resize(20 + rng.next() % 300);
                for (auto &b : st.group) b = (uint8_t)rng.next();
                st.started = false;
            }
            useful = std::min<int>(room, (int)st.group.size());
            const bool first = !st.started, last = useful == (int)st.group.size();
            fl = (first ? 2 : 0) | (last ? 1 : 0);
            std::memcpy(p + 3, st.group.data(), useful);
            st.group.erase(st.group.begin(), st.group.begin() + useful);
            st.started = true;
            a = addr;
        }
        p[0] = (uint8_t)((li << 6) | ((st.cont & 3) << 4) | (fl << 2) | ((a >> 8) & 3));
        p[1] = (uint8_t)(a & 0xFF);
        p[2] = (uint8_t)(useful & 0x7F);                  // command flag 0
        st.cont++;
        const uint16_t c = (uint16_t)~crc_ccitt(p, L - 2);
        p[L - 2] = (uint8_t)(c >> 8);
        p[L - 1] = (uint8_t)(c & 0xFF);
        pos += L;
    }
    for (int b = 0; b < nbytes; b++)
        for (int k = 0; k < 8; k++) info[8 * b + k] = (uint8_t)((out[b] >> (7 - k)) & 1);
}

}  // namespace

extern "C" {

void dabsynth_conv_encode(const uint8_t *bits, int nbits, uint8_t *coded) {
    static const int polys[4] = {0155, 0117, 0123, 0155};
    unsigned sr = 0;
    for (int i = 0; i < nbits + 6; i++) {
        unsigned b = (i < nbits) ? (bits[i] & 1u) : 0u;
        sr = ((sr << 1) | b) & 127u;
        for (int j = 0; j < 4; j++) coded[4 * i + j] = (uint8_t)__builtin_parity(sr & (unsigned)polys[j]);
    }
}

int dabsynth_puncture_msc(int uep, int bitRate, int protLevel, const uint8_t *mother, uint8_t *out) {
    int Ls[4], PIs[4];
    int nseg = profile(uep, bitRate, protLevel, Ls, PIs);
    if (!nseg) return -1;
    const Tables &t = T();
    int ic = 0, oc = 0;
    for (int s = 0; s < nseg; s++)
        for (int b = 0; b < Ls[s]; b++)
            for (int j = 0; j < 128; j++, ic++)
                if (t.pcode[PIs[s]][j % 32]) out[oc++] = mother[ic];
    for (int j = 0; j < 24; j++, ic++) if (kPIX[j]) out[oc++] = mother[ic];
    return oc;
}

void dabsynth_puncture_fic(const uint8_t *mother, uint8_t *out) {
    const Tables &t = T();
    int ic = 0, oc = 0;
    for (int b = 0; b < 24; b++)
        for (int j = 0; j < 128; j++, ic++)
            if (t.pcode[b < 21 ? 16 : 15][j % 32]) out[oc++] = mother[ic];
    for (int j = 0; j < 24; j++, ic++) if (kPIX[j]) out[oc++] = mother[ic];
}

// ETSI EN 300 401 table 8 index of a UEP (bit rate, level): rows per bit rate from
// level 5 down (56 kbit/s has no level 1; 320 no 3 and 1; 384 only 5, 3, 1)
static int uep_table_index(int kbps, int level) {
    static const struct { int kbps; int levels[5]; int n; } g[] = {
        {32, {5, 4, 3, 2, 1}, 5}, {48, {5, 4, 3, 2, 1}, 5}, {56, {5, 4, 3, 2, 0}, 4}, {64, {5, 4, 3, 2, 1}, 5},
        {80, {5, 4, 3, 2, 1}, 5}, {96, {5, 4, 3, 2, 1}, 5}, {112, {5, 4, 3, 2, 0}, 4}, {128, {5, 4, 3, 2, 1}, 5},
        {160, {5, 4, 3, 2, 1}, 5}, {192, {5, 4, 3, 2, 1}, 5}, {224, {5, 4, 3, 2, 1}, 5}, {256, {5, 4, 3, 2, 1}, 5},
        {320, {5, 4, 2, 0, 0}, 3}, {384, {5, 3, 1, 0, 0}, 3}};
    int idx = 0;
    for (const auto &r : g)
        for (int k = 0; k < r.n; k++, idx++)
            if (r.kbps == kbps && r.levels[k] == level) return idx;
    return -1;
}

namespace {
struct BitWriter {
    uint8_t *b;
    int pos = 0;
    void put(uint32_t v, int n) {
        for (int i = n - 1; i >= 0; i--, pos++)
            if ((v >> i) & 1) b[pos >> 3] |= (uint8_t)(0x80 >> (pos & 7));
    }
};
}  // namespace

// FIB number n of an ensemble with FIGs (cfg->figs): item n mod (1 + 2 * n_subch)
static void make_fig_fib(const dabsynth_cfg *cfg, int64_t n, uint8_t *fib) {
    uint8_t bytes[32];
    std::memset(bytes, 0, sizeof bytes);
    BitWriter w{bytes};
    const int items = 1 + 2 * cfg->n_subch;
    const int j = (int)(n % items);
    auto label = [&](const char *l) {
        for (int i = 0; i < 16; i++) w.put((uint8_t)l[i], 8);
        w.put(0xFF00, 16);
    };
    if (j == 0) {                                          // FIG 1/0 ensemble label
        w.put(1, 3), w.put(21, 5), w.put(0, 4), w.put(0, 1), w.put(0, 3), w.put(0xE1C3, 16);
        label("SYNTH ENSEMBLE  ");
    } else if (j & 1) {                                    // FIG 1/1 service label
        const int i = (j - 1) / 2;
        char l[17];
        std::snprintf(l, sizeof l, "SERVICE %02d      ", i % 100);
        w.put(1, 3), w.put(21, 5), w.put(0, 4), w.put(0, 1), w.put(1, 3), w.put(0xC000 + i, 16);
        label(l);
    } else {                                               // FIG 0/1 + FIG 0/2
        const int i = j / 2 - 1;
        const dabsynth_subch &sc = cfg->subch[i];
        const int tix = sc.uep ? uep_table_index(sc.bitRate, sc.protLevel) : -1;
        const bool shortform = sc.uep && tix >= 0;
        w.put(0, 3), w.put(shortform ? 4 : 5, 5), w.put(0, 3), w.put(1, 5);
        w.put(i, 6), w.put(sc.startAddr, 10);
        if (shortform) {
            w.put(0, 1), w.put(0, 1), w.put(tix, 6);
        } else {
            w.put(1, 1), w.put((sc.protLevel & 0200) ? 1 : 0, 3), w.put((sc.protLevel & 7) - 1, 2), w.put(sc.length, 10);
        }
        w.put(0, 3), w.put(6, 5), w.put(0, 3), w.put(2, 5);
        w.put(0xC000 + i, 16), w.put(0, 1), w.put(0, 3), w.put(1, 4);
        if (!sc.dabplus && sc.content == DABSYNTH_PACKET) {
            // packet-mode component (TMid 3, SCId 0x400 + i), then FIG 0/3: SCId -> DG flag 0,
            // DSCTy 60 (MOT), sub-channel i, packet address 0x100 + i
            w.put(3, 2), w.put(0x400 + i, 12), w.put(1, 1), w.put(0, 1);
            w.put(0, 3), w.put(6, 5), w.put(0, 3), w.put(3, 5);
            w.put(0x400 + i, 12), w.put(0, 3), w.put(0, 1), w.put(0, 1), w.put(0, 1);
            w.put(60, 6), w.put(i, 6), w.put(0x100 + i, 10);
        } else {
            w.put(0, 2), w.put(sc.dabplus ? 63 : 0, 6), w.put(i, 6), w.put(1, 1), w.put(0, 1);
        }
    }
    for (int k = (w.pos + 7) >> 3; k < 30; k++) bytes[k] = 0xFF;    // end marker / padding
    const uint16_t c = (uint16_t)~crc_ccitt(bytes, 30);
    bytes[30] = (uint8_t)(c >> 8);
    bytes[31] = (uint8_t)(c & 0xff);
    for (int i = 0; i < 256; i++) fib[i] = (uint8_t)((bytes[i >> 3] >> (7 - (i & 7))) & 1);
}

void dabsynth_make_fib(uint64_t *st, uint8_t *fib) {
    Rng rng(*st);
    uint8_t bytes[32];
    for (int i = 0; i < 30; i++) bytes[i] = (uint8_t)rng.next();
    uint16_t c = (uint16_t)~crc_ccitt(bytes, 30);
    bytes[30] = (uint8_t)(c >> 8); bytes[31] = (uint8_t)(c & 0xff);
    for (int i = 0; i < 256; i++) fib[i] = (uint8_t)((bytes[i >> 3] >> (7 - (i & 7))) & 1);
    *st = rng.next();
}

void dabsynth_rs_encode(const uint8_t *data, uint8_t *cw) { rs_encode(data, cw); }

int64_t dabsynth_stream_len(const dabsynth_cfg *cfg) {
    return (int64_t)(TF - cfg->pre_offset) + (int64_t)cfg->n_frames * TF + TNULL;
}

// The transmitter.  P == 0: a linear stream of dabsynth_stream_len samples (pre-roll
// frame -1, frames 0..F-1, a closing null; encoder CIFs from -19 so the receiver's
// CIF 16 onwards decodes).  P > 0: one period of a cyclic stream, P frames of TF
// samples starting at frame 0's null: the time interleaver and the DAB+ superframe
// grid wrap around the period, so the period repeated end to end is a valid stream
// everywhere (truth: receiver CIF n decodes encoder CIF (n - 15) mod 4P).
static int gen_core(const dabsynth_cfg *cfg, uint64_t seed, int P, float *iq, uint8_t *fic_bits,
                    uint8_t *msc_bits, uint8_t *coded_bits, int64_t *frame0_start) {
    const Tables &t = T();
    const bool cyc = P > 0;
    const int F = cyc ? P : cfg->n_frames, NS = cfg->n_subch;
    if (F < 0 || (!cyc && (cfg->pre_offset < 0 || cfg->pre_offset >= TF))) return -1;
    Rng rng(seed);
    int maxbr = 8;
    for (int s = 0; s < NS; s++) maxbr = std::max<int>(maxbr, cfg->subch[s].bitRate);
    // encoder CIFs e in [e0, 4F): slot e - e0
    const int e0 = cyc ? 0 : -19, NE = 4 * F - e0, NC = 4 * F;
    std::vector<std::vector<uint8_t>> enc_frag(NS);      // punctured bits per (e, s)
    std::vector<int> frag_len(NS);
    std::vector<PacketState> pst(NS);
    for (int s = 0; s < NS; s++) {
        const dabsynth_subch &sc = cfg->subch[s];
        int nb = 24 * sc.bitRate;
        if (cyc && sc.dabplus && NC % 5) return -3;      // superframes must tile the period
        if (cyc && !sc.dabplus && sc.content == DABSYNTH_PACKET) return -4;   // groups do not wrap (dabsynth.h)
        frag_len[s] = sc.length * 64;
        enc_frag[s].assign((size_t)NE * frag_len[s], 0);
        std::vector<uint8_t> info(nb), mother(4 * (nb + 6)), punct(std::max<size_t>(frag_len[s], mother.size()));
        int rsdims = sc.bitRate / 8;
        std::vector<uint8_t> sf(120 * std::max(rsdims, 1));
        // dabplus = 1 + k: the superframe grid is shifted by k CIFs (k = 1..4 makes the
        // receiver's first five CIFs straddle two superframes)
        const int shift = sc.dabplus > 1 ? (sc.dabplus - 1) % 5 : 0;
        int sf_pos = shift * (nb / 8);
        int sf_count = 0;                                 // superframes made (AU layout cycle)
        // cyclic with a shifted grid: the period's superframes are made on the unshifted
        // grid (CIF u = 0, 5, 10, ... starts one) and encoder CIF e carries grid CIF
        // (e + shift) mod 4P, so the superframe straddling the seam is whole
        std::vector<uint8_t> grid;
        if (cyc && sc.dabplus && shift) {
            const int per = nb / 8;
            grid.resize((size_t)NC * nb);
            int pos = 0;
            for (int u = 0; u < NC; u++)
                for (int byte = 0; byte < per; byte++) {
                    if (pos == 0) {
                        int layout = 0;
                        if (sc.content == DABSYNTH_AU_MIX) {
                            for (int k = 0; k < 4; k++) {
                                const int l = (sf_count + k) & 3;
                                if (superframe_layout_ok(rsdims, l)) { layout = l; break; }
                            }
                            sf_count++;
                        }
                        make_superframe(rng, rsdims, sf.data(), layout);
                    }
                    const uint8_t v = sf[pos];
                    for (int b = 0; b < 8; b++) grid[(size_t)u * nb + 8 * byte + b] = (uint8_t)((v >> (7 - b)) & 1);
                    pos = (pos + 1) % (120 * rsdims);
                }
        }
        for (int e = e0; e < NC; e++) {
            if (!grid.empty()) {
                std::memcpy(info.data(), &grid[(size_t)((e + shift) % NC) * nb], nb);
            } else if (sc.dabplus) {
                // 5 CIFs carry one superframe; superframes start at e = e0 + 5m
                int per = nb / 8;
                for (int byte = 0; byte < per; byte++) {
                    if (sf_pos == 0) {
                        int layout = 0;
                        if (sc.content == DABSYNTH_AU_MIX) {
                            // the next layout (cycling) whose AUs the reference accepts at
                            // this size: each < 960 bytes, 12-bit start addresses
                            for (int k = 0; k < 4; k++) {
                                const int l = (sf_count + k) & 3;
                                if (superframe_layout_ok(rsdims, l)) { layout = l; break; }
                            }
                            sf_count++;
                        }
                        make_superframe(rng, rsdims, sf.data(), layout);
                    }
                    uint8_t v = sf[sf_pos];
                    for (int b = 0; b < 8; b++) info[8 * byte + b] = (uint8_t)((v >> (7 - b)) & 1);
                    sf_pos = (sf_pos + 1) % (120 * rsdims);
                }
            } else if (sc.content == DABSYNTH_MP2) {
                make_mp2_frame(rng, sc.bitRate, info.data());
            } else if (sc.content == DABSYNTH_PACKET) {
                make_packet_cif(rng, pst[s], sc.bitRate, 0x100 + s, info.data());
            } else {
                for (int i = 0; i < nb; i++) info[i] = rng.bit();
            }
            int n = cyc ? (e + 15) % NC : e + 15;           // receiver CIF decoding this
            if (msc_bits && n >= 0 && n < NC)
                for (int i = 0; i < nb; i++)
                    msc_bits[((size_t)n * NS + s) * (24 * maxbr) + i] = info[i];
            std::vector<uint8_t> scr(nb);
            for (int i = 0; i < nb; i++) scr[i] = info[i] ^ t.prbs[i];
            dabsynth_conv_encode(scr.data(), nb, mother.data());
            std::fill(punct.begin(), punct.end(), 0);
            int np = dabsynth_puncture_msc(sc.uep, sc.bitRate, sc.protLevel, mother.data(), punct.data());
            if (np < 0 || np > frag_len[s]) return -2;
            std::memcpy(&enc_frag[s][(size_t)(e - e0) * frag_len[s]], punct.data(), frag_len[s]);
        }
    }
    // linear: the pre-roll frame (index -1) then F frames, then one null; cyclic: F frames
    const int64_t total = cyc ? (int64_t)P * TF : dabsynth_stream_len(cfg);
    const double amp = cfg->amplitude > 0 ? cfg->amplitude : 1.0;
    const double scale = amp / std::sqrt((double)K);
    const bool noisy = cfg->snr_db < 200.0f;
    const double sigma = noisy ? amp * std::pow(10.0, -cfg->snr_db / 20.0) / std::sqrt(2.0) : 0.0;
    const int64_t base = cyc ? -(int64_t)TF : -(int64_t)cfg->pre_offset;   // stream index of frame -1
    if (frame0_start) *frame0_start = base + TF;
    std::vector<uint8_t> symbits(3072);
    std::vector<int> phase(TU);
    std::vector<double> zr(TU), zi(TU), xr(TU), xi(TU);
    uint64_t fib_state = seed ^ 0xF1B0F1B0ull;
    for (int f = cyc ? 0 : -1; f < F; f++) {
        int64_t fstart = base + (int64_t)(f + 1) * TF;
        // FIC: 4 blocks x 3 FIBs -> 9216 punctured bits over symbols 1..3
        std::vector<uint8_t> ficsym(9216);
        for (int blk = 0; blk < 4; blk++) {
            uint8_t fib[768], mother[3096], punct[2304];
            for (int q = 0; q < 3; q++) {
                if (cfg->figs) make_fig_fib(cfg, ((int64_t)(f + (cyc ? 0 : 1)) * 4 + blk) * 3 + q, fib + 256 * q);
                else dabsynth_make_fib(&fib_state, fib + 256 * q);
            }
            if (fic_bits && f >= 0) std::memcpy(&fic_bits[((size_t)f * 4 + blk) * 768], fib, 768);
            for (int i = 0; i < 768; i++) fib[i] ^= t.prbs[i];
            dabsynth_conv_encode(fib, 768, mother);
            dabsynth_puncture_fic(mother, punct);
            std::memcpy(&ficsym[blk * 2304], punct, 2304);
        }
        for (int b = 0; b < TU; b++) phase[b] = t.prs_q8[b];
        for (int l = 0; l < L; l++) {
            if (l >= 1) {
                if (l <= 3) std::memcpy(symbits.data(), &ficsym[(l - 1) * 3072], 3072);
                else {
                    int c = (l - 4) / 18, off = ((l - 4) % 18) * 3072;
                    int m = 4 * f + c;                      // transmitted CIF index
                    for (int i = 0; i < 3072; i++) {
                        int pos = off + i;                  // position in the CIF
                        int cu = pos / 64;
                        uint8_t v = (uint8_t)(rng.next() >> 63);
                        for (int s = 0; s < NS; s++) {
                            const dabsynth_subch &sc = cfg->subch[s];
                            if (cu >= sc.startAddr && cu < sc.startAddr + sc.length) {
                                int j = pos - sc.startAddr * 64;
                                int br = j & 15;
                                int rv = ((br & 1) << 3) | ((br & 2) << 1) | ((br & 4) >> 1) | ((br & 8) >> 3);
                                int d = 15 - rv;            // receiver delay
                                int e = m - (15 - d);
                                if (cyc) e = (e + NC) % NC;
                                v = (e >= e0) ? enc_frag[s][(size_t)(e - e0) * frag_len[s] + j] : 0;
                            }
                        }
                        symbits[i] = v;
                    }
                }
                if (coded_bits && f >= 0) std::memcpy(&coded_bits[((size_t)f * 75 + (l - 1)) * 3072], symbits.data(), 3072);
                for (int i = 0; i < K; i++) {
                    int k = t.perm[i];
                    int bin = k < 0 ? k + TU : k;
                    int a = symbits[i], b = symbits[K + i];
                    int q = (a == 0) ? (b == 0 ? 1 : 7) : (b == 0 ? 3 : 5);   // (1-2a)+j(1-2b) in pi/4 units
                    phase[bin] = (phase[bin] + q) & 7;
                }
            }
            for (int b = 0; b < TU; b++) {
                if (phase[b] < 0) { zr[b] = zi[b] = 0; continue; }
                zr[b] = std::cos(M_PI / 4 * phase[b]);
                zi[b] = std::sin(M_PI / 4 * phase[b]);
            }
            idft2048(zr.data(), zi.data(), xr.data(), xi.data());
            int64_t s0 = fstart + TNULL + (int64_t)l * TS;       // guard start
            for (int n = 0; n < TS; n++) {
                int64_t p = s0 + n;
                if (p < 0 || p >= total) continue;
                int u = (n + TU - TG) % TU;
                iq[2 * p] = (float)(xr[u] * scale);
                iq[2 * p + 1] = (float)(xi[u] * scale);
            }
        }
        for (int n = 0; n < TNULL; n++) {
            int64_t p = fstart + n;
            if (p >= 0 && p < total) iq[2 * p] = iq[2 * p + 1] = 0.0f;
        }
    }
    for (int64_t p = base + (int64_t)(F + 1) * TF; p < total; p++)
        if (p >= 0) iq[2 * p] = iq[2 * p + 1] = 0.0f;
    // the carrier offset's phase restarts with each period: the step falls in frame 0's
    // null symbol, where a receiver's NCO sees no signal
    if (noisy || cfg->cfo_hz != 0.0f) {
        for (int64_t p = 0; p < total; p++) {
            double re = iq[2 * p], im = iq[2 * p + 1];
            if (cfg->cfo_hz != 0.0f) {
                double ph = 2.0 * M_PI * cfg->cfo_hz * (double)p / 2048000.0;
                double c = std::cos(ph), s = std::sin(ph);
                double r2 = re * c - im * s, i2 = re * s + im * c;
                re = r2; im = i2;
            }
            if (noisy) { re += sigma * rng.gauss(); im += sigma * rng.gauss(); }
            iq[2 * p] = (float)re; iq[2 * p + 1] = (float)im;
        }
    }
    return 0;
}

int dabsynth_generate(const dabsynth_cfg *cfg, uint64_t seed, float *iq,
                      uint8_t *fic_bits, uint8_t *msc_bits, uint8_t *coded_bits,
                      int64_t *frame0_start) {
    return gen_core(cfg, seed, 0, iq, fic_bits, msc_bits, coded_bits, frame0_start);
}

int dabsynth_generate_period(const dabsynth_cfg *cfg, uint64_t seed, int period, float *iq,
                             uint8_t *fic_bits, uint8_t *msc_bits) {
    if (period < 4) return -1;
    return gen_core(cfg, seed, period, iq, fic_bits, msc_bits, nullptr, nullptr);
}

int dabsynth_period_many(const dabsynth_cfg *cfg, uint64_t seed0, int period, int n_ens, int n_threads,
                         float *iq) {
    const size_t len = (size_t)period * TF;
    if (n_threads < 1) n_threads = 1;
    std::vector<int> rc(n_ens, 0);
    std::vector<std::thread> pool;
    for (int w = 0; w < n_threads; w++)
        pool.emplace_back([&, w]() {
            for (int e = w; e < n_ens; e += n_threads)
                rc[e] = dabsynth_generate_period(cfg, seed0 + (uint64_t)e, period, iq + (size_t)e * 2 * len,
                                                 nullptr, nullptr);
        });
    for (auto &th : pool) th.join();
    for (int e = 0; e < n_ens; e++) if (rc[e]) return rc[e];
    return 0;
}

int dabsynth_generate_many(const dabsynth_cfg *cfg, uint64_t seed0, int n_ens, int n_threads,
                           float *iq, uint8_t *fic_bits, uint8_t *msc_bits) {
    const int64_t len = dabsynth_stream_len(cfg);
    int maxbr = 8;
    for (int s = 0; s < cfg->n_subch; s++) maxbr = std::max<int>(maxbr, cfg->subch[s].bitRate);
    const size_t fic_sz = (size_t)cfg->n_frames * 4 * 768;
    const size_t msc_sz = (size_t)cfg->n_frames * 4 * cfg->n_subch * 24 * maxbr;
    if (n_threads < 1) n_threads = 1;
    std::vector<int> rc(n_ens, 0);
    std::vector<std::thread> pool;
    for (int w = 0; w < n_threads; w++)
        pool.emplace_back([&, w]() {
            for (int e = w; e < n_ens; e += n_threads)
                rc[e] = dabsynth_generate(cfg, seed0 + (uint64_t)e, iq + (size_t)e * 2 * len,
                                          fic_bits ? fic_bits + e * fic_sz : nullptr,
                                          msc_bits ? msc_bits + e * msc_sz : nullptr, nullptr, nullptr);
        });
    for (auto &th : pool) th.join();
    for (int e = 0; e < n_ens; e++) if (rc[e]) return rc[e];
    return 0;
}

}  // extern "C"
