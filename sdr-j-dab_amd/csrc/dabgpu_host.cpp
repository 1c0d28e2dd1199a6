// dabgpu_host.cpp -- the C ABI (include/dabgpu.h): context, device tables,
// batched operators and the streaming pipeline that replaces
// ofdmProcessor::run + ficHandler + mscHandler for many ensembles at once.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdarg>
#include <string>
#include <functional>
#include <vector>
#include <mutex>
#include <algorithm>
#include "../../include/dabgpu.h"
#include "dab_kernels.h"
#include "stage_layout.h"
#include "dab_tables.h"

using namespace dab;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;
static int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
#define HIPCHK(expr)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return fail(DABGPU_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                                      \
    } while (0)

// ------------------------------------------------------------- host tables
namespace {

constexpr int M = 2048000;


// Mode-I phase reference rows (k_min, i, n), k_max = k_min + 31 (phasetable.cpp:115-166)
const int16_t kPhi[48][3] = {
    {-768,0,1},{-736,1,2},{-704,2,0},{-672,3,1},{-640,0,3},{-608,1,2},{-576,2,2},{-544,3,3},
    {-512,0,2},{-480,1,1},{-448,2,2},{-416,3,3},{-384,0,1},{-352,1,2},{-320,2,3},{-288,3,3},
    {-256,0,2},{-224,1,2},{-192,2,2},{-160,3,1},{-128,0,1},{ -96,1,3},{ -64,2,1},{ -32,3,2},
    {   1,0,3},{  33,3,1},{  65,2,1},{  97,1,1},{ 129,0,2},{ 161,3,2},{ 193,2,1},{ 225,1,0},
    { 257,0,2},{ 289,3,2},{ 321,2,3},{ 353,1,3},{ 385,0,0},{ 417,3,2},{ 449,2,1},{ 481,1,3},
    { 513,0,3},{ 545,3,3},{ 577,2,3},{ 609,1,0},{ 641,0,3},{ 673,3,0},{ 705,2,1},{ 737,1,1}};
const int8_t kHpar[4][16] = {
    {0,2,0,0,0,0,1,1,2,0,0,0,2,2,1,1},
    {0,3,2,3,0,1,3,0,2,1,2,3,2,3,3,0},
    {0,0,0,2,0,2,1,3,2,2,0,2,2,0,1,3},
    {0,1,2,1,0,3,3,2,2,3,2,1,2,1,3,2}};

float get_phi(int k) {                                   // phasetable.cpp:261-274 (float result)
    for (auto &r : kPhi)
        if (r[0] <= k && k <= r[0] + 31) return (float)(M_PI / 2 * (kHpar[r[1]][(k - r[0]) & 15] + r[2]));
    return 0.0f;
}

struct HostTables {
    std::vector<float2> osc;
    std::vector<double2> nco;               // factor tables of the NCO (dab_kernels.h)
    std::vector<uint32_t> prbs_words;
    std::vector<float2> w2048;
    std::vector<int16_t> carrier_bin;
    bool stage_ok = true;
    std::vector<float> refarg;
    std::vector<float2> ref;                // natural order refTable
    std::vector<int16_t> perm;              // carrier -> signed carrier (mapIn)
    HostTables() {
#pragma clang fp contract(off)
        osc.resize(M);
        for (int i = 0; i < M; i++)          // ofdm-processor.cpp:79-81
            osc[i] = make_float2((float)cos(2.0 * M_PI * i / M), (float)sin(2.0 * M_PI * i / M));
        nco.assign(NCO_N, make_double2(0.0, 0.0));
        for (int k = 0; k < 128; k++) nco[NCO_A + k] = make_double2(cos(2.0 * M_PI * k / 128), sin(2.0 * M_PI * k / 128));
        for (int k = 0; k < 125; k++)
            nco[NCO_B + k] = make_double2(cos(2.0 * M_PI * k / 16000), sin(2.0 * M_PI * k / 16000));
        for (int k = 0; k < 128; k++) nco[NCO_C + k] = make_double2(cos(2.0 * M_PI * k / M), sin(2.0 * M_PI * k / M));
        ref.assign(2048, make_float2(0.0f, 0.0f));
        for (int i = 1; i <= 768; i++) {      // phasereference.cpp:42-47
            float phi = get_phi(i);
            ref[i] = make_float2(cosf(phi), sinf(phi));
            phi = get_phi(-i);
            ref[2048 - i] = make_float2(cosf(phi), sinf(phi));
        }
        // mapper.cpp:33-55 (Mode I: V1 = 511, [256, 1792] \ {1024})
        int16_t seq[2048];
        seq[0] = 0;
        for (int i = 1; i < 2048; i++) seq[i] = (int16_t)((13 * seq[i - 1] + 511) % 2048);
        for (int i = 0; i < 2048; i++) {
            int v = seq[i];
            if (v == 1024 || v < 256 || v > 256 + 1536) continue;
            perm.push_back((int16_t)(v - 1024));
        }
        std::vector<int> carrier_of_bin(2048, -1);
        for (int c = 0; c < 1536; c++) { int k = perm[c]; carrier_of_bin[k < 0 ? k + 2048 : k] = c; }
        // k_demod: carrier of each FFT bin [2048], then the soft-bit stage words of the
        // bins [2048] and of the carrier pairs [768] (stage_layout.h)
        carrier_bin.assign(2048 + 2048 + 768, -1);
        for (int b = 0; b < 2048; b++) carrier_bin[b] = (int16_t)carrier_of_bin[b];
        {
            int rank[32] = {};
            std::vector<int> sig(768);
            for (int p = 0; p < 768; p++) sig[p] = 32 * rank[STAGE_COL[p]]++ + STAGE_COL[p];
            for (int r : rank) stage_ok = stage_ok && r == 24;        // a permutation of the 1536 words
            for (int p = 0; p < 768; p++) carrier_bin[4096 + p] = (int16_t)(2 * sig[p]);
            // bin b of thread t is b0(t) + 64 k3 (k_demod.hip bin0_of); one store half-wave
            // = 32 threads of one k3: its dump bins take the banks its carriers leave free
            auto b0 = [](int t) { const int g = t >> 2, tq = t & 3; return (g >> 3) + 8 * (g & 7) + 512 * (((tq & 1) << 1) | (tq >> 1)); };
            for (int h = 0; h < 8; h++)
                for (int k3 = 0; k3 < 8; k3++) {
                    bool used[32] = {};
                    for (int l = 0; l < 32; l++) {
                        const int b = b0(32 * h + l) + 64 * k3, cc = carrier_of_bin[b];
                        if (cc < 0) continue;
                        const int w = 2 * sig[cc >> 1] + (cc & 1);
                        carrier_bin[2048 + b] = (int16_t)w;
                        used[w & 31] = true;
                    }
                    int nb = 0;
                    for (int l = 0; l < 32; l++) {
                        const int b = b0(32 * h + l) + 64 * k3;
                        if (carrier_of_bin[b] >= 0) continue;
                        while (nb < 31 && used[nb]) nb++;
                        used[nb] = true;
                        carrier_bin[2048 + b] = (int16_t)(1536 + nb);
                    }
                }
        }
        w2048.resize(2048);                    // k_demod twiddles
        for (int j = 0; j < 2048; j++) {
            const double ph = -2.0 * M_PI * j / 2048.0;
            w2048[j] = make_float2((float)cos(ph), (float)sin(ph));
        }
        refarg.resize(18);
        for (int i = 0; i < 18; i++) {        // ofdm-decoder.cpp:71-74
            float2 a = ref[(2048 + i) % 2048], b = ref[(2048 + i + 1) % 2048];
            float nb = -b.y;
            float ac = a.x * b.x, bd = a.y * nb, ad = a.x * nb, bc = a.y * b.x;
            float re = ac - bd, im = ad + bc;
            refarg[i] = atan2f(im, re);
        }
        // energy dispersal (fic-handler.cpp:100-108), 32768 bits
        prbs_words.assign(1024, 0u);
        uint8_t sr[9];
        memset(sr, 1, 9);
        for (int i = 0; i < 32768; i++) {
            uint8_t b = sr[8] ^ sr[4];
            for (int j = 8; j > 0; j--) sr[j] = sr[j - 1];
            sr[0] = b;
            if (b) prbs_words[i >> 5] |= 1u << (i & 31);
        }
        // DAB+ tables: GF(2^8) with poly 0435 (galois.cpp:33-63, mp4processor.cpp:74)
        // and the fire-code syndrome table (firecode-checker.cpp:31-74)
        dptab.assign(DP_TAB_BYTES, 0);
        uint8_t *gexp = dptab.data(), *glog = dptab.data() + 256;
        glog[0] = 255;
        gexp[255] = 0;
        for (int i = 0, sr = 1; i < 255; i++) {
            glog[sr] = (uint8_t)i;
            gexp[i] = (uint8_t)sr;
            sr <<= 1;
            if (sr & 256) sr ^= 0435;
            sr &= 255;
        }
        static const uint8_t fg[16] = {1, 1, 1, 1, 0, 1, 0, 0, 0, 0, 0, 1, 1, 1, 1, 0};
        uint16_t itab[8];
        for (int i = 0; i < 8; i++) {
            uint8_t regs[16] = {};
            regs[8 + i] = 1;
            for (int r = 0; r < 8; r++) {
                const uint8_t z = regs[15];
                for (int j = 15; j > 0; j--) regs[j] = regs[j - 1] ^ (z & fg[j]);
                regs[0] = z;
            }
            uint16_t v = 0;
            for (int j = 15; j >= 0; j--) v = (uint16_t)((v << 1) | regs[j]);
            itab[i] = v;
        }
        uint16_t *fire = (uint16_t *)(dptab.data() + 512);
        for (int i = 0; i < 256; i++) {
            uint16_t v = 0;
            for (int j = 0; j < 8; j++) if (i & (1 << j)) v ^= itab[j];
            fire[i] = v;
        }
        uint8_t *mul = dptab.data() + 1024;            // mul[i][s] = s * alpha^i
        for (int i = 0; i < 10; i++)
            for (int v = 0; v < 256; v++) mul[i * 256 + v] = v ? gexp[(glog[v] + i) % 255] : 0;
        uint16_t *crc = (uint16_t *)(dptab.data() + 1024 + 2560);   // CRC-CCITT, msb first
        for (int b = 0; b < 256; b++) {
            uint32_t c = (uint32_t)b << 8;
            for (int k = 0; k < 8; k++) c = (c & 0x8000u) ? ((c << 1) ^ 0x1021u) : (c << 1);
            crc[b] = (uint16_t)(c & 0xFFFFu);
        }
        // x^(8d) mod the CRC polynomial: shifts a partial CRC past d bytes
        uint16_t *pow8 = (uint16_t *)(dptab.data() + 1024 + 2560 + 512);
        pow8[0] = 1;
        for (int d = 1; d < 1024; d++)
            pow8[d] = (uint16_t)(((uint32_t)pow8[d - 1] << 8) ^ crc[pow8[d - 1] >> 8]);
        // FIB CRC (dab-constants.h:310-340) by linearity: the register after 256 bits is
        // the XOR of each 1 bit's contribution (a lone 1 at position i, zeros after) and
        // of the all-ones initial value's (256 zero bits): k_fic_post reduces it over a wave
        uint16_t *fc = (uint16_t *)(dptab.data() + FIBCRC_OFF);
        auto run = [](uint32_t r, int one_at) {
            for (int i = 0; i < 256; i++) {
                const uint32_t top = (r >> 15) & 1u;
                r = (r << 1) & 0xFFFFu;
                if (top ^ (uint32_t)(i == one_at)) r ^= 0x1021u;
            }
            return (uint16_t)r;
        };
        for (int i = 0; i < 256; i++) fc[i] = run(0, i);
        fc[256] = run(0xFFFF, -1);
    }
    std::vector<uint8_t> dptab;             // GF exp[256], log[256], fire uint16[256]
};
const HostTables &host_tables() {
    static HostTables t;
    return t;
}

// depuncturing profile of a subchannel (deconvolve.cpp:142-366)
int make_profile(const dabgpu_subch &s, Profile &p) {
    memset(&p, 0, sizeof p);
    int Ls[4] = {0, 0, 0, 0}, PIs[4] = {0, 0, 0, 0}, nseg = 0;
    const int br = s.bitRate;
    if (s.uepFlag == 0) {
        int idx = -1;
        for (int i = 0; i < kNumUep; i++)
            if (kUepProfiles[i][0] == br && kUepProfiles[i][1] == s.protLevel) { idx = i; break; }
        if (idx < 0) idx = 1;               // deconvolve.cpp:150-153 fallback
        for (int j = 0; j < 4; j++) { Ls[j] = kUepProfiles[idx][2 + j]; PIs[j] = kUepProfiles[idx][6 + j]; }
        nseg = 4;
    } else {
        const int lvl = s.protLevel & 7;
        if (s.protLevel & 0100) {
            switch (lvl) {
            case 1: Ls[0] = 6 * br / 8 - 3; Ls[1] = 3; PIs[0] = 24; PIs[1] = 23; break;
            case 2: if (br == 8) { Ls[0] = 5; Ls[1] = 1; PIs[0] = 13; PIs[1] = 12; }
                    else { Ls[0] = 2 * br / 8 - 3; Ls[1] = 4 * br / 8 + 3; PIs[0] = 14; PIs[1] = 13; } break;
            case 3: Ls[0] = 6 * br / 8 - 3; Ls[1] = 3; PIs[0] = 8; PIs[1] = 7; break;
            case 4: Ls[0] = 4 * br / 8 - 3; Ls[1] = 2 * br / 8 + 3; PIs[0] = 3; PIs[1] = 2; break;
            default: return -1;
            }
        } else if (s.protLevel & 0200) {
            Ls[0] = 24 * br / 32 - 3; Ls[1] = 3;
            switch (lvl) {
            case 4: PIs[0] = 2; PIs[1] = 1; break;
            case 3: PIs[0] = 4; PIs[1] = 3; break;
            case 2: PIs[0] = 6; PIs[1] = 5; break;
            case 1: PIs[0] = 10; PIs[1] = 9; break;
            default: return -1;
            }
        } else {
            return -1;                       // protection not defined by the reference
        }
        nseg = 2;
    }
    p.nbits = 24 * br;
    // drop empty segments, keep order
    int ns = 0, blk = 0, in = 0;
    for (int j = 0; j < nseg; j++) {
        if (Ls[j] <= 0) continue;
        uint32_t m = pcode_mask(PIs[j]);
        p.mask[ns] = m;
        p.in_base[ns] = in;
        blk += Ls[j];
        in += Ls[j] * 4 * __builtin_popcount(m);
        p.blk_end[ns] = blk;
        ns++;
    }
    p.nseg = ns;
    p.in_base[ns] = in;
    p.tail_mask = kPiXMask;
    p.frag = in + 12;
    // an unknown UEP (bitRate, level) falls back to row 1 (deconvolve.cpp:150-153): its
    // blocks then cover fewer than 4*nbits mother bits and the rest stays zero
    if (blk * 128 > 4 * p.nbits) return -2;
    return 0;
}

Profile fic_profile() {                      // fic-handler.cpp:254-288
    Profile p;
    memset(&p, 0, sizeof p);
    p.nbits = 768;
    p.nseg = 2;
    p.mask[0] = pcode_mask(16);
    p.mask[1] = pcode_mask(15);
    p.blk_end[0] = 21;
    p.blk_end[1] = 24;
    p.in_base[0] = 0;
    p.in_base[1] = 21 * 4 * 24;
    p.in_base[2] = p.in_base[1] + 3 * 4 * 23;
    p.tail_mask = kPiXMask;
    p.frag = 2304;
    return p;
}

// Inverse depuncturing table of a profile: the mother-code position q = 4 * step + e of
// each punctured input, in input order (the same rule as the kernels' idx4 /
// in_index: PI masks per 128-bit block, then the 24-bit PI_X tail, deconvolve.cpp:172-237),
// stored as its position within the ACS tile holding it (q mod VIT_TILE_POS < 240: one
// byte, and the tile loader scatters with no offset arithmetic)
std::vector<uint8_t> make_inv(const Profile &P) {
    std::vector<uint8_t> inv;
    inv.reserve(P.frag);
    const int last_end = P.nseg ? P.blk_end[P.nseg - 1] : 0;
    for (int q = 0; q < 4 * (P.nbits + 6); q++) {
        const int blk = q >> 7;
        bool keep;
        if (blk < last_end) {
            int k = 0;
            while (blk >= P.blk_end[k]) k++;
            keep = (P.mask[k] >> (q & 31)) & 1u;
        } else {
            const int b = q - 128 * last_end;
            keep = b < 24 && ((P.tail_mask >> b) & 1u);
        }
        if (keep) inv.push_back((uint8_t)(q % VIT_TILE_POS));
    }
    return inv;
}

}  // namespace

// ----------------------------------------------------------------- context
struct dabgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[16] = {};
    float2 *osc = nullptr, *ref = nullptr;
    double2 *nco = nullptr;
    uint32_t *prbs = nullptr;
    float2 *w2048 = nullptr;
    int16_t *carrier_bin = nullptr;
    float *refarg = nullptr;
    uint8_t *dptab = nullptr;    // DAB+ tables (HostTables::dptab)
    uint8_t *fic_inv = nullptr;  // the FIC profile's inverse depuncturing table (make_inv)
    int32_t *err = nullptr;      // device error word (KERR_* bits)
    int32_t *h_err = nullptr;    // its pinned host copy (read after every synchronising pass)
    OfdmTables T{};
    // growable scratch
    void *scratch[8] = {};
    size_t scratch_sz[8] = {};
};

static int scratch(dabgpu_ctx *c, int slot, size_t bytes, void **p) {
    if (c->scratch_sz[slot] < bytes) {
        if (c->scratch[slot]) HIPCHK(hipFree(c->scratch[slot]));
        c->scratch[slot] = nullptr;
        c->scratch_sz[slot] = 0;
        size_t sz = std::max<size_t>(bytes, 4096);
        HIPCHK(hipMalloc(&c->scratch[slot], sz));
        c->scratch_sz[slot] = sz;
    }
    *p = c->scratch[slot];
    return 0;
}
enum { SC_DEC = 0, SC_PROF = 1, SC_I32 = 2, SC_FRAMES = 3, SC_FC = 4, SC_MISC = 5, SC_ACQ = 6 };

// read (and clear) the device error word; call after a stream synchronisation
static int kernel_errors(dabgpu_ctx *c) {
    HIPCHK(hipMemcpyAsync(c->h_err, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const int32_t e = *c->h_err;
    if (!e) return 0;
    HIPCHK(hipMemsetAsync(c->err, 0, sizeof(int32_t), c->stream));
    return fail(DABGPU_E_BOUNDS, "kernel refused out-of-bounds work:%s%s", (e & KERR_FRAME) ? " frame descriptor" : "",
                (e & KERR_VITERBI) ? " viterbi source" : "");
}

template <class T>
static int upload(dabgpu_ctx *c, T **dst, const std::vector<T> &v) {
    HIPCHK(hipMalloc((void **)dst, v.size() * sizeof(T)));
    HIPCHK(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return 0;
}

extern "C" {

int dabgpu_abi_version(void) { return DABGPU_ABI_VERSION; }

int dabgpu_host_table(int which, void *out, size_t bytes) {
    const HostTables &t = host_tables();
    const void *src = nullptr;
    size_t n = 0;
    switch (which) {
    case DABGPU_TABLE_PRS: src = t.ref.data(); n = t.ref.size() * sizeof(float2); break;
    case DABGPU_TABLE_MAPPER: src = t.perm.data(); n = t.perm.size() * sizeof(int16_t); break;
    case DABGPU_TABLE_REFARG: src = t.refarg.data(); n = t.refarg.size() * sizeof(float); break;
    case DABGPU_TABLE_NCO: src = t.nco.data(); n = t.nco.size() * sizeof(double2); break;
    case DABGPU_TABLE_OSC: src = t.osc.data(); n = t.osc.size() * sizeof(float2); break;
    default: return fail(DABGPU_E_ARG, "unknown table %d", which);
    }
    if (!out || bytes < n) return fail(DABGPU_E_ARG, "table %d needs %zu bytes", which, n);
    memcpy(out, src, n);
    return 0;
}

int dabgpu_subch_profile(const dabgpu_subch *s, int32_t *nbits, int32_t *frag, int32_t *nseg, int32_t *L, int32_t *PI) {
    if (!s || !nbits || !frag || !nseg || !L || !PI) return fail(DABGPU_E_ARG, "null arg");
    Profile p;
    if (make_profile(*s, p)) return fail(DABGPU_E_UNSUP, "protection (uep=%d, level 0%o) undefined", s->uepFlag, s->protLevel);
    bool fallback = false;
    if (s->uepFlag == 0) {
        fallback = true;
        for (int i = 0; i < kNumUep; i++)
            if (kUepProfiles[i][0] == s->bitRate && kUepProfiles[i][1] == s->protLevel) fallback = false;
    }
    *nbits = p.nbits;
    *frag = p.frag;
    *nseg = p.nseg;
    for (int k = 0; k < 4; k++) {
        L[k] = k < p.nseg ? p.blk_end[k] - (k ? p.blk_end[k - 1] : 0) : 0;
        PI[k] = k < p.nseg ? __builtin_popcount(p.mask[k]) - 8 : 0;
    }
    return fallback ? 1 : 0;
}
const char *dabgpu_last_error(void) { return g_err.c_str(); }

int dabgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int dabgpu_ctx_create(int device, dabgpu_ctx **out) {
    if (!out) return fail(DABGPU_E_ARG, "out is null");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(DABGPU_E_NODEV, "no HIP device");
    if (device < 0 || device >= n) return fail(DABGPU_E_ARG, "device %d out of range (%d)", device, n);
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(DABGPU_E_NODEV, "device %d is %s, this build targets gfx950", device, prop.gcnArchName);
    HIPCHK(hipSetDevice(device));
    auto *c = new dabgpu_ctx();
    c->device = device;
    // the context stream carries the OFDM front end: highest priority, so a streaming
    // pipeline's next front end takes the SIMDs the Viterbi tail leaves idle
    {
        int least = 0, greatest = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPCHK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest));
    }
    for (auto &e : c->ev) HIPCHK(hipEventCreate(&e));
    const HostTables &t = host_tables();
    if (!t.stage_ok) {
        dabgpu_ctx_destroy(c);
        return fail(DABGPU_E_STATE, "stage_layout.h: STAGE_COL is not 24 pairs per colour");
    }
    int rc = 0;
    if ((rc = upload(c, &c->osc, t.osc)) || (rc = upload(c, &c->nco, t.nco)) || (rc = upload(c, &c->ref, t.ref)) ||
        (rc = upload(c, &c->w2048, t.w2048)) || (rc = upload(c, &c->carrier_bin, t.carrier_bin)) ||
        (rc = upload(c, &c->prbs, t.prbs_words)) ||
        (rc = upload(c, &c->refarg, t.refarg)) || (rc = upload(c, &c->dptab, t.dptab)) ||
        (rc = upload(c, &c->fic_inv, make_inv(fic_profile())))) {
        dabgpu_ctx_destroy(c);
        return rc;
    }
    c->T.osc = c->osc;
    c->T.nco = c->nco;
    c->T.ref = c->ref;
    c->T.w2048 = c->w2048;
    c->T.carrier_of_bin = c->carrier_bin;
    c->T.stage_of_bin = c->carrier_bin + 2048;
    c->T.stage_pair = c->carrier_bin + 4096;
    c->T.refarg = c->refarg;
    if (hipMalloc((void **)&c->err, sizeof(int32_t)) != hipSuccess || hipMemset(c->err, 0, sizeof(int32_t)) != hipSuccess ||
        hipHostMalloc((void **)&c->h_err, sizeof(int32_t), hipHostMallocDefault) != hipSuccess) {
        dabgpu_ctx_destroy(c);
        return fail(DABGPU_E_HIP, "error word alloc");
    }
    c->T.err = c->err;
    *out = c;
    return 0;
}

int dabgpu_ctx_destroy(dabgpu_ctx *c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void *p : {(void *)c->osc, (void *)c->nco, (void *)c->ref, (void *)c->w2048, (void *)c->carrier_bin, (void *)c->prbs,
                    (void *)c->refarg, (void *)c->err, (void *)c->dptab, (void *)c->fic_inv})
        if (p) (void)hipFree(p);
    if (c->h_err) (void)hipHostFree(c->h_err);
    for (auto p : c->scratch) if (p) (void)hipFree(p);
    for (auto e : c->ev) if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

int dabgpu_sync(dabgpu_ctx *c) {
    if (!c) return fail(DABGPU_E_ARG, "null ctx");
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}
int dabgpu_alloc(dabgpu_ctx *c, size_t bytes, void **p) {
    if (!c || !p) return fail(DABGPU_E_ARG, "null arg");
    HIPCHK(hipSetDevice(c->device));
    if (hipMalloc(p, bytes) != hipSuccess) return fail(DABGPU_E_NOMEM, "hipMalloc(%zu) failed", bytes);
    return 0;
}
int dabgpu_free(dabgpu_ctx *c, void *p) {
    if (!c) return fail(DABGPU_E_ARG, "null ctx");
    if (p) HIPCHK(hipFree(p));
    return 0;
}
int dabgpu_memcpy_h2d(dabgpu_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!c) return fail(DABGPU_E_ARG, "null ctx");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}
int dabgpu_memcpy_d2h(dabgpu_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!c) return fail(DABGPU_E_ARG, "null ctx");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}
int dabgpu_host_alloc(dabgpu_ctx *c, size_t bytes, void **h) {
    if (!c || !h) return fail(DABGPU_E_ARG, "bad args");
    *h = nullptr;
    if (!bytes) return 0;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipHostMalloc(h, bytes, hipHostMallocDefault));
    return 0;
}
int dabgpu_host_free(dabgpu_ctx *c, void *h) {
    if (!c) return fail(DABGPU_E_ARG, "bad args");
    if (h) HIPCHK(hipHostFree(h));
    return 0;
}
int dabgpu_memcpy_d2d(dabgpu_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!c) return fail(DABGPU_E_ARG, "null ctx");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
    return 0;
}
int dabgpu_iq_convert(dabgpu_ctx *c, int format, const void *src, int64_t n_pairs, float *iq) {
    if (!c || (!src && n_pairs > 0) || (!iq && n_pairs > 0) || n_pairs < 0) return fail(DABGPU_E_ARG, "bad args");
    if (format != DABGPU_IQ_U8 && format != DABGPU_IQ_S16) return fail(DABGPU_E_ARG, "unknown IQ format %d", format);
    // the vector path reads 16 B per 16 values: the source must be 16-byte aligned
    if (((uintptr_t)src & 15) || ((uintptr_t)iq & 15)) return fail(DABGPU_E_ARG, "IQ buffers must be 16-byte aligned");
    HIPCHK(launch_iq_convert(c->stream, format, src, 2 * n_pairs, iq));
    return 0;
}
int dabgpu_memset_d(dabgpu_ctx *c, void *dst, int value, size_t bytes) {
    if (!c) return fail(DABGPU_E_ARG, "null ctx");
    HIPCHK(hipMemsetAsync(dst, value, bytes, c->stream));
    return 0;
}
int dabgpu_kernel_errors(dabgpu_ctx *c) {
    if (!c) return fail(DABGPU_E_ARG, "null ctx");
    return kernel_errors(c);
}

int dabgpu_event_record(dabgpu_ctx *c, int slot) {
    if (!c || slot < 0 || slot >= 16) return fail(DABGPU_E_ARG, "bad event slot");
    HIPCHK(hipEventRecord(c->ev[slot], c->stream));
    return 0;
}
int dabgpu_event_elapsed(dabgpu_ctx *c, int a, int b, float *ms) {
    if (!c || a < 0 || a >= 16 || b < 0 || b >= 16 || !ms) return fail(DABGPU_E_ARG, "bad event slot");
    HIPCHK(hipEventSynchronize(c->ev[b]));
    HIPCHK(hipEventElapsedTime(ms, c->ev[a], c->ev[b]));
    return 0;
}

// ---- OFDM operators --------------------------------------------------------
int dabgpu_prs_sync(dabgpu_ctx *c, const float *iq, const dabgpu_frame *fr, int n, int16_t level, int32_t *si,
                    float *mx, float *sm) {
    if (!c || !iq || !fr || !si || n < 0) return fail(DABGPU_E_ARG, "bad args");
    HIPCHK(launch_prs_sync(c->stream, iq, DABGPU_IQ_F32, fr, n, c->T, level, si, mx, sm, true));
    return 0;
}
int dabgpu_block0(dabgpu_ctx *c, const float *iq, const dabgpu_frame *fr, int n, int method, int16_t *corr,
                  int16_t *snr) {
    if (!c || !iq || !fr || !corr || n < 0) return fail(DABGPU_E_ARG, "bad args");
    if (method < 0 || method > 2) return fail(DABGPU_E_UNSUP, "freqSyncMethod %d", method);
    HIPCHK(launch_block0(c->stream, iq, DABGPU_IQ_F32, fr, n, c->T, method, corr, snr, true));
    return 0;
}
// symbols 1..75 of a frame are split over `chunks` workgroups of k_demod (each
// recomputes the FFT of the symbol before its first one).  Pick the split whose
// rounds of resident workgroups (kDemodWgPerCu per CU) cost least:
// rounds * (symbols per chunk + 1 warm-up symbol).
static const int kMaxChunks = 25;
#ifndef DEMOD_CHUNK_WG_PER_CU
#define DEMOD_CHUNK_WG_PER_CU 3
#endif
static const int kDemodWgPerCu = DEMOD_CHUNK_WG_PER_CU;
static int num_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        cus = std::max(cus, 1);
    }
    return cus;
}
// extra: FFTs every chunk adds besides its warm-up symbol (2 when it runs findIndex)
static int demod_chunks(int n, int extra = 0) {
    const int cus = num_cus();
    const int64_t slots = (int64_t)kDemodWgPerCu * cus;
    int best = 1;
    double best_cost = 1e30;
    for (int c : {1, 2, 3, 5, 15, 25}) {
        const int64_t items = (int64_t)n * c;
        const double cost = (double)((items + slots - 1) / slots) * ((NSYM + c - 1) / c + 1 + extra);
        if (cost < best_cost - 1e-9) { best_cost = cost; best = c; }
    }
    return best;
}
static int demod_impl(dabgpu_ctx *c, const float *iq, const dabgpu_frame *fr, int n, int16_t *soft, float *softf,
                      float *fc, bool general) {
    void *part = nullptr;
    const int kChunks = demod_chunks(n);
    int rc = scratch(c, SC_FC, sizeof(float2) * (size_t)n * kChunks, &part);
    if (rc) return rc;
    DemodAux aux{};
    HIPCHK(launch_demod(c->stream, iq, fr, n, kChunks, c->T, soft, softf, (float *)part, general, aux));
    if (fc) HIPCHK(launch_fc_reduce(c->stream, (const float *)part, kChunks, n, fc));
    return 0;
}
int dabgpu_ofdm_demod(dabgpu_ctx *c, const float *iq, const dabgpu_frame *fr, int n, int16_t *soft, float *softf,
                      float *fc) {
    if (!c || !iq || !fr || !soft || n < 0) return fail(DABGPU_E_ARG, "bad args");
    return demod_impl(c, iq, fr, n, soft, softf, fc, true);
}
int dabgpu_ofdm_symbol(dabgpu_ctx *c, const float *smp, int kind, float *spec, int16_t *ibits) {
    if (!c || !smp || !spec || (kind != 0 && kind != 1) || (kind == 1 && !ibits)) return fail(DABGPU_E_ARG, "bad args");
    HIPCHK(launch_symbol(c->stream, smp, kind, c->T, spec, ibits));
    return 0;
}
int dabgpu_get_snr(dabgpu_ctx *c, const float *spectrum, int16_t *snr) {
    if (!c || !spectrum || !snr) return fail(DABGPU_E_ARG, "bad args");
    HIPCHK(launch_snr(c->stream, spectrum, snr));
    return 0;
}
int dabgpu_ofdm_demod_mix(dabgpu_ctx *c, const void *iq, int format, const dabgpu_frame *fr, int n, int chunks,
                          int16_t level, int32_t *si, float *mix, float *spec, void *soft) {
    if (!c || !iq || !fr || !mix || !spec || !soft || n < 0 || chunks < 1 || chunks > NSYM) return fail(DABGPU_E_ARG, "bad args");
    if (format != DABGPU_IQ_F32 && format != DABGPU_IQ_S16 && format != DABGPU_IQ_U8) return fail(DABGPU_E_ARG, "format %d", format);
    if (!si && format != DABGPU_IQ_F32) return fail(DABGPU_E_UNSUP, "the operator form reads cf32");
    void *part = nullptr;
    int rc = scratch(c, SC_FC, sizeof(float2) * (size_t)n * chunks, &part);
    if (rc) return rc;
    DemodAux aux{};
    aux.mix = (float2 *)mix;
    aux.spec = (float2 *)spec;
    aux.fmt = format;
    if (si) {                                          // the pipeline's instantiation: findIndex + RING8
        aux.si = si;
        aux.level = level;
        aux.ring8 = 1;
    }
    HIPCHK(launch_demod(c->stream, iq, fr, n, chunks, c->T, (int16_t *)soft, nullptr, (float *)part, true, aux));
    return 0;
}
int dabgpu_nco_eval(dabgpu_ctx *c, int32_t first, int32_t n, float *out) {
    if (!c || !out || first < 0 || n < 0 || (int64_t)first + n > M) return fail(DABGPU_E_ARG, "bad args");
    if (n) HIPCHK(launch_nco_eval(c->stream, c->T, first, n, (float2 *)out));
    return 0;
}
int dabgpu_ofdm_sync_demod(dabgpu_ctx *c, const float *iq, const dabgpu_frame *fr, int n, int16_t level, int32_t *si,
                           int16_t *snr, int16_t *soft, float *softf, float *fc) {
    if (!c || !iq || !fr || !si || !soft || n < 0) return fail(DABGPU_E_ARG, "bad args");
    void *part = nullptr;
    const int kChunks = demod_chunks(n, 2);
    int rc = scratch(c, SC_FC, sizeof(float2) * (size_t)n * kChunks, &part);
    if (rc) return rc;
    DemodAux aux{};
    aux.si = si;
    aux.snr = snr;
    aux.level = level;
    HIPCHK(launch_demod(c->stream, iq, fr, n, kChunks, c->T, soft, softf, (float *)part, true, aux));
    if (fc) HIPCHK(launch_fc_reduce(c->stream, (const float *)part, kChunks, n, fc));
    return 0;
}

// ---- Viterbi operators -------------------------------------------------------
static int run_viterbi(dabgpu_ctx *c, VitJob &J, int max_nbits) {
    void *dec = nullptr;
    int rc = scratch(c, SC_DEC, (size_t)dec_bytes(J.n_cw, max_nbits), &dec);
    if (rc) return rc;
    J.dec = (uint32_t *)dec;
    J.dec_ncw = dec_rows(J.n_cw);
    J.dec_nch = dec_chunks(max_nbits);
    J.prbs_words = c->prbs;
    J.err = c->err;
    HIPCHK(launch_viterbi(c->stream, J));
    return 0;
}

int dabgpu_viterbi(dabgpu_ctx *c, const int16_t *in, int n_cw, int nbits, uint8_t *out) {
    if (!c || !in || !out || n_cw < 0 || nbits <= 0 || nbits > 32768) return fail(DABGPU_E_ARG, "bad args");
    Profile p;
    memset(&p, 0, sizeof p);
    p.nbits = nbits;
    void *pd = nullptr;
    int rc = scratch(c, SC_PROF, sizeof p, &pd);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(pd, &p, sizeof p, hipMemcpyHostToDevice, c->stream));
    VitJob J;
    memset(&J, 0, sizeof J);
    J.kind = SRC_MOTHER;
    J.n_cw = n_cw;
    J.src = in;
    J.src_stride = 4 * (int64_t)(nbits + 6);
    J.src_len = (int64_t)n_cw * J.src_stride;
    J.prof = (const Profile *)pd;
    J.out = out;
    J.out_stride = nbits;
    J.prbs = 0;
    return run_viterbi(c, J, nbits);
}

static int fic_common(dabgpu_ctx *c, VitJob &J, uint8_t *bits, uint8_t *ok) {
    Profile p = fic_profile();
    void *pd = nullptr;
    int rc = scratch(c, SC_PROF, sizeof p, &pd);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(pd, &p, sizeof p, hipMemcpyHostToDevice, c->stream));
    J.prof = (const Profile *)pd;
    J.out = bits;
    J.out_stride = 768;
    J.prbs = 1;
    if ((rc = run_viterbi(c, J, 768))) return rc;
    if (ok) HIPCHK(launch_fic_post(c->stream, bits, ok, 3 * J.n_cw, c->dptab));
    return 0;
}

int dabgpu_fic_decode(dabgpu_ctx *c, const int16_t *soft, int n, uint8_t *bits, uint8_t *ok) {
    if (!c || !soft || !bits || n < 0) return fail(DABGPU_E_ARG, "bad args");
    VitJob J;
    memset(&J, 0, sizeof J);
    J.kind = SRC_FRAG;
    J.n_cw = n;
    J.src = soft;
    J.src_stride = 2304;
    J.src_len = (int64_t)n * 2304;
    return fic_common(c, J, bits, ok);
}

int dabgpu_fic_decode_frames(dabgpu_ctx *c, const int16_t *soft, const int32_t *slots_h, int nf, uint8_t *bits,
                             uint8_t *ok) {
    if (!c || !soft || !slots_h || !bits || nf < 0) return fail(DABGPU_E_ARG, "bad args");
    void *sd = nullptr;
    int rc = scratch(c, SC_I32, sizeof(int32_t) * (size_t)std::max(nf, 1), &sd);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(sd, slots_h, sizeof(int32_t) * nf, hipMemcpyHostToDevice, c->stream));
    VitJob J;
    memset(&J, 0, sizeof J);
    J.kind = SRC_FIC;
    J.n_cw = 4 * nf;
    J.src = soft;
    J.inv = c->fic_inv;
    J.slots = (const int32_t *)sd;
    {
        int32_t mx = 0;
        for (int i = 0; i < nf; i++) {
            if (slots_h[i] < 0) return fail(DABGPU_E_ARG, "negative slot");
            mx = std::max(mx, slots_h[i]);
        }
        J.src_len = (int64_t)(mx + 1) * FRAME_SOFT;
    }
    rc = fic_common(c, J, bits, ok);
    if (rc) return rc;
    return kernel_errors(c);                       // also: slots scratch may be reused by the next call
}

int dabgpu_msc_deconvolve(dabgpu_ctx *c, const int16_t *frag, int64_t frag_stride, const dabgpu_subch *sub,
                          int n_cw, uint8_t *bits, int64_t out_stride) {
    if (!c || !frag || !sub || !bits || n_cw < 0) return fail(DABGPU_E_ARG, "bad args");
    std::vector<Profile> profs;
    std::vector<int32_t> cwp(n_cw);
    int maxbits = 8;
    const int raw = n_cw ? (sub[0].flags & DABGPU_SUBCH_RAW) : 0;
    for (int i = 0; i < n_cw; i++) {
        if ((sub[i].flags & DABGPU_SUBCH_RAW) != raw)
            return fail(DABGPU_E_ARG, "DABGPU_SUBCH_RAW must be the same for every codeword of a call");
        Profile p;
        int rc = make_profile(sub[i], p);
        if (rc) return fail(DABGPU_E_UNSUP, "subchannel %d: protection (uep=%d, level 0%o, %d kbps) undefined",
                            i, sub[i].uepFlag, sub[i].protLevel, sub[i].bitRate);
        if (p.frag > frag_stride) return fail(DABGPU_E_ARG, "fragment stride %lld < %d", (long long)frag_stride, p.frag);
        if (p.nbits > out_stride) return fail(DABGPU_E_ARG, "out stride too small");
        int found = -1;
        for (size_t j = 0; j < profs.size(); j++)
            if (!memcmp(&profs[j], &p, sizeof p)) { found = (int)j; break; }
        if (found < 0) { found = (int)profs.size(); profs.push_back(p); }
        cwp[i] = found;
        maxbits = std::max(maxbits, p.nbits);
    }
    void *pd = nullptr, *cd = nullptr;
    int rc = scratch(c, SC_PROF, sizeof(Profile) * std::max<size_t>(profs.size(), 1), &pd);
    if (rc) return rc;
    if ((rc = scratch(c, SC_I32, sizeof(int32_t) * std::max(n_cw, 1), &cd))) return rc;
    if (!profs.empty()) HIPCHK(hipMemcpyAsync(pd, profs.data(), sizeof(Profile) * profs.size(), hipMemcpyHostToDevice, c->stream));
    if (n_cw) HIPCHK(hipMemcpyAsync(cd, cwp.data(), sizeof(int32_t) * n_cw, hipMemcpyHostToDevice, c->stream));
    VitJob J;
    memset(&J, 0, sizeof J);
    J.kind = SRC_FRAG;
    J.n_cw = n_cw;
    J.src = frag;
    J.src_stride = frag_stride;
    J.src_len = (int64_t)n_cw * frag_stride;
    J.prof = (const Profile *)pd;
    J.cw_prof = (const int32_t *)cd;
    J.out = bits;
    J.out_stride = out_stride;
    J.prbs = raw ? 0 : 1;
    if ((rc = run_viterbi(c, J, maxbits))) return rc;
    return kernel_errors(c);
}

}  // extern "C"

// ========================================================================
// streaming pipeline
// ========================================================================
struct StreamSt {
    int64_t window = 0;      // next SyncOnPhase position
    int32_t lp = 0;          // localPhase before `window`
    int32_t coarse = 0;
    int16_t fine = 0;
    bool f2 = true;
    int16_t prev1 = 1000, prev2 = 999;
    bool synced = false;
    int64_t cif_count = 0;
    int64_t frame_count = 0;
    int32_t last_si = 504;
    int32_t resyncs = 0;
    int32_t attempts = 0;        // ofdmProcessor::run's `attempts` (ofdm-processor.cpp:274-314)
    bool in_attempt = false;     // a null search cut by the end of the samples: `attempts` counts it
    int32_t no_signal = 0;       // No_Signal_Found emissions (scan mode)
    int32_t frames_run = 0;      // frames committed by the last dabgpu_pipe_run
    int32_t acquisitions = 0;    // null-symbol searches completed
};

struct dabgpu_pipe {
    dabgpu_ctx *c = nullptr;
    int S = 0, F = 0, NSUB = 0, R = 0;
    int16_t threshold = 3;
    int16_t method = 1;              // freqSyncMethod
    bool scan = false;               // scanMode (No_Signal_Found after > 5 attempts)
    std::vector<dabgpu_subch> sub;
    std::vector<StreamSt> st;
    uint8_t *ring = nullptr;         // [S][R][75][3072] RING8 bytes (soft bit + 127, dab_kernels.h)
    Profile *prof_d = nullptr;       // [NSUB]
    int32_t *substart_d = nullptr;   // [NSUB]
    dabgpu_frame *frames_d = nullptr;
    int32_t *si_d = nullptr;
    int16_t *corr_d = nullptr, *snr_d = nullptr;
    float *fc_d = nullptr, *fcpart_d = nullptr;
    // the back end's per-run descriptors, one block per back-end stream (parity), uploaded
    // with ONE copy per run (each runtime copy is a kernel of its own on the back-end
    // stream, ~6 us, in front of the ACS): [S] int64 CIF index of each stream's first CIF
    // slot | [S] int32 CIFs each stream delivered | [S * F] int32 FIC ring slots
    uint8_t *desc_d = nullptr;
    size_t desc_sz = 0;
    int64_t *cif0_dev(int par) const { return (int64_t *)(desc_d + par * desc_sz); }
    int32_t *ncif_dev(int par) const { return (int32_t *)(desc_d + par * desc_sz + 8 * (size_t)S); }
    int32_t *slots_dev(int par) const { return (int32_t *)(desc_d + par * desc_sz + 12 * (size_t)S); }
    uint32_t *dec_d[2] = {nullptr, nullptr};   // Viterbi decisions, per back-end stream
    size_t dec_sz = 0;
    int64_t dec_fic_off = 0;                    // FIC decisions: words after the MSC's
    // pinned host staging of the front end's per-pass copies (frame descriptors in,
    // startIndex / FreqCorr out): DMA without the pageable bounce, each pass syncs
    // before the buffers are touched again
    dabgpu_frame *h_frames = nullptr;
    int32_t *h_si = nullptr;
    float2 *h_fc = nullptr;
    int16_t *h_snr = nullptr;
    // pinned staging of the descriptor blocks (desc_d's layout), one per back-end
    // stream; ev_copy[par] marks the upload done before reuse
    uint8_t *h_desc = nullptr;
    int64_t *h_cif0(int par) const { return (int64_t *)(h_desc + par * desc_sz); }
    int32_t *h_ncif(int par) const { return (int32_t *)(h_desc + par * desc_sz + 8 * (size_t)S); }
    int32_t *h_slots(int par) const { return (int32_t *)(h_desc + par * desc_sz + 12 * (size_t)S); }
    hipEvent_t ev_copy[2] = {nullptr, nullptr};
    bool copy_rec[2] = {false, false};
    // the back-end streams' own error words (the front end's is the context's): the
    // Viterbi jobs of run r set berr_d[r & 1], which the back end publishes into
    // h_berr[r & 1] (and clears) as its last step; read once ev_back[r & 1] completed
    int32_t *berr_d = nullptr, *h_berr = nullptr;
    // speculative back end (dabgpu_pipe_run): queued behind the first front pass
    bool speculate = true;                      // env DABGPU_NO_SPECULATE=1: off (A/B)
    // env DABGPU_VIT_SLICES=K (A/B): the MSC Viterbi in K slices -- slice
    // i's ACS on the back-end stream, its traceback on ts behind an event, so it reads
    // decisions the ACS wrote moments before (<= 256 MB per slice: Infinity-Cache resident)
    int vit_slices = 1;
    hipStream_t ts = nullptr;
    std::vector<hipEvent_t> ev_slice;
    hipEvent_t ev_tb = nullptr;
    int64_t front_launches = 0, spec_runs = 0, spec_hits = 0;
    int max_nbits = 0;
    std::vector<dabgpu_frame> last_frames;   // [S][F]
    std::vector<int32_t> last_si;
    std::vector<dabgpu_frame_info> last_info;   // [S][F] observables of the last run
    // DAB+ superframe layer (mp4Processor per DAB+ subchannel and stream)
    int NDP = 0, dp_max_rs = 0;
    // compact superframe output (dabgpu_pipe_set_dabplus_compact): the layer decodes into
    // this sparse scratch and stores the run's superframes in CIF order for the caller
    bool dp_compact = false;
    uint8_t *sf_sparse_d = nullptr;
    size_t sf_sparse_bytes = 0;
    int32_t *dp_sub_d = nullptr;
    int16_t *dp_br_d = nullptr;
    uint8_t *dp_ring_d = nullptr;     // [S][NDP][120*DP_MAX_RS]
    DpState *dp_state_d = nullptr;    // [S][NDP]
    uint8_t *dp_code_d = nullptr;     // [S][NDP][4F] superframe verdict per candidate CIF
    int32_t *dp_cand_d = nullptr;     // [S*NDP*4F + 1] fire-code-passing candidates + count
    const uint8_t *last_msc = nullptr; // MSC bits of the last run
    int32_t last_msc_stride = 0;
    // channel decoding (FIC/MSC Viterbi, DAB+) of run r runs on back-end stream
    // vs[r & 1], so run r's back end overlaps run r+1's front end AND run r+1's back
    // end (whose first waves fill the SIMDs run r's last Viterbi waves leave idle).
    // The ring holds 2F+4 frames per stream so run r+1's demod and MSC never touch a
    // slot run r's MSC still reads; run r+2's front end waits for run r's ACS.
    // The caller gives consecutive runs different output buffers (or syncs).
    hipStream_t vs[2] = {nullptr, nullptr};
    int cur = 0;                                // back-end stream of the last run
    hipEvent_t ev_front = nullptr, ev_back[2] = {nullptr, nullptr}, ev_dp = nullptr;
    bool ev_front_demod = false;     // ev_front marks this pass's demod (the speculative back end's gate)
    bool dp_rec = false;
    bool back_rec[2] = {false, false};
    hipEvent_t ev_acs[2] = {nullptr, nullptr};  // run r's ACS done (the ring's last reader)
    bool acs_rec[2] = {false, false};
    int64_t run_idx = 0;
    Profile *ficprof_d = nullptr;
    uint8_t *inv_d = nullptr;        // the subchannel profiles' inverse depuncturing tables
    // the iqBuffer feed (dabgpu_pipe_set_display): symbol 2's display carriers per ring slot
    float2 *disp_d = nullptr;        // [S][R][K]
    bool display = false;
    bool packed = false;             // MSC output 8 bits per byte (dabgpu_pipe_set_packed)
    bool fic_packed = false;         // FIC output as FIB bytes (DABGPU_PACK_FIC)
    int iq_fmt = DABGPU_IQ_F32;      // sample format of the streams (dabgpu_pipe_set_iq_format)
    int disp_token = 2;              // the display feed's symbol (ofdm-decoder.cpp:61 displayToken)
    // background null search (DABGPU_CTL_ACQ_ASYNC, the default since round 6): a stream
    // that loses sync after an acquisition is searched on its own low-priority stream while
    // the others keep decoding; its results are taken by the first dabgpu_pipe_run after
    // they arrive (set true by dabgpu_pipe_create)
    bool acq_async = false;
    hipStream_t as = nullptr;
    hipEvent_t ev_acq = nullptr;
    AcqJob *acq_jobs_d = nullptr;
    AcqResult *acq_res_d = nullptr, *h_acq = nullptr;   // [S]
    AcqJob *h_acq_jobs = nullptr;                         // [S] pinned staging
    std::vector<int> acq_who;
    std::vector<char> acquiring;                          // [S]
    bool acq_inflight = false;
    // fault injection (DABGPU_CTL_INJECT_BOUNDS): the next run's MSC job gets a subchannel
    // table whose first entry points past the ring, which the Viterbi loader refuses
    bool inject_bounds = false;
    int32_t *substart_bad_d = nullptr;
    bool last_msc_packed = false;
    // optional per-stage kernel timing (HIP events on the stage's stream)
    int profiling = 0;                          // 1: last run, 2: every run since enabled, 3: 2 + stages alone
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, int>> ev_rec;   // (stage, index of start event; end = +1)
    float stage_ms[DABGPU_NSTAGE] = {};
    int32_t stage_n[DABGPU_NSTAGE] = {};
};

static hipError_t prof_mark(dabgpu_pipe *p, int stage, bool start) {
    if (!p->profiling) return hipSuccess;
    hipStream_t st = (stage >= DABGPU_STAGE_FIC) ? p->vs[p->cur] : p->c->stream;
    if (p->profiling == 3) {                    // the stage alone on the device
        hipError_t r = hipDeviceSynchronize();
        if (r != hipSuccess) return r;
    }
    if (start) {
        size_t need = 2 * (p->ev_rec.size() + 1);
        while (p->ev_pool.size() < need) {
            hipEvent_t e;
            hipError_t r = hipEventCreate(&e);
            if (r != hipSuccess) return r;
            p->ev_pool.push_back(e);
        }
        int idx = (int)(2 * p->ev_rec.size());
        p->ev_rec.push_back({stage, idx});
        return hipEventRecord(p->ev_pool[idx], st);
    }
    hipError_t r = hipEventRecord(p->ev_pool[p->ev_rec.back().second + 1], st);
    if (r == hipSuccess && p->profiling == 3) r = hipDeviceSynchronize();
    return r;
}

// errors the back-end streams' kernels raised (refused out-of-bounds Viterbi sources):
// read for every back end known complete -- after a sync (wait) or by a non-blocking
// query -- and reported once
static int back_errors(dabgpu_pipe *p, bool wait) {
    for (int par = 0; par < 2; par++) {
        if (!p->back_rec[par]) continue;
        if (!wait) {
            const hipError_t q = hipEventQuery(p->ev_back[par]);
            if (q == hipErrorNotReady) continue;
            if (q != hipSuccess) return fail(DABGPU_E_HIP, "back-end stream %d: %s", par, hipGetErrorString(q));
        }
        const int32_t e = *(volatile int32_t *)&p->h_berr[par];
        if (e) {
            p->h_berr[par] = 0;
            return fail(DABGPU_E_BOUNDS, "kernel refused out-of-bounds work on back-end stream %d:%s", par,
                        (e & KERR_VITERBI) ? " viterbi source" : " (unknown)");
        }
    }
    return 0;
}

namespace {
inline int32_t modM(int64_t x) {
    int64_t r = x % M;
    return (int32_t)(r < 0 ? r + M : r);
}
// advance localPhase over n samples read with `phase` (getSamples, ofdm-processor.cpp:217-219)
inline int32_t lp_after(int32_t lp, int64_t n, int32_t phase) { return modM((int64_t)lp - n * (int64_t)phase); }
}  // namespace

extern "C" {

int dabgpu_rs_decode(dabgpu_ctx *c, const uint8_t *in, int n, uint8_t *out, int16_t *ret) {
    if (!c || !in || !out || !ret || n < 0) return fail(DABGPU_E_ARG, "bad args");
    HIPCHK(launch_rs(c->stream, in, n, c->dptab, out, ret));
    return 0;
}

// the background null search's stream (lowest priority), event and buffers
static int acq_async_setup(dabgpu_pipe *p) {
    if (p->as) return 0;
    int lo = 0, hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPCHK(hipStreamCreateWithPriority(&p->as, hipStreamNonBlocking, lo));
    HIPCHK(hipEventCreateWithFlags(&p->ev_acq, hipEventDisableTiming));
    HIPCHK(hipMalloc((void **)&p->acq_jobs_d, sizeof(AcqJob) * p->S));
    HIPCHK(hipMalloc((void **)&p->acq_res_d, sizeof(AcqResult) * p->S));
    HIPCHK(hipHostMalloc((void **)&p->h_acq, sizeof(AcqResult) * p->S, hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void **)&p->h_acq_jobs, sizeof(AcqJob) * p->S, hipHostMallocDefault));
    p->acquiring.assign(p->S, 0);
    return 0;
}

int dabgpu_pipe_create(dabgpu_ctx *c, const dabgpu_pipe_cfg *cfg, dabgpu_pipe **out) {
    if (!c || !cfg || !out) return fail(DABGPU_E_ARG, "null arg");
    *out = nullptr;
    if (cfg->n_streams <= 0 || cfg->n_frames <= 0 || cfg->n_subch < 0) return fail(DABGPU_E_ARG, "bad sizes");
    if (cfg->freq_sync_method < 0 || cfg->freq_sync_method > 2)
        return fail(DABGPU_E_UNSUP, "freqSyncMethod %d (0, 1 or 2: ofdm-decoder.cpp:103-161)", cfg->freq_sync_method);
    auto *p = new dabgpu_pipe();
    p->c = c;
    p->S = cfg->n_streams;
    p->F = cfg->n_frames;
    p->NSUB = cfg->n_subch;
    p->R = 2 * cfg->n_frames + 4;
    p->threshold = cfg->threshold;
    p->method = cfg->freq_sync_method;
    p->sub.assign(cfg->subch, cfg->subch + cfg->n_subch);
    p->st.assign(p->S, StreamSt());
    std::vector<Profile> profs(std::max(1, p->NSUB));
    std::vector<int32_t> ss(std::max(1, p->NSUB), 0);
    p->max_nbits = 768;
    for (int i = 0; i < p->NSUB; i++) {
        if (make_profile(p->sub[i], profs[i])) {
            delete p;
            return fail(DABGPU_E_UNSUP, "subchannel %d protection undefined", i);
        }
        if (p->sub[i].startAddr < 0 || p->sub[i].startAddr + p->sub[i].length > 864 || profs[i].frag > p->sub[i].length * 64) {
            delete p;
            return fail(DABGPU_E_ARG, "subchannel %d does not fit its CUs", i);
        }
        ss[i] = p->sub[i].startAddr * 64;
        p->max_nbits = std::max(p->max_nbits, profs[i].nbits);
    }
    std::vector<uint8_t> inv;
    for (int i = 0; i < p->NSUB; i++) {
        profs[i].inv_off = (int32_t)inv.size();
        const std::vector<uint8_t> v = make_inv(profs[i]);
        inv.insert(inv.end(), v.begin(), v.end());
    }
    if (inv.empty()) inv.push_back(0);
    const size_t SF = (size_t)p->S * p->F;
    int rc = 0;
    auto A = [&](void **ptr, size_t bytes) {
        if (rc) return;
        if (hipMalloc(ptr, std::max<size_t>(bytes, 256)) != hipSuccess) rc = fail(DABGPU_E_NOMEM, "pipe alloc %zu", bytes);
    };
    A((void **)&p->ring, (size_t)p->S * p->R * FRAME_SOFT);
    A((void **)&p->prof_d, sizeof(Profile) * profs.size());
    A((void **)&p->substart_d, sizeof(int32_t) * ss.size());
    A((void **)&p->frames_d, sizeof(dabgpu_frame) * SF);
    A((void **)&p->si_d, sizeof(int32_t) * SF);
    A((void **)&p->corr_d, sizeof(int16_t) * SF);
    A((void **)&p->snr_d, sizeof(int16_t) * SF);
    A((void **)&p->fc_d, sizeof(float2) * SF);
    A((void **)&p->fcpart_d, sizeof(float2) * SF * kMaxChunks);
    p->desc_sz = (12 * (size_t)p->S + 4 * (size_t)SF + 15) / 16 * 16;
    if (!rc && (hipHostMalloc((void **)&p->h_frames, sizeof(dabgpu_frame) * SF, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void **)&p->h_si, sizeof(int32_t) * SF, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void **)&p->h_fc, sizeof(float2) * SF, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void **)&p->h_snr, sizeof(int16_t) * SF, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void **)&p->h_desc, 2 * p->desc_sz, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void **)&p->h_berr, sizeof(int32_t) * 2, hipHostMallocDefault) != hipSuccess))
        rc = fail(DABGPU_E_NOMEM, "pipe pinned staging");
    A((void **)&p->berr_d, sizeof(int32_t) * 2);
    if (!rc && (hipMemset(p->berr_d, 0, sizeof(int32_t) * 2) != hipSuccess)) rc = fail(DABGPU_E_HIP, "pipe error words");
    if (!rc) p->h_berr[0] = p->h_berr[1] = 0;
    if (const char *e = getenv("DABGPU_NO_SPECULATE")) p->speculate = !(e[0] == '1');
    if (const char *e = getenv("DABGPU_VIT_SLICES")) p->vit_slices = std::max(1, std::min(64, atoi(e)));
    if (!rc && p->vit_slices > 1) {
        int lo = 0, hi = 0;
        p->ev_slice.assign(p->vit_slices, nullptr);
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
            hipStreamCreateWithPriority(&p->ts, hipStreamNonBlocking, lo) != hipSuccess ||
            hipEventCreateWithFlags(&p->ev_tb, hipEventDisableTiming) != hipSuccess)
            rc = fail(DABGPU_E_HIP, "slice stream");
        for (auto &e : p->ev_slice)
            if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = fail(DABGPU_E_HIP, "slice events");
    }
    A((void **)&p->desc_d, 2 * p->desc_sz);
    // MSC decisions, then the FIC's (both jobs of one run decode in one launch)
    const int64_t msc_words = p->NSUB > 0 ? dec_bytes(SF * 4 * p->NSUB, p->max_nbits) / 4 : 0;
    p->dec_fic_off = msc_words;
    p->dec_sz = (size_t)(4 * msc_words + dec_bytes(SF * 4, 768));
    A((void **)&p->dec_d[0], p->dec_sz);
    A((void **)&p->dec_d[1], p->dec_sz);
    A((void **)&p->ficprof_d, sizeof(Profile));
    A((void **)&p->inv_d, inv.size());
    int prio_least = 0, prio_greatest = 0;
    if (!rc && hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) rc = fail(DABGPU_E_HIP, "priority range");
    if (!rc && (hipStreamCreateWithPriority(&p->vs[0], hipStreamNonBlocking, prio_least) != hipSuccess ||
                hipStreamCreateWithPriority(&p->vs[1], hipStreamNonBlocking, prio_least) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_dp, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_front, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_back[0], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_back[1], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_copy[0], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_acs[0], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_acs[1], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_copy[1], hipEventDisableTiming) != hipSuccess))
        rc = fail(DABGPU_E_HIP, "pipe stream/event create failed");
    if (!rc) {
        const Profile fp = fic_profile();
        if (hipMemcpy(p->ficprof_d, &fp, sizeof fp, hipMemcpyHostToDevice) != hipSuccess)
            rc = fail(DABGPU_E_HIP, "pipe FIC profile upload failed");
    }
    // DAB+ subchannels (mp4Processor: RSDims = bitRate / 8, mp4processor.cpp:83-84)
    std::vector<int32_t> dps;
    std::vector<int16_t> dpb;
    for (int i = 0; i < p->NSUB; i++) {
        if (!(p->sub[i].flags & DABGPU_SUBCH_DABPLUS)) continue;
        const int br = p->sub[i].bitRate;
        if (br < 8 || br % 8 || br / 8 > DP_MAX_RS) {
            dabgpu_pipe_destroy(p);
            return fail(DABGPU_E_UNSUP, "DAB+ subchannel %d: bitRate %d is not a multiple of 8 in [8, 384]", i, br);
        }
        dps.push_back(i);
        dpb.push_back((int16_t)br);
        p->dp_max_rs = std::max(p->dp_max_rs, br / 8);
    }
    p->NDP = (int)dps.size();
    if (p->NDP) {
        A((void **)&p->dp_sub_d, sizeof(int32_t) * dps.size());
        A((void **)&p->dp_br_d, sizeof(int16_t) * dpb.size());
        A((void **)&p->dp_ring_d, (size_t)p->S * p->NDP * 120 * DP_MAX_RS);
        A((void **)&p->dp_state_d, sizeof(DpState) * (size_t)p->S * p->NDP);
        A((void **)&p->dp_code_d, (size_t)p->S * p->NDP * 4 * p->F);
        A((void **)&p->dp_cand_d, sizeof(int32_t) * ((size_t)p->S * p->NDP * 4 * p->F + 1));
        if (!rc && (hipMemcpy(p->dp_sub_d, dps.data(), sizeof(int32_t) * dps.size(), hipMemcpyHostToDevice) != hipSuccess ||
                    hipMemcpy(p->dp_br_d, dpb.data(), sizeof(int16_t) * dpb.size(), hipMemcpyHostToDevice) != hipSuccess ||
                    hipMemset(p->dp_ring_d, 0, (size_t)p->S * p->NDP * 120 * DP_MAX_RS) != hipSuccess ||
                    hipMemset(p->dp_state_d, 0, sizeof(DpState) * (size_t)p->S * p->NDP) != hipSuccess))
            rc = fail(DABGPU_E_HIP, "pipe DAB+ init failed");
    }
    if (!rc) {
        if (hipMemcpy(p->prof_d, profs.data(), sizeof(Profile) * profs.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(p->substart_d, ss.data(), sizeof(int32_t) * ss.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(p->inv_d, inv.data(), inv.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemset(p->ring, RING8_BIAS, (size_t)p->S * p->R * FRAME_SOFT) != hipSuccess)
            rc = fail(DABGPU_E_HIP, "pipe init copy failed");
    }
    // the default re-acquisition mode: a stream that loses sync is searched in the
    // background (DABGPU_CTL_ACQ_ASYNC; DABGPU_CTL_ACQ_SYNC restores the in-run search)
    if (!rc && !(rc = acq_async_setup(p))) p->acq_async = true;
    if (rc) {
        dabgpu_pipe_destroy(p);
        return rc;
    }
    *out = p;
    return 0;
}

int dabgpu_pipe_destroy(dabgpu_pipe *p) {
    if (!p) return 0;
    (void)hipStreamSynchronize(p->c->stream);
    for (hipStream_t v : p->vs) if (v) (void)hipStreamSynchronize(v);
    for (auto e : p->ev_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : {p->ev_front, p->ev_back[0], p->ev_back[1], p->ev_dp, p->ev_copy[0], p->ev_copy[1],
                        p->ev_acs[0], p->ev_acs[1]})
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t v : p->vs) if (v) (void)hipStreamDestroy(v);
    if (p->ts) {
        (void)hipStreamSynchronize(p->ts);
        (void)hipStreamDestroy(p->ts);
    }
    for (hipEvent_t e : p->ev_slice) if (e) (void)hipEventDestroy(e);
    if (p->ev_tb) (void)hipEventDestroy(p->ev_tb);
    if (p->as) {                                    // a background null search still running
        (void)hipStreamSynchronize(p->as);
        (void)hipStreamDestroy(p->as);
    }
    if (p->ev_acq) (void)hipEventDestroy(p->ev_acq);
    for (void *h : {(void *)p->h_acq, (void *)p->h_acq_jobs})
        if (h) (void)hipHostFree(h);
    for (void *x : {(void *)p->acq_jobs_d, (void *)p->acq_res_d})
        if (x) (void)hipFree(x);
    if (p->ficprof_d) (void)hipFree(p->ficprof_d);
    for (void *h : {(void *)p->h_frames, (void *)p->h_si, (void *)p->h_fc, (void *)p->h_snr, (void *)p->h_desc,
                    (void *)p->h_berr})
        if (h) (void)hipHostFree(h);
    if (p->sf_sparse_d) (void)hipFree(p->sf_sparse_d);
    for (void *x : {(void *)p->ring, (void *)p->prof_d, (void *)p->inv_d, (void *)p->substart_d, (void *)p->frames_d, (void *)p->si_d,
                    (void *)p->corr_d, (void *)p->snr_d, (void *)p->fc_d, (void *)p->fcpart_d, (void *)p->desc_d, (void *)p->dec_d[0], (void *)p->dec_d[1],
                    (void *)p->berr_d,
                    (void *)p->dp_sub_d, (void *)p->dp_br_d, (void *)p->dp_ring_d, (void *)p->dp_state_d, (void *)p->dp_code_d,
                    (void *)p->dp_cand_d, (void *)p->disp_d, (void *)p->substart_bad_d})
        if (x) (void)hipFree(x);
    delete p;
    return 0;
}

}  // extern "C"

static AcqJob acq_job(const dabgpu_pipe *p, const StreamSt &x, int s, int64_t stride, const int64_t *n_avail) {
    AcqJob j;
    memset(&j, 0, sizeof j);
    j.iq_base = stride * s;
    j.start = x.window;
    j.end = n_avail[s];
    j.local_phase = x.lp;
    j.phase = x.coarse + x.fine;
    // the kernel enters notSynced (attempts++) first; a cut attempt is repeated whole
    j.attempts = x.attempts - (x.in_attempt ? 1 : 0);
    j.scan = p->scan ? 1 : 0;
    return j;
}
// a search's outcome into the stream state; 1 if it found the end of a null symbol
static int acq_apply(StreamSt &x, const AcqResult &r) {
    x.lp = r.local_phase;
    x.window = r.window;
    x.attempts = r.attempts;
    x.in_attempt = r.status != 0;
    x.no_signal += r.no_signal;
    if (r.status != 0) return 0;
    x.synced = true;
    x.acquisitions++;
    return 1;
}

// Null-symbol search (notSynced .. SyncOnEndNull, ofdm-processor.cpp:274-338) for the
// streams `who` of `cur`, each from its current position (window, localPhase) with
// its correctors: one k_acquire wave per stream.  A stream that finds the end of a
// null symbol is synchronised at SyncOnPhase; one that runs out of samples stays
// unsynchronised at the end of its samples (the next call continues from there).
static int acquire_streams(dabgpu_pipe *p, const void *iq, int64_t stride, const int64_t *n_avail,
                           const std::vector<int> &who, std::vector<StreamSt> &cur, int &found) {
    dabgpu_ctx *c = p->c;
    found = 0;
    if (who.empty()) return 0;
    std::vector<AcqJob> jobs;
    for (int s : who) jobs.push_back(acq_job(p, cur[s], s, stride, n_avail));
    void *jd = nullptr, *rd = nullptr;
    int rc = scratch(c, SC_MISC, sizeof(AcqJob) * jobs.size(), &jd);
    if (rc) return rc;
    if ((rc = scratch(c, SC_ACQ, sizeof(AcqResult) * jobs.size(), &rd))) return rc;
    HIPCHK(hipMemcpyAsync(jd, jobs.data(), sizeof(AcqJob) * jobs.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_acquire(c->stream, iq, p->iq_fmt, (const AcqJob *)jd, (int)jobs.size(), c->osc, (AcqResult *)rd));
    std::vector<AcqResult> res(jobs.size());
    HIPCHK(hipMemcpyAsync(res.data(), rd, sizeof(AcqResult) * jobs.size(), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (size_t i = 0; i < jobs.size(); i++) found += acq_apply(cur[who[i]], res[i]);
    return 0;
}

// Background form (DABGPU_CTL_ACQ_ASYNC): the same search launched on the pipeline's
// acquisition stream without waiting; acq_collect applies the results once they are in.
static int acquire_streams_async(dabgpu_pipe *p, const void *iq, int64_t stride, const int64_t *n_avail,
                                 const std::vector<int> &who, const std::vector<StreamSt> &cur) {
    for (size_t i = 0; i < who.size(); i++) p->h_acq_jobs[i] = acq_job(p, cur[who[i]], who[i], stride, n_avail);
    const size_t n = who.size();
    HIPCHK(hipMemcpyAsync(p->acq_jobs_d, p->h_acq_jobs, sizeof(AcqJob) * n, hipMemcpyHostToDevice, p->as));
    HIPCHK(launch_acquire(p->as, iq, p->iq_fmt, p->acq_jobs_d, (int)n, p->c->osc, p->acq_res_d));
    HIPCHK(hipMemcpyAsync(p->h_acq, p->acq_res_d, sizeof(AcqResult) * n, hipMemcpyDeviceToHost, p->as));
    HIPCHK(hipEventRecord(p->ev_acq, p->as));
    p->acq_who = who;
    for (int s : who) p->acquiring[s] = 1;
    p->acq_inflight = true;
    return 0;
}
static int acq_collect(dabgpu_pipe *p, bool wait) {
    if (!p->acq_inflight) return 0;
    const hipError_t q = wait ? hipEventSynchronize(p->ev_acq) : hipEventQuery(p->ev_acq);
    if (q == hipErrorNotReady) return 0;
    if (q != hipSuccess) return fail(DABGPU_E_HIP, "background null search: %s", hipGetErrorString(q));
    for (size_t i = 0; i < p->acq_who.size(); i++) {
        const int s = p->acq_who[i];
        (void)acq_apply(p->st[s], p->h_acq[i]);
        p->acquiring[s] = 0;
    }
    p->acq_who.clear();
    p->acq_inflight = false;
    return 0;
}

extern "C" int dabgpu_pipe_acquire(dabgpu_pipe *p, const void *iq, int64_t stride, const int64_t *start_h,
                                   const int64_t *n_avail_h) {
    if (!p || !iq || !start_h || !n_avail_h) return fail(DABGPU_E_ARG, "null arg");
    std::vector<int> who;
    for (int s = 0; s < p->S; s++)
        if (!p->st[s].synced) {
            who.push_back(s);
            p->st[s].window = start_h[s];
        }
    int found = 0;
    if (int rc = acquire_streams(p, iq, stride, n_avail_h, who, p->st, found)) return rc;
    if (found < (int)who.size()) return fail(DABGPU_E_STATE, "%d stream(s) found no null symbol", (int)who.size() - found);
    return 0;
}

// One speculative front-end pass over the uncommitted frames of every stream.
// Predicts windows (startIndex = last one) and correctors (unchanged), runs the
// batched kernels, then replays ofdmProcessor::run's sequential logic on the
// host with the measured values and commits the longest correctly predicted
// prefix of each stream (ofdm-processor.cpp:344-468).
static int pipe_front_pass(dabgpu_pipe *p, const void *iq, int64_t stride, const int64_t *n_avail,
                           std::vector<int> &done, std::vector<StreamSt> &cur, bool &progress, bool &lost,
                           const std::function<int()> &after_launch = nullptr) {
    dabgpu_ctx *c = p->c;
    const int S = p->S, F = p->F;
    std::vector<dabgpu_frame> fr;
    std::vector<int> fs, ff;          // stream, frame of each pending entry
    std::vector<int16_t> pred_f2;
    std::vector<int32_t> pred_si;
    bool general = false;
    for (int s = 0; s < S; s++) {
        if (done[s] >= F || !cur[s].synced) continue;
        StreamSt x = cur[s];
        for (int f = done[s]; f < F; f++) {
            dabgpu_frame d;
            memset(&d, 0, sizeof d);
            const int32_t si = x.last_si;
            const int32_t pa = x.coarse + x.fine;
            d.iq_base = stride * s;
            d.n_samples = n_avail[s];
            d.window = x.window;
            d.block0 = x.window + si;
            d.lp_window = x.lp;
            d.phase_a = pa;
            // the reference reads the T_u window first (ofdm-processor.cpp:344-352); whether
            // the rest of the frame is there is known once startIndex is (pass 1)
            if (d.window + TU > n_avail[s]) break;
            int64_t end = d.block0 + TU + (int64_t)NSYM * TS + TNULL;
            // f2 logic with the predicted correction 0 (ofdm-processor.cpp:395-406)
            d.flags = x.f2 ? 1 : 0;
            bool f2 = x.f2;
            int16_t p1 = x.prev1, p2 = x.prev2;
            if (f2) {
                if (p1 == 0 && p2 == 0) f2 = false;
                else { p2 = p1; p1 = 0; }
            }
            const int32_t pb = x.coarse + x.fine;
            d.lp_data = lp_after(x.lp, (int64_t)TU + si, pa);
            d.phase_b = pb;
            d.out_slot = (int32_t)((int64_t)s * p->R + (x.frame_count + (f - done[s])) % p->R);
            fr.push_back(d);
            fs.push_back(s);
            ff.push_back(f);
            pred_si.push_back(si);
            if (pa || pb) general = true;
            // next frame prediction: fine unchanged, null skipped
            int32_t lp_end = lp_after(d.lp_data, (int64_t)NSYM * TS, pb);
            x.lp = lp_after(lp_end, TNULL, pb);
            x.window = end;
            x.f2 = f2; x.prev1 = p1; x.prev2 = p2;
        }
    }
    const int n = (int)fr.size();
    progress = false;
    if (n == 0) return 0;
    // Steady state (no stream runs the coarse AFC of processBlock_0): ONE launch per
    // pass -- every predicted frame's workgroup runs findIndex on its window, places
    // the frame at the startIndex it finds, reports get_snr of block 0 and demodulates
    // the 75 symbols (k_demod_wg<.., SYNC>); one host round trip per pass.  Frames the
    // replay below does not commit are re-predicted and decoded again.  While a
    // stream's coarse AFC is pending the host needs startIndex and processBlock_0's
    // correction first: findIndex, block 0 and the demod run as three launches.
    bool fast = true;
    for (const dabgpu_frame &d : fr) fast = fast && !(d.flags & 1);
    p->front_launches++;
    memcpy(p->h_frames, fr.data(), sizeof(dabgpu_frame) * n);
    HIPCHK(hipMemcpyAsync(p->frames_d, p->h_frames, sizeof(dabgpu_frame) * n, hipMemcpyHostToDevice, c->stream));
    std::vector<int32_t> si(n);
    std::vector<float2> fc_all;
    std::vector<int16_t> snr_all;
    if (fast) {
        fc_all.resize(n);
        snr_all.resize(n);
        DemodAux aux{};
        aux.si = p->si_d;
        aux.snr = p->snr_d;
        aux.level = p->threshold;
        aux.disp = p->display ? p->disp_d : nullptr;
        aux.disp_token = p->disp_token;
        HIPCHK(prof_mark(p, DABGPU_STAGE_DEMOD, true));
        const int kChunks = demod_chunks(n, 2);
        aux.ring8 = 1;
        aux.fmt = p->iq_fmt;
        HIPCHK(launch_demod(c->stream, iq, p->frames_d, n, kChunks, c->T, (int16_t *)p->ring, nullptr, p->fcpart_d, general, aux));
        HIPCHK(prof_mark(p, DABGPU_STAGE_DEMOD, false));
#ifndef DABGPU_BACK_AFTER_PUBLISH
        // the speculative back end (after_launch, queued below) waits for the demod only:
        // the publish feeds the host, not the decoders -- one kernel and its dispatch off
        // the ACS's critical path.  The publish is still launched first, so the ACS's waves
        // do not take the slot it needs before the host can read the pass.
        if (after_launch) {
            HIPCHK(hipEventRecord(p->ev_front, c->stream));
            p->ev_front_demod = true;
        }
#endif
        // the host's values and the error word straight into pinned memory (no copies)
        HIPCHK(launch_front_publish(c->stream, p->fcpart_d, kChunks, n, (float *)p->fc_d, (float *)p->h_fc, p->si_d,
                                    p->h_si, p->snr_d, p->h_snr, c->err, c->h_err));
    } else {
        HIPCHK(prof_mark(p, DABGPU_STAGE_PRS, true));
        HIPCHK(launch_prs_sync(c->stream, iq, p->iq_fmt, p->frames_d, n, c->T, p->threshold, p->si_d, nullptr, nullptr, general));
        HIPCHK(prof_mark(p, DABGPU_STAGE_PRS, false));
        HIPCHK(hipMemcpyAsync(p->h_si, p->si_d, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
    }
    if (after_launch)
        if (int rc = after_launch()) return rc;
    if (fast) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (const int32_t e = *(volatile int32_t *)c->h_err)
            return fail(DABGPU_E_BOUNDS, "kernel refused out-of-bounds work:%s%s", (e & KERR_FRAME) ? " frame descriptor" : "",
                        (e & KERR_VITERBI) ? " viterbi source" : "");
    } else if (int rc = kernel_errors(c)) {
        return rc;
    }
    memcpy(si.data(), p->h_si, sizeof(int32_t) * n);
    if (fast) {
        memcpy(fc_all.data(), p->h_fc, sizeof(float2) * n);
        memcpy(snr_all.data(), p->h_snr, sizeof(int16_t) * n);
    }
    // pass 1: windows.  A frame is usable if every earlier frame of its stream
    // had the predicted startIndex; its own startIndex fixes block0.
    std::vector<char> ok(n, 0);
    std::vector<char> cut(n, 0);          // frames after this one are invalid
    {
        int prev_s = -1;
        bool valid = true;
        for (int i = 0; i < n; i++) {
            if (fs[i] != prev_s) { prev_s = fs[i]; valid = true; }
            if (!valid) continue;
            if (si[i] < 0) {               // sync lost (ofdm-processor.cpp:354-357)
                valid = false;
                continue;
            }
            if (fr[i].window + si[i] + TU + (int64_t)NSYM * TS > n_avail[fs[i]]) {
                valid = false;             // symbols 1..75 not all there yet: wait for samples
                continue;
            }
            // (the null symbol after the frame is skipped when the next frame is read,
            // as the reference's getSamples(T_null) does, ofdm-processor.cpp:449-453)
            ok[i] = 1;
            fr[i].block0 = fr[i].window + si[i];
            fr[i].lp_data = lp_after(fr[i].lp_window, (int64_t)TU + si[i], fr[i].phase_a);
            if (si[i] != pred_si[i]) { cut[i] = 1; valid = false; }
        }
    }
    // pass 2: processBlock_0 (get_snr; coarse AFC for the frames with f2 on) of the
    // usable frames -- in the steady state the fused demod did it already
    std::vector<int> idx;
    for (int i = 0; i < n; i++) if (ok[i]) idx.push_back(i);
    std::vector<dabgpu_frame> fr2;
    for (int i : idx) fr2.push_back(fr[i]);
    const int n2 = (int)fr2.size();
    std::vector<int16_t> corr(n2, 0), snr2(n2, 0);
    if (n2 && !fast) {
        HIPCHK(hipMemcpyAsync(p->frames_d, fr2.data(), sizeof(dabgpu_frame) * n2, hipMemcpyHostToDevice, c->stream));
        HIPCHK(prof_mark(p, DABGPU_STAGE_BLOCK0, true));
        HIPCHK(launch_block0(c->stream, iq, p->iq_fmt, p->frames_d, n2, c->T, p->method, p->corr_d, p->snr_d, general));
        HIPCHK(prof_mark(p, DABGPU_STAGE_BLOCK0, false));
        HIPCHK(hipMemcpyAsync(corr.data(), p->corr_d, sizeof(int16_t) * n2, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(snr2.data(), p->snr_d, sizeof(int16_t) * n2, hipMemcpyDeviceToHost, c->stream));
        if (int rc = kernel_errors(c)) return rc;
    } else if (n2) {
        for (int k = 0; k < n2; k++) snr2[k] = snr_all[idx[k]];
    }
    // replay the coarse corrector with the measured corrections; phase_b of a
    // frame uses its own correction, later frames are cut if the corrector moved
    {
        int prev_s = -1;
        StreamSt x;
        bool valid = true;
        for (int k = 0; k < n2; k++) {
            const int i = idx[k];
            if (fs[i] != prev_s) { prev_s = fs[i]; x = cur[fs[i]]; valid = true; }
            if (!valid) { ok[i] = 0; continue; }
            const int32_t coarse0 = x.coarse;
            if (x.f2) {
                const int16_t cr = corr[k];
                if (cr == 0 && x.prev1 == 0 && x.prev2 == 0) x.f2 = false;
                else if (cr != 100) {
                    x.coarse += cr * 1000;
                    if (std::abs(x.coarse) > 35000) x.coarse = 0;
                    x.prev2 = x.prev1;
                    x.prev1 = cr;
                }
            }
            fr2[k].phase_b = x.coarse + x.fine;
            fr[i].phase_b = fr2[k].phase_b;
            if (fr2[k].phase_b) general = true;
            if (corr[k] != 0 || x.coarse != coarse0) cut[i] = 1;   // prediction assumed correction 0
            if (cut[i]) valid = false;
        }
    }
    std::vector<int16_t> corr_i(n, 0), snr_i(n, 0);
    for (int k = 0; k < n2; k++) {
        corr_i[idx[k]] = corr[k];
        snr_i[idx[k]] = snr2[k];
    }
    // pass 3: demod of the frames still usable
    std::vector<int> idx3;
    std::vector<dabgpu_frame> fr3;
    for (int k = 0; k < n2; k++) if (ok[idx[k]]) { idx3.push_back(idx[k]); fr3.push_back(fr2[k]); }
    const int n3 = (int)fr3.size();
    std::vector<float2> fc(n3);
    if (n3 && fast) {
        for (int k = 0; k < n3; k++) fc[k] = fc_all[idx3[k]];   // demodulated above
    } else if (n3) {
        HIPCHK(hipMemcpyAsync(p->frames_d, fr3.data(), sizeof(dabgpu_frame) * n3, hipMemcpyHostToDevice, c->stream));
        HIPCHK(prof_mark(p, DABGPU_STAGE_DEMOD, true));
        const int kChunks = demod_chunks(n3);
        DemodAux aux{};
        aux.disp = p->display ? p->disp_d : nullptr;
        aux.disp_token = p->disp_token;
        aux.ring8 = 1;
        aux.fmt = p->iq_fmt;
        HIPCHK(launch_demod(c->stream, iq, p->frames_d, n3, kChunks, c->T, (int16_t *)p->ring, nullptr, p->fcpart_d, general, aux));
        HIPCHK(prof_mark(p, DABGPU_STAGE_DEMOD, false));
        HIPCHK(launch_fc_reduce(c->stream, p->fcpart_d, kChunks, n3, p->fc_d));
        HIPCHK(hipMemcpyAsync(fc.data(), p->fc_d, sizeof(float2) * n3, hipMemcpyDeviceToHost, c->stream));
        if (int rc = kernel_errors(c)) return rc;
    }
    // commit: replay the full per-frame state update (ofdm-processor.cpp:395-468)
    {
        int prev_s = -1;
        bool valid = true;
        for (int k = 0; k < n3; k++) {
            const int i = idx3[k];
            const int s = fs[i];
            if (s != prev_s) { prev_s = s; valid = true; }
            if (!valid) continue;
            StreamSt &x = cur[s];
            const dabgpu_frame &d = fr3[k];
            // coarse (same replay as above)
            if (x.f2) {
                const int16_t cr = corr_i[i];
                if (cr == 0 && x.prev1 == 0 && x.prev2 == 0) x.f2 = false;
                else if (cr != 100) {
                    x.coarse += cr * 1000;
                    if (std::abs(x.coarse) > 35000) x.coarse = 0;
                    x.prev2 = x.prev1;
                    x.prev1 = cr;
                }
            }
            const int16_t fine0 = x.fine;
            const int32_t coarse0 = x.coarse;
            // fineCorrector += 0.1 * arg(FreqCorr) / M_PI * (carrierDiff / 2)
            const float a = atan2f(fc[k].y, fc[k].x);
            x.fine = (int16_t)(x.fine + 0.1 * a / M_PI * (1000 / 2));
            int32_t lp_end = lp_after(d.lp_data, (int64_t)NSYM * TS, d.phase_b);
            x.lp = lp_after(lp_end, TNULL, x.coarse + x.fine);
            if (x.fine > 500) { x.coarse += 1000; x.fine -= 1000; }
            else if (x.fine < -500) { x.coarse -= 1000; x.fine += 1000; }
            x.window = d.block0 + TU + (int64_t)NSYM * TS + TNULL;
            x.last_si = (int32_t)(d.block0 - d.window);
            p->last_frames[(size_t)s * p->F + done[s]] = d;
            p->last_si[(size_t)s * p->F + done[s]] = x.last_si;
            {
                dabgpu_frame_info &fi = p->last_info[(size_t)s * p->F + done[s]];
                fi.window = d.window;
                fi.start_index = x.last_si;
                fi.coarse = coarse0;
                fi.fine = fine0;
                fi.correction = corr_i[i];
                fi.snr = snr_i[i];
                fi.committed = 1;
            }
            done[s]++;
            x.frame_count++;
            progress = true;
            if (x.fine != fine0 || x.coarse != coarse0 || cut[i]) valid = false;
        }
    }
    // sync loss: the first uncommitted frame's window was read exactly as the
    // reference would and findIndex failed -> goto notSynced (ofdm-processor.cpp:354-357)
    for (int i = 0; i < n; i++) {
        const int s = fs[i];
        StreamSt &x = cur[s];
        if (ff[i] == done[s] && si[i] < 0 && fr[i].window == x.window && fr[i].lp_window == x.lp &&
            fr[i].phase_a == x.coarse + x.fine) {
            x.synced = false;
            x.lp = lp_after(x.lp, TU, x.coarse + x.fine);
            x.window += TU;
            x.resyncs++;
            lost = true;
        }
    }
    return 0;
}

extern "C" {

int dabgpu_pipe_run(dabgpu_pipe *p, const void *iq, int64_t stride, const int64_t *n_avail, uint8_t *fic_bits,
                    uint8_t *fic_crc, uint8_t *msc_bits, int32_t msc_stride, uint8_t *msc_valid) {
    if (!p || !iq || !n_avail) return fail(DABGPU_E_ARG, "null arg");
    dabgpu_ctx *c = p->c;
    const int S = p->S, F = p->F;
    const bool do_msc = msc_bits && p->NSUB > 0;
    const int need = p->packed ? (p->max_nbits + 7) / 8 : p->max_nbits;
    if (do_msc && msc_stride < need) return fail(DABGPU_E_ARG, "msc_stride %d < %d", msc_stride, need);
    if (int rc = back_errors(p, false)) return rc;
    if (int rc = acq_collect(p, false)) return rc;        // a background null search that finished
    p->last_frames.assign((size_t)S * F, dabgpu_frame());
    p->last_si.assign((size_t)S * F, 0);
    p->last_info.assign((size_t)S * F, dabgpu_frame_info());
    p->last_msc = nullptr;
    if (p->profiling == 1) p->ev_rec.clear();   // modes 2, 3 accumulate over runs
    p->ev_front_demod = false;
    // at most one run of overlap: run r-2's ACS, the last reader of the ring slots this
    // run's demod reuses, must be done (not its traceback, FIC CRC and DAB+ layer: waiting
    // for those held the demod back from the slots the ACS's last waves leave free --
    // profiles/r04_front_gate_ab.txt)
    const int par = (int)(p->run_idx & 1);
    if (p->acs_rec[par]) HIPCHK(hipStreamWaitEvent(c->stream, p->ev_acs[par], 0));
    std::vector<int> done(S, 0);
    std::vector<StreamSt> cur = p->st;
    p->cur = par;
    hipStream_t bs = p->vs[par];
    // Channel decoding on the pipeline's back-end stream, after this run's front end:
    // FIC for every committed frame (slot[s*F+f] = its ring slot, -1 none), MSC for all
    // subchannels of every delivered CIF (dn[s] frames of stream s).  With both, one ACS
    // and one traceback launch decode them together (the FIC's short waves fill the SIMDs
    // the MSC's last waves leave idle); decisions in separate halves of the stream's
    // decision buffer.
    auto enqueue_back = [&](const std::vector<int> &dn, const std::vector<int32_t> &slots) -> int {
        // per stream: CIF index of its first CIF slot and the CIFs it delivered (the
        // staging half is reused only once its previous uploads have executed)
        if (p->copy_rec[par]) HIPCHK(hipEventSynchronize(p->ev_copy[par]));
        for (int s = 0; s < S; s++) {
            p->h_cif0(par)[s] = p->st[s].cif_count;
            p->h_ncif(par)[s] = 4 * dn[s];
        }
        if (fic_bits) memcpy(p->h_slots(par), slots.data(), sizeof(int32_t) * S * F);
        // one upload of the block (the FIC slots only when the FIC is decoded)
        HIPCHK(hipMemcpyAsync(p->cif0_dev(par), p->h_cif0(par), 12 * (size_t)S + (fic_bits ? 4 * (size_t)S * F : 0),
                              hipMemcpyHostToDevice, bs));
        VitJob JF, JM;
        memset(&JF, 0, sizeof JF);
        memset(&JM, 0, sizeof JM);
        int32_t *slots_d = p->slots_dev(par);
        HIPCHK(hipEventRecord(p->ev_copy[par], bs));
        p->copy_rec[par] = true;
        if (fic_bits) {
            JF.kind = SRC_FIC;
            JF.n_cw = 4 * S * F;
            JF.src = (const int16_t *)p->ring;
            JF.ring8 = 1;
            JF.src_len = (int64_t)S * p->R * FRAME_SOFT;
            JF.err = p->berr_d + par;
            JF.slots = slots_d;
            JF.prof = (const Profile *)p->ficprof_d;
            JF.inv = c->fic_inv;
            JF.out = fic_bits;
            JF.out_stride = p->fic_packed ? 96 : 768;     // 3 FIBs of 32 bytes, or 768 bits
            JF.packed = p->fic_packed ? 1 : 0;
            JF.prbs = 1;
            JF.prbs_words = c->prbs;
            JF.dec = p->dec_d[par] + p->dec_fic_off;
            JF.dec_ncw = dec_rows(JF.n_cw);
            JF.dec_nch = dec_chunks(768);
        }
        if (do_msc) {
            JM.kind = SRC_MSC;
            JM.n_cw = S * 4 * F * p->NSUB;
            JM.src = (const int16_t *)p->ring;
            JM.ring8 = 1;
            JM.src_len = (int64_t)S * p->R * FRAME_SOFT;
            JM.err = p->berr_d + par;
            JM.prof = p->prof_d;
            JM.inv = p->inv_d;
            JM.nsub = p->NSUB;
            JM.ncif = 4 * F;
            JM.ring = p->R;
            JM.cif0s = p->cif0_dev(par);
            JM.ncifs = p->ncif_dev(par);
            JM.sub_start = p->inject_bounds ? p->substart_bad_d : p->substart_d;
            JM.out = msc_bits;
            JM.out_stride = msc_stride;
            JM.packed = p->packed ? 1 : 0;
            JM.prbs = 1;
            JM.prbs_words = c->prbs;
            JM.dec = p->dec_d[par];
            JM.dec_ncw = dec_rows(JM.n_cw);
            JM.dec_nch = dec_chunks(p->max_nbits);
        }
        // the small uploads above run on the back-end stream while the front end still
        // works; only the decoders wait for it.
        // What the back end may read of the front end's output: the soft-bit ring (p->ring,
        // written by the demod) and the host-built descriptors uploaded on bs above -- never
        // what k_front_publish writes (fc_d, si_d, snr_d, the error word): ev_front may mark
        // the demod alone (ev_front_demod), before the publish.  A back-end reader of those
        // must wait for an event recorded after the publish (DABGPU_BACK_AFTER_PUBLISH).
        // (Measured: launching run r's traceback
        // beside run r+1's ACS instead of beside run r+1's demod is 2 % slower -- the ACS
        // loses more than the demod gains.)
        if (!p->ev_front_demod) HIPCHK(hipEventRecord(p->ev_front, c->stream));
        p->ev_front_demod = false;
        HIPCHK(hipStreamWaitEvent(bs, p->ev_front, 0));
        if (fic_bits && do_msc && p->vit_slices > 1) {
            // the A/B form: K slices of traceback blocks; slice i's traceback on ts reads the
            // decisions slice i's ACS has just written while slice i + 1's ACS runs
            const int nblk = (JM.n_cw + 63) / 64, K = p->vit_slices, per = (nblk + K - 1) / K;
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_ACS, true));
            for (int i = 0; i * per < nblk; i++) {
                const int b0 = i * per, b1 = std::min(nblk, b0 + per);
                HIPCHK(launch_acs_msc_fic_range(bs, JM, JF, b0, b1, b1 == nblk));
                HIPCHK(hipEventRecord(p->ev_slice[i], bs));
                HIPCHK(hipStreamWaitEvent(p->ts, p->ev_slice[i], 0));
                HIPCHK(launch_traceback_msc_fic_range(p->ts, JM, JF, b0, b1, b1 == nblk));
            }
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_ACS, false));
            HIPCHK(hipEventRecord(p->ev_acs[par], bs));
            p->acs_rec[par] = true;
            HIPCHK(hipEventRecord(p->ev_tb, p->ts));
            HIPCHK(hipStreamWaitEvent(bs, p->ev_tb, 0));
            HIPCHK(prof_mark(p, DABGPU_STAGE_FIC, true));
            if (fic_crc) HIPCHK(launch_fic_post(bs, fic_bits, fic_crc, 12 * S * F, c->dptab, slots_d, p->fic_packed));
            HIPCHK(prof_mark(p, DABGPU_STAGE_FIC, false));
        } else if (fic_bits && do_msc) {
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_ACS, true));
            HIPCHK(launch_acs_msc_fic(bs, JM, JF));
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_ACS, false));
            HIPCHK(hipEventRecord(p->ev_acs[par], bs));
            p->acs_rec[par] = true;
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_TB, true));
            HIPCHK(launch_traceback_msc_fic(bs, JM, JF));
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_TB, false));
            HIPCHK(prof_mark(p, DABGPU_STAGE_FIC, true));
            if (fic_crc) HIPCHK(launch_fic_post(bs, fic_bits, fic_crc, 12 * S * F, c->dptab, slots_d, p->fic_packed));
            HIPCHK(prof_mark(p, DABGPU_STAGE_FIC, false));
        } else if (fic_bits) {
            HIPCHK(prof_mark(p, DABGPU_STAGE_FIC, true));
            HIPCHK(launch_viterbi(bs, JF));
            HIPCHK(hipEventRecord(p->ev_acs[par], bs));
            p->acs_rec[par] = true;
            if (fic_crc) HIPCHK(launch_fic_post(bs, fic_bits, fic_crc, 12 * S * F, c->dptab, slots_d, p->fic_packed));
            HIPCHK(prof_mark(p, DABGPU_STAGE_FIC, false));
        } else if (do_msc) {
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_ACS, true));
            HIPCHK(launch_acs(bs, JM));
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_ACS, false));
            HIPCHK(hipEventRecord(p->ev_acs[par], bs));
            p->acs_rec[par] = true;
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_TB, true));
            HIPCHK(launch_traceback(bs, JM));
            HIPCHK(prof_mark(p, DABGPU_STAGE_MSC_TB, false));
        }
        return 0;
    };
    // Speculative back end: in steady state (every stream synchronised, no coarse AFC
    // pending) the first front pass commits exactly the frames it predicts, so the
    // channel decoding of those frames is queued right behind it, before the host has
    // read and verified the pass -- the GPU does not idle through the host's replay.  If
    // the replay commits anything else, or a second pass rewrites frames, the back end
    // is queued again with the committed frames and overwrites the outputs.
    std::vector<int> pred(S, 0);
    std::vector<int32_t> pred_slot((size_t)S * F, -1);
    bool spec = (fic_bits || do_msc) && p->speculate;
    for (int s = 0; s < S && spec; s++) {
        const StreamSt &x = cur[s];
        if (!x.synced || x.f2) { spec = false; break; }
        int64_t w = x.window;
        for (int f = 0; f < F; f++) {
            const int64_t end = w + x.last_si + TU + (int64_t)NSYM * TS;
            if (end > n_avail[s]) break;
            pred_slot[(size_t)s * F + f] = (int32_t)((int64_t)s * p->R + (x.frame_count + f) % p->R);
            pred[s] = f + 1;
            w = end + TNULL;
        }
    }
    bool spec_sent = false;
    size_t spec_rec0 = 0, spec_rec1 = 0;         // profiling records of the speculative enqueue
    int passes = 0;
    // an error after the speculative back end was queued: it still writes the caller's
    // outputs and reads ring slots, so it is tracked like a completed run's back end
    // (the next run's demod waits for it) and finished before the error returns
    auto bail = [&](int rc) -> int {
        if (spec_sent) {
            (void)launch_take_error(bs, p->berr_d + par, p->h_berr + par);
            (void)hipEventRecord(p->ev_back[par], bs);
            p->back_rec[par] = true;
            (void)hipStreamSynchronize(bs);
        }
        return rc;
    };
    // ofdmProcessor::run per stream: speculative front-end passes commit frames; a
    // stream that loses sync (or was never synchronised) searches the next null
    // symbol from where it is and continues (goto notSynced, ofdm-processor.cpp:354-357).
    // Every pass either commits a frame or moves a stream past samples, so this ends.
    for (int it = 0; it < 64 * F + 64; it++) {
        // streams that need the null search: in the background (DABGPU_CTL_ACQ_ASYNC, the
        // default) those that lost sync after an acquisition -- this run goes on without
        // them, one batch in flight; inside the run (the reference's order) the others: a
        // stream's first search (it has no frames to decode before it) and, with
        // DABGPU_CTL_ACQ_SYNC, every search
        std::vector<int> who, bg;
        for (int s = 0; s < S; s++) {
            if (cur[s].synced || done[s] >= F) continue;
            if (p->acq_async && cur[s].acquisitions > 0) {
                if (!p->acquiring[s]) bg.push_back(s);
            } else {
                who.push_back(s);
            }
        }
        int found = 0;
        if (!bg.empty() && !p->acq_inflight)
            if (int rc = acquire_streams_async(p, iq, stride, n_avail, bg, cur)) return bail(rc);
        if (int rc = acquire_streams(p, iq, stride, n_avail, who, cur, found)) return bail(rc);
        bool progress = false, lost = false;
        std::function<int()> after;
        if (spec && it == 0 && found == 0)
            after = [&]() -> int {
                spec_sent = true;
                spec_rec0 = p->ev_rec.size();
                const int rc = enqueue_back(pred, pred_slot);
                spec_rec1 = p->ev_rec.size();
                return rc;
            };
        const int64_t launches_before = p->front_launches;
        if (int rc = pipe_front_pass(p, iq, stride, n_avail, done, cur, progress, lost, after)) return bail(rc);
        if (p->front_launches != launches_before) passes++;
        if (!progress && !lost && !found) break;
    }
    bool all = true;
    for (int s = 0; s < S; s++) {
        if (done[s] != F && !(p->acq_async && cur[s].acquisitions > 0 && (p->acquiring[s] || !cur[s].synced))) all = false;
        cur[s].frames_run = done[s];
    }
    std::vector<int32_t> slot((size_t)S * F, -1);
    for (int s = 0; s < S; s++)
        for (int f = 0; f < done[s]; f++) slot[(size_t)s * F + f] = p->last_frames[(size_t)s * F + f].out_slot;
    bool hit = spec_sent && passes == 1 && done == pred && slot == pred_slot;
    p->spec_runs += spec_sent ? 1 : 0;
    p->spec_hits += hit ? 1 : 0;
    if (!hit) {
        // the speculative decode is overwritten: its stage times are not this run's
        for (size_t i = spec_rec0; i < spec_rec1; i++) p->ev_rec[i].first = -1;
        if (int rc = enqueue_back(done, slot)) return bail(rc);
    }
    HIPCHK(launch_take_error(bs, p->berr_d + par, p->h_berr + par));
    HIPCHK(hipEventRecord(p->ev_back[par], bs));
    p->back_rec[par] = true;
    p->run_idx++;
    p->inject_bounds = false;
    p->last_msc = do_msc ? msc_bits : nullptr;
    p->last_msc_stride = msc_stride;
    p->last_msc_packed = p->packed;
    if (msc_valid)
        for (int s = 0; s < S; s++)
            for (int q = 0; q < 4 * F; q++)
                msc_valid[(size_t)s * 4 * F + q] = (q < 4 * done[s] && p->st[s].cif_count + q >= 16) ? 1 : 0;
    for (int s = 0; s < S; s++) cur[s].cif_count = p->st[s].cif_count + 4 * (int64_t)done[s];
    p->st = cur;
    if (!all) return fail(DABGPU_E_STATE, "a stream ran out of samples (see dabgpu_pipe_state)");
    return 0;
}

int dabgpu_pipe_set_profiling(dabgpu_pipe *p, int on) {
    if (!p) return fail(DABGPU_E_ARG, "null pipe");
    if (on < 0 || on > 3) return fail(DABGPU_E_ARG, "profiling mode %d", on);
    HIPCHK(hipStreamSynchronize(p->c->stream));         // events of earlier runs are complete
    for (hipStream_t v : p->vs) HIPCHK(hipStreamSynchronize(v));
    p->profiling = on;
    p->ev_rec.clear();
    return 0;
}
int dabgpu_pipe_timing(dabgpu_pipe *p, float *ms, int32_t *launches) {
    if (!p || !ms) return fail(DABGPU_E_ARG, "bad args");
    // stages recorded since the last dabgpu_pipe_run started (incl. dabgpu_pipe_dabplus)
    HIPCHK(hipStreamSynchronize(p->c->stream));
    for (hipStream_t v : p->vs) HIPCHK(hipStreamSynchronize(v));
    for (int k = 0; k < DABGPU_NSTAGE; k++) { p->stage_ms[k] = 0.0f; p->stage_n[k] = 0; }
    for (auto &r : p->ev_rec) {
        if (r.first < 0) continue;              // discarded (a missed speculation)
        float t = 0.0f;
        HIPCHK(hipEventElapsedTime(&t, p->ev_pool[r.second], p->ev_pool[r.second + 1]));
        p->stage_ms[r.first] += t;
        p->stage_n[r.first] += 1;
    }
    for (int k = 0; k < DABGPU_NSTAGE; k++) {
        ms[k] = p->stage_ms[k];
        if (launches) launches[k] = p->stage_n[k];
    }
    return 0;
}

int dabgpu_pipe_acquire_wait(dabgpu_pipe *p) {
    if (!p) return fail(DABGPU_E_ARG, "null pipe");
    return acq_collect(p, true);
}

int dabgpu_pipe_sync(dabgpu_pipe *p) {
    if (!p) return fail(DABGPU_E_ARG, "null pipe");
    HIPCHK(hipStreamSynchronize(p->c->stream));
    for (hipStream_t v : p->vs) HIPCHK(hipStreamSynchronize(v));
    if (int rc = back_errors(p, true)) return rc;
    return kernel_errors(p->c);
}

int dabgpu_pipe_dabplus(dabgpu_pipe *p, uint8_t *sf_bytes, int32_t sf_stride, dabgpu_superframe *info) {
    if (!p || !sf_bytes || !info) return fail(DABGPU_E_ARG, "null arg");
    if (p->NDP == 0) return fail(DABGPU_E_STATE, "no DAB+ subchannel in this pipeline");
    if (!p->last_msc) return fail(DABGPU_E_STATE, "no dabgpu_pipe_run with MSC output to consume");
    if (sf_stride < 110 * p->dp_max_rs) return fail(DABGPU_E_ARG, "sf_stride %d < %d", sf_stride, 110 * p->dp_max_rs);
    dabgpu_ctx *c = p->c;
    DpJob J;
    memset(&J, 0, sizeof J);
    J.msc = p->last_msc;
    J.msc_stride = p->last_msc_stride;
    J.packed = p->last_msc_packed ? 1 : 0;
    J.ncif = 4 * p->F;
    J.nsub = p->NSUB;
    J.ndp = p->NDP;
    J.nstreams = p->S;
    J.cif0s = p->cif0_dev(p->cur);
    J.ncifs = p->ncif_dev(p->cur);
    J.dp_sub = p->dp_sub_d;
    J.dp_br = p->dp_br_d;
    J.ring = p->dp_ring_d;
    J.state = p->dp_state_d;
    J.code = p->dp_code_d;
    J.ncand = p->dp_cand_d;
    J.cand = p->dp_cand_d + 1;
    J.sf_out = sf_bytes;
    J.sf_stride = sf_stride;
    if (p->dp_compact) {
        if (p->F > 512) return fail(DABGPU_E_UNSUP, "compact DAB+ output: at most 512 frames per run");
        const size_t need = (size_t)p->S * 4 * p->F * p->NDP * (size_t)sf_stride;
        if (need > p->sf_sparse_bytes) {
            // the layers that wrote the old scratch ran on this pipeline's back-end streams:
            // wait for those (not the whole device: other pipelines, the null search)
            for (hipStream_t v : p->vs) HIPCHK(hipStreamSynchronize(v));
            if (p->sf_sparse_d) HIPCHK(hipFree(p->sf_sparse_d));
            p->sf_sparse_d = nullptr;
            p->sf_sparse_bytes = 0;
            HIPCHK(hipMalloc((void **)&p->sf_sparse_d, need));
            p->sf_sparse_bytes = need;
        }
        J.sf_out = p->sf_sparse_d;
        J.sf_compact = sf_bytes;
        J.kmax = DABGPU_SF_SLOTS(p->F);
    }
    J.info = info;
    J.tabs = c->dptab;
    // on the last run's back-end stream (after its MSC), after the previous
    // superframe pass (the 5-CIF rings carry state from run to run)
    hipStream_t bs = p->vs[p->cur];
    if (p->dp_rec) HIPCHK(hipStreamWaitEvent(bs, p->ev_dp, 0));
    HIPCHK(prof_mark(p, DABGPU_STAGE_DABPLUS, true));
    HIPCHK(launch_dabplus(bs, J));
    HIPCHK(prof_mark(p, DABGPU_STAGE_DABPLUS, false));
    HIPCHK(hipEventRecord(p->ev_dp, bs));
    p->dp_rec = true;
    // (the run after next does not wait for this: the layer reads this run's MSC output
    // and CIF counters, which that run's back end overwrites behind it on this stream)
    p->last_msc = nullptr;                     // each run's CIFs enter the superframe layer once
    return 0;
}

int dabgpu_pipe_state(dabgpu_pipe *p, int s, dabgpu_stream_state *o) {
    if (!p || !o || s < 0 || s >= p->S) return fail(DABGPU_E_ARG, "bad args");
    // a background null search that has finished is taken now (not at the next run), so
    // `acquiring` says whether the search still reads iq_d
    if (int rc = acq_collect(p, false)) return rc;
    const StreamSt &x = p->st[s];
    o->next_pos = x.window;
    o->local_phase = x.lp;
    o->coarse = x.coarse;
    o->fine = x.fine;
    o->f2correction = x.f2;
    o->prev1 = x.prev1;
    o->prev2 = x.prev2;
    o->synced = x.synced;
    o->cif_count = x.cif_count;
    o->last_start_index = x.last_si;
    o->resyncs = x.resyncs;
    o->acquisitions = x.acquisitions;
    o->attempts = x.attempts;
    o->no_signal = x.no_signal;
    o->frames_run = x.frames_run;
    o->acquiring = (p->acq_async && !p->acquiring.empty() && p->acquiring[s]) ? 1 : 0;
    return 0;
}

int dabgpu_pipe_frame_info(dabgpu_pipe *p, dabgpu_frame_info *info) {
    if (!p || !info) return fail(DABGPU_E_ARG, "bad args");
    if (p->last_info.empty()) memset(info, 0, sizeof(dabgpu_frame_info) * (size_t)p->S * p->F);
    else memcpy(info, p->last_info.data(), sizeof(dabgpu_frame_info) * p->last_info.size());
    return 0;
}

int dabgpu_pipe_control(dabgpu_pipe *p, int stream, int op) {
    if (!p || stream < -1 || stream >= p->S) return fail(DABGPU_E_ARG, "bad args");
    if (op == DABGPU_CTL_SCAN_ON || op == DABGPU_CTL_SCAN_OFF) {      // set_scanMode (one flag, like the reference's)
        p->scan = op == DABGPU_CTL_SCAN_ON;
        return 0;
    }
    if (op == DABGPU_CTL_INJECT_BOUNDS) {
        if (p->NSUB == 0) return fail(DABGPU_E_STATE, "no MSC subchannel to corrupt");
        if (!p->substart_bad_d) {
            HIPCHK(hipMalloc((void **)&p->substart_bad_d, sizeof(int32_t) * p->NSUB));
            std::vector<int32_t> bad(p->NSUB);
            for (int i = 0; i < p->NSUB; i++) bad[i] = p->sub[i].startAddr * 64;
            bad[0] = 0x40000000;                        // far past any ring (no int32 overflow in the loader)
            HIPCHK(hipMemcpy(p->substart_bad_d, bad.data(), sizeof(int32_t) * p->NSUB, hipMemcpyHostToDevice));
        }
        p->inject_bounds = true;
        return 0;
    }
    if (op == DABGPU_CTL_ACQ_ASYNC || op == DABGPU_CTL_ACQ_SYNC) {
        if (op == DABGPU_CTL_ACQ_SYNC) {
            if (int rc = acq_collect(p, true)) return rc;   // a search in flight completes first
            p->acq_async = false;
            return 0;
        }
        if (int rc = acq_async_setup(p)) return rc;
        p->acq_async = true;
        return 0;
    }
    // a background search in flight carries the stream's old correctors and position: it
    // completes and is applied first, so the control below is the last word (the reference
    // runs these methods between its own sequential steps)
    if (int rc = acq_collect(p, true)) return rc;
    for (int s = (stream < 0 ? 0 : stream); s < (stream < 0 ? p->S : stream + 1); s++) {
        StreamSt &x = p->st[s];
        switch (op) {
        case DABGPU_CTL_RESET: x.fine = 0; x.coarse = 0; x.f2 = true; break;      // ofdm-processor.cpp:476-479
        case DABGPU_CTL_COARSE_ON: x.f2 = true; x.coarse = 0; break;             // :498-501
        case DABGPU_CTL_COARSE_OFF: x.f2 = false; break;                         // :503-505
        case DABGPU_CTL_RESYNC: x.synced = false; break;
        default: return fail(DABGPU_E_ARG, "unknown control op %d", op);
        }
    }
    return 0;
}

int dabgpu_pipe_softbits(dabgpu_pipe *p, const uint8_t **soft, int32_t *ring) {
    if (!p || !soft || !ring) return fail(DABGPU_E_ARG, "bad args");
    *soft = p->ring;
    *ring = p->R;
    return 0;
}
int dabgpu_pipe_frame_slot(dabgpu_pipe *p, int frame, int32_t *slot) {
    if (!p || !slot || frame < 0 || frame >= p->F) return fail(DABGPU_E_ARG, "bad args");
    *slot = p->last_frames.empty() ? -1 : p->last_frames[frame].out_slot;
    return 0;
}
int dabgpu_pipe_set_packed(dabgpu_pipe *p, int on) {
    if (!p || on < 0 || on > (DABGPU_PACK_MSC | DABGPU_PACK_FIC)) return fail(DABGPU_E_ARG, "packing %d", on);
    p->packed = (on & DABGPU_PACK_MSC) != 0;
    p->fic_packed = (on & DABGPU_PACK_FIC) != 0;
    return 0;
}
int dabgpu_pipe_set_iq_format(dabgpu_pipe *p, int format) {
    if (!p || (format != DABGPU_IQ_F32 && format != DABGPU_IQ_S16 && format != DABGPU_IQ_U8))
        return fail(DABGPU_E_ARG, "bad args");
    p->iq_fmt = format;
    return 0;
}
int dabgpu_pipe_set_dabplus_compact(dabgpu_pipe *p, int on) {
    if (!p) return fail(DABGPU_E_ARG, "bad args");
    p->dp_compact = on != 0;
    return 0;
}
int dabgpu_pipe_fetch(dabgpu_pipe *p, void *dst_h, const void *src_d, size_t bytes) {
    if (!p || (bytes && (!dst_h || !src_d))) return fail(DABGPU_E_ARG, "bad args");
    if (p->run_idx == 0) return fail(DABGPU_E_STATE, "no dabgpu_pipe_run to fetch from");
    if (!bytes) return 0;
    // on the last run's back-end stream, behind its channel decoding (and DAB+ layer)
    // (the runtime's copy is a blit kernel on this runtime; queued on a high-priority
    // stream of its own it delivered 10 % less -- it then takes wave slots from the next
    // run's ACS: profiles/r04_delivered_ab.txt)
    hipStream_t bs = p->vs[p->cur];
    // into pinned host memory the device can address (dabgpu_host_alloc), 16-byte
    // aligned: k_to_host's few waves; otherwise the runtime's copy
    static const int wgs = [] { const char *e = getenv("DABGPU_D2H_WGS"); return e ? atoi(e) : 4; }();
    void *dd = nullptr;
    if (wgs > 0 && !((((uintptr_t)dst_h | (uintptr_t)src_d | bytes) & 15)) &&
        hipHostGetDevicePointer(&dd, dst_h, 0) == hipSuccess && dd)
        HIPCHK(launch_to_host(bs, src_d, dd, bytes, wgs));
    else {
        (void)hipGetLastError();                  // a refused device-pointer query is not an error here
        HIPCHK(hipMemcpyAsync(dst_h, src_d, bytes, hipMemcpyDeviceToHost, bs));
    }
    // no ev_back record: the copy reads only this run's outputs, which the next run on
    // this stream (the run after next) overwrites in stream order; the front end of that
    // run does not wait for it
    return 0;
}
int dabgpu_pipe_set_display(dabgpu_pipe *p, int on) {
    if (!p) return fail(DABGPU_E_ARG, "bad args");
    if (on && !p->disp_d) {
        HIPCHK(hipStreamSynchronize(p->c->stream));
        HIPCHK(hipMalloc((void **)&p->disp_d, sizeof(float2) * (size_t)p->S * p->R * K));
        HIPCHK(hipMemset(p->disp_d, 0, sizeof(float2) * (size_t)p->S * p->R * K));
    }
    p->display = on != 0;
    return 0;
}
int dabgpu_pipe_set_display_token(dabgpu_pipe *p, int token) {
    if (!p || token < 1 || token > NSYM) return fail(DABGPU_E_ARG, "display token %d outside 1..75", token);
    p->disp_token = token;
    return 0;
}
int dabgpu_pipe_iq_display(dabgpu_pipe *p, int stream, int frame, float *carriers_h) {
    if (!p || !carriers_h || stream < 0 || stream >= p->S || frame < 0 || frame >= p->F)
        return fail(DABGPU_E_ARG, "bad args");
    if (!p->display || !p->disp_d) return fail(DABGPU_E_STATE, "display feed off (dabgpu_pipe_set_display)");
    const size_t i = (size_t)stream * p->F + frame;
    if (p->last_info.size() <= i || !p->last_info[i].committed)
        return fail(DABGPU_E_STATE, "stream %d frame %d was not decoded in the last run", stream, frame);
    const int32_t slot = p->last_frames[i].out_slot;
    HIPCHK(hipMemcpyAsync(carriers_h, p->disp_d + (size_t)slot * K, sizeof(float2) * K, hipMemcpyDeviceToHost,
                          p->c->stream));
    HIPCHK(hipStreamSynchronize(p->c->stream));
    return 0;
}
int dabgpu_pipe_frames(dabgpu_pipe *p, dabgpu_frame *fr, int32_t *si) {
    if (!p) return fail(DABGPU_E_ARG, "bad args");
    if (fr) memcpy(fr, p->last_frames.data(), sizeof(dabgpu_frame) * p->last_frames.size());
    if (si) memcpy(si, p->last_si.data(), sizeof(int32_t) * p->last_si.size());
    return 0;
}

}  // extern "C"
