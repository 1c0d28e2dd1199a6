// ref_wrap.cpp -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" shims around the reference's own compilable classes, so the
// parity tests and tests/golden/make_golden.py can run the REAL reference
// code (compiled from /root/reference by oracle/Makefile into
// oracle/_ref/libdabref.so; nothing from the reference is copied here).
// Compiled with the reference's CMake defaults: SSE_AVAILABLE + spiral-sse.c
// (CMakeLists.txt:96-105).
#include "dab-constants.h"
#include "viterbi.h"
#include "deconvolve.h"
#include "protTables.h"
#include "reed-solomon.h"
#include "firecode-checker.h"
#include "mapper.h"
#include "phasetable.h"
#include <cstring>

extern "C" {

void ref_viterbi(const int16_t *in, int nbits, uint8_t *out) {          // viterbi.cpp:225
    viterbi v((int16_t)nbits);
    v.deconvolve(const_cast<int16_t *>(in), out);
}

void ref_uep_deconvolve(int bitRate, int protLevel, const int16_t *in, int size, uint8_t *out) { // deconvolve.cpp:172
    uep_deconvolve u((int16_t)bitRate, (int16_t)protLevel);
    u.deconvolve(const_cast<int16_t *>(in), size, out);
}

void ref_eep_deconvolve(int bitRate, int protLevel, const int16_t *in, int size, uint8_t *out) { // deconvolve.cpp:325
    eep_deconvolve e((int16_t)bitRate, (int16_t)protLevel);
    e.deconvolve(const_cast<int16_t *>(in), size, out);
}

int ref_rs_dec(const uint8_t *in, uint8_t *out) {                        // reed-solomon.cpp:129
    reedSolomon rs(8, 0435, 0, 1, 10);
    return rs.dec(in, out, 135);
}

void ref_rs_enc(const uint8_t *in, uint8_t *out) {                       // reed-solomon.cpp:110
    uint8_t tmp[120] = {0};
    for (int i = 0; i < 110; i++) tmp[i] = in[i];
    reedSolomon rs(8, 0435, 0, 1, 10);
    rs.enc(tmp, out, 135);
}

int ref_firecode_check(const uint8_t *x) {                               // firecode-checker.cpp:76
    firecode_checker fc;
    return fc.check(x) ? 1 : 0;
}

void ref_mapper(int16_t *out) {                                          // mapper.cpp:57-117
    DabParams p;
    p.dabMode = 1; p.L = 76; p.K = 1536; p.T_null = 2656; p.T_F = 196608;
    p.T_s = 2552; p.T_u = 2048; p.guardLength = 504; p.carrierDiff = 1000;
    permVector pv(&p);
    for (int i = 0; i < 1536; i++) out[i] = pv.mapIn((int16_t)i);
}

float ref_get_phi(int k) {                                                // phasetable.cpp:261
    phaseTable pt(1);
    return pt.get_Phi(k);
}

int ref_check_crc_bits(uint8_t *in, int size) {                          // dab-constants.h:311
    return check_CRC_bits(in, (int16_t)size) ? 1 : 0;
}

void ref_pcode(int idx, int8_t *out) {                                    // protTables.cpp:56
    int8_t *p = get_PCodes((int16_t)(idx - 1));
    for (int i = 0; i < 32; i++) out[i] = p[i];
}

// mp4Processor::addtoFrame / processSuperframe (mp4processor.cpp:107-292) minus faad,
// for the CPU baseline: the reference's own firecode_checker and reedSolomon classes
// do the work; the byte packing, block counting, RS column interleave, AU table and
// AU CRC around them are restated (mp4processor.cpp cannot be compiled: Qt, faad).
// Returns 0 (fewer than 5 blocks), 1 (fire code failed), 2 (superframe rejected),
// 3 (decoded; *n_aus_ok = AUs whose CRC holds).
struct ref_mp4 {
    int bitRate, fill, blocks;
    uint8_t ring[120 * 48];
};
static bool au_crc(const uint8_t *msg, int16_t len) {                   // mp4processor.cpp:40-61
    uint16_t accumulator = 0xFFFF;
    for (int i = 0; i < len; i++) {
        int16_t data = (int16_t)(msg[i] << 8);
        for (int j = 8; j > 0; j--) {
            if ((data ^ accumulator) & 0x8000) accumulator = ((accumulator << 1) ^ 0x1021) & 0xFFFF;
            else accumulator = (accumulator << 1) & 0xFFFF;
            data = (data << 1) & 0xFFFF;
        }
    }
    const uint16_t crc = ~((msg[len] << 8) | msg[len + 1]) & 0xFFFF;
    return (crc ^ accumulator) == 0;
}
int ref_mp4_add(ref_mp4 *m, const uint8_t *V, int *n_aus_ok) {
    static firecode_checker fc;
    static reedSolomon rs(8, 0435, 0, 1, 10);
    const int nbits = 24 * m->bitRate, RS = m->bitRate / 8;
    *n_aus_ok = 0;
    for (int i = 0; i < nbits / 8; i++) {
        uint8_t t = 0;
        for (int j = 0; j < 8; j++) t = (uint8_t)((t << 1) | (V[i * 8 + j] & 1));
        m->ring[m->fill * nbits / 8 + i] = t;
    }
    m->blocks++;
    m->fill = (m->fill + 1) % 5;
    if (m->blocks < 5) return 0;
    const int base = m->fill * nbits / 8;
    if (!fc.check(&m->ring[base])) { m->blocks = 4; return 1; }
    uint8_t rsIn[120], rsOut[110], out[110 * 48];
    for (int j = 0; j < RS; j++) {
        for (int k = 0; k < 120; k++) rsIn[k] = m->ring[(base + j + k * RS) % (RS * 120)];
        if (rs.dec(rsIn, rsOut, 135) < 0) { m->blocks = 4; return 2; }
        for (int k = 0; k < 110; k++) out[j + k * RS] = rsOut[k];
    }
    int n = 0, a[7];
    const int end = 110 * RS;
    switch (2 * ((out[2] >> 6) & 1) + ((out[2] >> 5) & 1)) {
    default:
    case 0: n = 4; a[0] = 8; a[1] = out[3] * 16 + (out[4] >> 4); a[2] = (out[4] & 0xf) * 256 + out[5];
            a[3] = out[6] * 16 + (out[7] >> 4); a[4] = end; break;
    case 1: n = 2; a[0] = 5; a[1] = out[3] * 16 + (out[4] >> 4); a[2] = end; break;
    case 2: n = 6; a[0] = 11; a[1] = out[3] * 16 + (out[4] >> 4); a[2] = (out[4] & 0xf) * 256 + out[5];
            a[3] = out[6] * 16 + (out[7] >> 4); a[4] = (out[7] & 0xf) * 256 + out[8];
            a[5] = out[9] * 16 + (out[10] >> 4); a[6] = end; break;
    case 3: n = 3; a[0] = 6; a[1] = out[3] * 16 + (out[4] >> 4); a[2] = (out[4] & 0xf) * 256 + out[5];
            a[3] = end; break;
    }
    for (int i = 0; i < n; i++) {
        const int len = a[i + 1] - a[i] - 2;
        if (a[i + 1] < a[i] || len >= 960 || len < 0) { m->blocks = 4; return 2; }
        if (au_crc(&out[a[i]], (int16_t)len)) (*n_aus_ok)++;
    }
    m->blocks = 0;
    return 3;
}

}
