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

}
