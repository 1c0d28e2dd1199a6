// dab_kernels.h -- host/device shared structs and kernel launchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/dabgpu.h"

namespace dab {

constexpr int TU = 2048, TS = 2552, TG = 504, TNULL = 2656, TF = 196608, K = 1536, L = 76;
constexpr int NSYM = 75;                 // data symbols per frame
constexpr int SYMBITS = 2 * K;           // 3072 soft bits per symbol
constexpr int FRAME_SOFT = NSYM * SYMBITS;
constexpr int INPUT_RATE = 2048000;

// device tables for the OFDM kernels (built on the host with the reference's
// own float expressions, see dabgpu.cpp: make_tables)
struct OfdmTables {
    const float2 *osc;      // oscillatorTable[2048000] (ofdm-processor.cpp:79-81)
    const float2 *tw;       // twiddle bases [12][64]: rows a=0..7 W2048^{n2*a}, rows 8+b W2048^{n2*8b}
    const float2 *ref_l;    // PRS refTable in FFT output lane layout [i][lane]
    const float *refarg;    // refArg[18] (ofdm-decoder.cpp:71-74)
    const float2 *w2048;    // W2048^j = e^{-2 pi i j/2048}, j < 2048 (double, rounded to float)
    const int16_t *carrier_of_bin;   // [2048] carrier index of an FFT bin (mapper.cpp), -1 if none
    int32_t *err;           // device error word: kernels OR in DABGPU_KERR_* bits
};
constexpr int FRAME_SI_ON_DEVICE = 2;   // dabgpu_frame.flags bit (pipeline-internal)
constexpr int KERR_FRAME = 1;      // frame descriptor outside its stream / bad NCO phase
constexpr int KERR_VITERBI = 2;    // Viterbi source outside its buffer

struct AcqJob {
    int64_t iq_base;
    int64_t start;
    int64_t end;
    int32_t local_phase;
    int32_t phase;          // coarse + fine
};
struct AcqResult {
    int64_t window;
    int32_t local_phase;
    int32_t status;
    int32_t attempts;
    int32_t pad;
};

// ---- Viterbi ------------------------------------------------------------
// decision words: per chunk of DEC_WORD_STEPS trellis steps and codeword row, 64
// lanes x 32 bits (k_viterbi.hip: dec[(chunk * dec_ncw + row) * 64 + lane]); rows
// padded to a whole traceback wave of 64
constexpr int DEC_WORD_STEPS = 30;
inline __host__ __device__ int64_t dec_rows(int n_cw) { return ((int64_t)n_cw + 63) / 64 * 64; }
inline __host__ __device__ int64_t dec_bytes(int n_cw, int nbits) {
    return (int64_t)((nbits + 6 + DEC_WORD_STEPS - 1) / DEC_WORD_STEPS) * dec_rows(n_cw) * 64 * 4;
}

// depuncturing profile: up to 4 (L_i, PI_i) segments + the 24-bit PI_X tail
// (deconvolve.cpp:172-237, fic-handler.cpp:254-288)
struct Profile {
    int32_t nbits;          // decoded bits N; trellis steps N+6
    int32_t nseg;           // 0 = no puncturing (mother code given directly)
    uint32_t mask[4];       // PI vectors as 32-bit masks (bit j = P_Code[j])
    int32_t blk_end[4];     // cumulative 128-bit blocks at end of segment
    int32_t in_base[5];     // input soft-bit index at segment start / tail start
    uint32_t tail_mask;     // PI_X (24 bits)
    int32_t frag;           // punctured input length (fragment size)
};

enum SrcKind : int32_t {
    SRC_MOTHER = 0,         // contiguous depunctured stream, stride 4*(N+6)
    SRC_FRAG = 1,           // contiguous punctured fragments, stride frag_stride
    SRC_FIC = 2,            // FIC blocks inside the demod soft-bit buffer
    SRC_MSC = 3,            // MSC subchannels with 16-CIF time de-interleave from the ring
};

struct VitJob {
    int32_t kind;
    int32_t n_cw;
    const int16_t *src;
    int64_t src_len;        // elements readable from src (bounds check)
    int32_t *err;           // device error word
    int64_t src_stride;     // SRC_MOTHER / SRC_FRAG: elements per codeword
    const Profile *prof;    // per-profile table
    const int32_t *cw_prof; // SRC_FRAG: profile per codeword; else null (profile 0 / by subch)
    // SRC_FIC: codeword = 4*i + blk over slots[i]
    const int32_t *slots;
    // SRC_MSC: codeword = ((stream * ncif) + c) * nsub + sub
    int32_t nsub, ncif, ring;      // subchannels, CIFs in this batch, ring frames
    int64_t cif0;                   // global CIF index of the batch's first CIF (per stream, same for all)
    int32_t first_slot;             // ring slot of the batch's first frame
    const int32_t *sub_start;       // startAddr*64 per subchannel (up to 55232: int32)
    // outputs
    uint32_t *dec;                  // decision words (dec_bytes(n_cw, max nbits) bytes)
    int64_t dec_ncw;                // rows of the decision buffer: >= dec_rows(n_cw)
    uint8_t *out;
    int64_t out_stride;             // bytes per codeword
    int32_t prbs;                   // xor energy-dispersal sequence
    const uint32_t *prbs_words;     // PRBS packed 32 bits per word, bit i = prbs[32w+i]
    const uint8_t *valid;           // optional per-codeword flag: 0 = skip
};

// DAB+ superframe layer (k_dabplus.hip)
constexpr int DP_MAX_RS = 48;       // RSDims = bitRate / 8, bitRate <= 384
constexpr int DP_TAB_BYTES = 256 + 256 + 512 + 2560 + 512 + 2048;   // GF exp/log, fire, mul[10], crc, pow8
struct DpState {
    int32_t fill, blocks;           // blockFillIndex, blocksInBuffer (mp4processor.cpp:86-87)
};
struct DpJob {
    const uint8_t *msc;             // MSC bits of the run: [S][ncif][nsub][msc_stride]
    int32_t msc_stride, ncif, nsub, ndp, nstreams;
    int64_t cif0;
    const int32_t *dp_sub;          // [ndp] subchannel index of each DAB+ subchannel
    const int16_t *dp_br;           // [ndp] its bitRate
    uint8_t *ring;                  // [S][ndp][120*DP_MAX_RS] 5-CIF byte rings
    DpState *state;                 // [S][ndp]
    uint8_t *code;                  // [S][ndp][ncif] scratch: 0 fire code failed, 2 rejected, 3 decoded
    uint8_t *sf_out;                // [S][ncif][ndp][sf_stride]
    int64_t sf_stride;
    dabgpu_superframe *info;        // [S][ncif][ndp]
    const uint8_t *tabs;            // DP_TAB_BYTES: GF exp, log, fire table, alpha^i multiply, CRC
};

hipError_t launch_prs_sync(hipStream_t st, const float *iq, const dabgpu_frame *fr, int n, const OfdmTables &T,
                           int level, int32_t *si, float *mx, float *sm, bool general);
hipError_t launch_block0(hipStream_t st, const float *iq, const dabgpu_frame *fr, int n, const OfdmTables &T,
                         int16_t *corr, bool general);
// si (optional): per-frame startIndex from k_prs_sync, used by frames flagged
// FRAME_SI_ON_DEVICE (block0 and lp_data derived on the device)
hipError_t launch_demod(hipStream_t st, const float *iq, const dabgpu_frame *fr, int n, int nchunks,
                        const OfdmTables &T, int16_t *soft, float *softf, float *fcpart, bool general,
                        const int32_t *si = nullptr);
hipError_t launch_fc_reduce(hipStream_t st, const float *part, int nchunks, int n, float *out);
hipError_t launch_acquire(hipStream_t st, const float *iq, const AcqJob *jobs, int n, const float2 *osc,
                          AcqResult *res);
hipError_t launch_viterbi(hipStream_t st, const VitJob &job);
hipError_t launch_acs(hipStream_t st, const VitJob &job);
hipError_t launch_traceback(hipStream_t st, const VitJob &job);
hipError_t launch_acs_msc_fic(hipStream_t st, const VitJob &msc, const VitJob &fic);
hipError_t launch_traceback_msc_fic(hipStream_t st, const VitJob &msc, const VitJob &fic);
hipError_t launch_fic_post(hipStream_t st, uint8_t *bits, uint8_t *crc_ok, int n_fib);
hipError_t launch_dabplus(hipStream_t st, const DpJob &job);
hipError_t launch_iq_convert(hipStream_t st, int format, const void *src, int64_t n_values, float *dst);
hipError_t launch_rs(hipStream_t st, const uint8_t *in, int n, const uint8_t *tabs, uint8_t *out, int16_t *ret);

}  // namespace dab
