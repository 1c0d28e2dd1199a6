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
// The NCO without its 16 MB table: oscillatorTable[t] (ofdm-processor.cpp:79-81) is
// float(e^{2 pi i t / 2048000}); with t = 16000 a + 128 b + c it is the float rounding
// of A[a] (B[b] C[c]) in double (fma complex products), A[a] = e^{2 pi i a/128},
// B[b] = e^{2 pi i b/16000}, C[c] = e^{2 pi i c/2048000}: 381 double2 that fit in LDS.
// The rounded product equals the table at every one of the 2048000 indices
// (tests/cpp/test_nco.c on the host, test_gpu_parity's exhaustive check on the GPU).
constexpr int NCO_A = 0, NCO_B = 128, NCO_C = 253, NCO_N = 384, NCO_USED = 381;

struct OfdmTables {
    const float2 *osc;      // oscillatorTable[2048000] (ofdm-processor.cpp:79-81)
    const double2 *nco;     // the factor tables above, [NCO_N]
    const float2 *ref;      // PRS refTable[2048] (phasereference.cpp:40-47), natural bin order
    const float *refarg;    // refArg[18] (ofdm-decoder.cpp:71-74)
    const float2 *w2048;    // W2048^j = e^{-2 pi i j/2048}, j < 2048 (double, rounded to float)
    const int16_t *carrier_of_bin;   // [2048] carrier index of an FFT bin (mapper.cpp), -1 if none
    const int16_t *stage_of_bin;     // [2048] the demod's soft-bit stage word of an FFT bin (stage_layout.h)
    const int16_t *stage_pair;       // [768] stage word of carrier pair p (carriers 2p, 2p+1)
    int32_t *err;           // device error word: kernels OR in DABGPU_KERR_* bits
};
// outputs of the front-end kernels besides the soft bits
struct DemodAux {
    int32_t *si;            // findIndex per frame (k_demod_wg<.., true>, k_prs_wg); null: frames give block0
    float *maxv, *sumv;     // optional: findIndex's Max and sum |r|
    int16_t *snr;           // optional: get_snr of block 0 per frame
    int32_t level;          // findIndex threshold
    float2 *disp;           // optional: [out_slot][K] symbol 2's FFT at bins [0, K/2) and
                            // [T_u-1-K/2, T_u-1) -- the iqBuffer feed of processToken
                            // (ofdm-decoder.cpp:192-206)
    int32_t ring8;          // soft bits as RING8 bytes (the pipeline's ring), else int16
    int32_t fmt;            // sample format of iq (DABGPU_IQ_F32 / S16 / U8)
    int32_t disp_token;     // the symbol disp receives (ofdmDecoder's displayToken, 2 by default)
    float2 *mix;            // test hook (dabgpu_ofdm_demod_mix): [out_slot][75][T_u] the NCO-mixed
                            // FFT input of every data symbol, as the demod's FFT sees it
    float2 *spec;           // with mix: [out_slot][75][T_u] that FFT's output, natural bin order
                            // (both in absolute units: the recorded formats' scale taken out)
};
// The pipeline's soft-bit ring holds each ibits value v as the byte v + 127: processToken's
// values are (int16_t)(q * 127.0) with |q| <= 1 (ofdm-decoder.cpp:188-189; a 0/0 gives 0),
// so v + 127 lies in 0..254, and v + 127 is exactly the Viterbi's branch-metric input
// (viterbi.cpp:230-233: (int16_t)(v + 127) clamped to 0..255, a no-op on that range).
constexpr int RING8_BIAS = 127;
constexpr int KERR_FRAME = 1;      // frame descriptor outside its stream / bad NCO phase
constexpr int KERR_VITERBI = 2;    // Viterbi source outside its buffer

struct AcqJob {
    int64_t iq_base;
    int64_t start;
    int64_t end;
    int32_t local_phase;
    int32_t phase;          // coarse + fine
    int32_t attempts;       // ofdmProcessor::run's `attempts` carried in (ofdm-processor.cpp:274-314)
    int32_t scan;           // scanMode: count No_Signal_Found after > 5 failed attempts
};
struct AcqResult {
    int64_t window;
    int32_t local_phase;
    int32_t status;
    int32_t attempts;       // `attempts` after the search
    int32_t no_signal;      // No_Signal_Found emissions during the search
};

// ---- Viterbi ------------------------------------------------------------
// decision words: per chunk of DEC_WORD_STEPS trellis steps and codeword row, 64
// lanes x 32 bits, in blocks of 64 rows (one traceback wave) whose chunks are
// contiguous: dec[((row / 64 * dec_nch + chunk) * 64 + row % 64) * 64 + lane]
// (dec_word_index); rows padded to a whole block of 64
constexpr int DEC_WORD_STEPS = 30;
// mother-code positions (4 per trellis step) of one ACS branch-metric tile (two decision
// words, 60 steps): the inverse depuncturing tables hold positions within their tile
constexpr int VIT_TILE_POS = 4 * 2 * DEC_WORD_STEPS;
inline __host__ __device__ int64_t dec_rows(int n_cw) { return ((int64_t)n_cw + 63) / 64 * 64; }
inline __host__ __device__ int32_t dec_chunks(int nbits) { return (nbits + 6 + DEC_WORD_STEPS - 1) / DEC_WORD_STEPS; }
inline __host__ __device__ int64_t dec_bytes(int n_cw, int nbits) {
    return (int64_t)dec_chunks(nbits) * dec_rows(n_cw) * 64 * 4;
}
// first word of (row, chunk 0); chunk c of the row is 4096 words further on
inline __host__ __device__ int64_t dec_word_index(int64_t row, int32_t nch) {
    return ((row >> 6) * nch * 64 + (row & 63)) * 64;
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
    int32_t inv_off;        // its inverse table in VitJob::inv (input -> mother position)
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
    int32_t nsub, ncif, ring;      // subchannels, CIF slots per stream in this batch, ring frames
    const int64_t *cif0s;           // [stream] CIF index (count delivered so far) of the batch's first CIF
    const int32_t *ncifs;           // [stream] CIFs of the batch the stream delivered (<= ncif)
    const int32_t *sub_start;       // startAddr*64 per subchannel (up to 55232: int32)
    // outputs
    uint32_t *dec;                  // decision words (dec_bytes(n_cw, max nbits) bytes)
    int64_t dec_ncw;                // rows of the decision buffer: >= dec_rows(n_cw)
    int32_t dec_nch;                // chunks per row: dec_chunks(max nbits)
    uint8_t *out;
    int64_t out_stride;             // bytes per codeword
    int32_t prbs;                   // xor energy-dispersal sequence
    int32_t packed;                 // out: 8 bits per byte, msb first (else one bit per byte)
    const uint32_t *prbs_words;     // PRBS packed 32 bits per word, bit i = prbs[32w+i]
    const uint8_t *valid;           // optional per-codeword flag: 0 = skip
    int32_t ring8;                  // SRC_FIC / SRC_MSC: src holds RING8 bytes (v + 127), not int16
    // SRC_MSC / SRC_FIC: inverse depuncturing tables, Profile::frag bytes per profile at
    // Profile::inv_off (make_inv): each input's mother-code position within its 60-step
    // tile (q mod VIT_TILE_POS); null: step-major loader
    const uint8_t *inv;
};

// DAB+ superframe layer (k_dabplus.hip)
constexpr int DP_MAX_RS = 48;       // RSDims = bitRate / 8, bitRate <= 384
constexpr int DP_TAB_BYTES = 256 + 256 + 512 + 2560 + 512 + 2048 + 516;   // GF exp/log, fire, mul[10], crc, pow8, fibcrc
constexpr int FIBCRC_OFF = 256 + 256 + 512 + 2560 + 512 + 2048;   // uint16 bit contribution[256] + init effect
struct DpState {
    int32_t fill, blocks;           // blockFillIndex, blocksInBuffer (mp4processor.cpp:86-87)
};
struct DpJob {
    const uint8_t *msc;             // MSC bits of the run: [S][ncif][nsub][msc_stride]
    int32_t msc_stride, ncif, nsub, ndp, nstreams;
    int32_t packed;                 // msc holds bytes (8 bits msb first), else one bit per byte
    const int64_t *cif0s;           // [stream] CIF index of the run's first CIF slot
    const int32_t *ncifs;           // [stream] CIFs the stream delivered in the run
    const int32_t *dp_sub;          // [ndp] subchannel index of each DAB+ subchannel
    const int16_t *dp_br;           // [ndp] its bitRate
    uint8_t *ring;                  // [S][ndp][120*DP_MAX_RS] 5-CIF byte rings
    DpState *state;                 // [S][ndp]
    uint8_t *code;                  // [S][ndp][ncif] scratch: 0 fire code failed, 2 rejected, 3 decoded
    uint8_t *sf_out;                // [S][ncif][ndp][sf_stride]
    int64_t sf_stride;
    dabgpu_superframe *info;        // [S][ncif][ndp]
    const uint8_t *tabs;            // DP_TAB_BYTES: GF exp, log, fire table, alpha^i multiply, CRC
    int32_t *cand;                  // [S * ndp * ncif] queue of fire-code-passing candidates
    int32_t *ncand;                 // its length (reset per launch)
    // compact output (dabgpu_pipe_set_dabplus_compact): the superframes that complete in
    // the run, per (stream, DAB+ subchannel) in CIF order, at sf_compact[(s*ndp+dp)*kmax+k]
    // (stride sf_stride); sf_out is then the pipeline's own sparse scratch
    uint8_t *sf_compact;
    int32_t kmax;
};

// iq: samples in format fmt (DABGPU_IQ_*); frame descriptors count samples
hipError_t launch_prs_sync(hipStream_t st, const void *iq, int fmt, const dabgpu_frame *fr, int n, const OfdmTables &T,
                           int level, int32_t *si, float *mx, float *sm, bool general);
hipError_t launch_block0(hipStream_t st, const void *iq, int fmt, const dabgpu_frame *fr, int n, const OfdmTables &T,
                         int method, int16_t *corr, int16_t *snr, bool general);
// aux.si non-null: every frame is placed by its own findIndex (block0 = window +
// startIndex), reported through aux; else the descriptors' block0 / lp_data are used
hipError_t launch_demod(hipStream_t st, const void *iq, const dabgpu_frame *fr, int n, int nchunks,
                        const OfdmTables &T, int16_t *soft, float *softf, float *fcpart, bool general,
                        const DemodAux &aux);
hipError_t launch_nco_eval(hipStream_t st, const OfdmTables &T, int32_t first, int32_t n, float2 *out);
hipError_t launch_snr(hipStream_t st, const float *spec, int16_t *out);
hipError_t launch_symbol(hipStream_t st, const float *smp, int kind, const OfdmTables &T, float *spec, int16_t *ibits);
hipError_t launch_fc_reduce(hipStream_t st, const float *part, int nchunks, int n, float *out);
hipError_t launch_take_error(hipStream_t st, int32_t *err, int32_t *h_err);
hipError_t launch_front_publish(hipStream_t st, const float *part, int nchunks, int n, float *fc_d, float *h_fc,
                                const int32_t *si_d, int32_t *h_si, const int16_t *snr_d, int16_t *h_snr,
                                int32_t *err, int32_t *h_err);
hipError_t launch_acquire(hipStream_t st, const void *iq, int fmt, const AcqJob *jobs, int n, const float2 *osc,
                          AcqResult *res);
hipError_t launch_viterbi(hipStream_t st, const VitJob &job);
hipError_t launch_acs(hipStream_t st, const VitJob &job);
hipError_t launch_traceback(hipStream_t st, const VitJob &job);
hipError_t launch_acs_msc_fic(hipStream_t st, const VitJob &msc, const VitJob &fic);
hipError_t launch_traceback_msc_fic(hipStream_t st, const VitJob &msc, const VitJob &fic);
hipError_t launch_acs_msc_fic_range(hipStream_t st, const VitJob &msc, const VitJob &fic, int b0, int b1, bool with_fic);
hipError_t launch_traceback_msc_fic_range(hipStream_t st, const VitJob &msc, const VitJob &fic, int b0, int b1,
                                          bool with_fic);
hipError_t launch_fic_post(hipStream_t st, uint8_t *bits, uint8_t *crc_ok, int n_fib, const uint8_t *tabs,
                           const int32_t *slots = nullptr, bool packed = false);
hipError_t launch_dabplus(hipStream_t st, const DpJob &job);
hipError_t launch_iq_convert(hipStream_t st, int format, const void *src, int64_t n_values, float *dst);
// device -> mapped pinned host memory by `wgs` workgroups; src, dst, bytes 16-byte aligned
hipError_t launch_to_host(hipStream_t st, const void *src, void *dst, size_t bytes, int wgs);
hipError_t launch_rs(hipStream_t st, const uint8_t *in, int n, const uint8_t *tabs, uint8_t *out, int16_t *ret);

}  // namespace dab
