/*
 * dabgpu.h -- C ABI of the MI355X-native DAB Mode-I demod/decode path.
 *
 * Plain C: pointers, sizes and PODs only (no HIP or torch types), so a C++
 * drop-in for sdr-j-dab's ofdmProcessor / ficHandler / mscHandler, a ctypes
 * or a cgo binding can all call it.  Every entry point names the reference
 * interface it replaces (paths relative to the sdr-j-dab v0.997 tree).
 *
 * Conventions
 *  - return value: 0 on success, a negative DABGPU_E* code on failure; the
 *    message of the last failure on this thread is dabgpu_last_error().
 *    No C++ exception crosses this boundary.
 *  - "_d" pointers are device (HBM) pointers obtained from dabgpu_alloc or
 *    any HIP allocation on the context's device; "_h" pointers are host.
 *  - every device-side call is asynchronous on the context's stream;
 *    dabgpu_sync() waits.  Calls that return host data synchronise.
 *  - one context per calling thread (contexts are independent streams).
 *  - data formats follow the reference: IQ is interleaved cf32 (re, im)
 *    scaled to about +-1 (virtual-input.h:51-70); soft bits are int16 in
 *    [-127, 127] (ofdm-decoder.cpp:186-189); decoded bits are one bit per
 *    uint8 (viterbi.cpp:240-241).
 */
#ifndef DABGPU_H
#define DABGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DABGPU_ABI_VERSION 7

/* error codes */
#define DABGPU_OK          0
#define DABGPU_E_ARG      -1   /* invalid argument / shape */
#define DABGPU_E_HIP      -2   /* HIP runtime error */
#define DABGPU_E_NODEV    -3   /* no usable gfx950 device */
#define DABGPU_E_NOMEM    -4
#define DABGPU_E_UNSUP    -5   /* configuration the reference does not define */
#define DABGPU_E_STATE    -6   /* call out of sequence */
#define DABGPU_E_BOUNDS   -7   /* a kernel refused a descriptor that points outside its stream */

/* Mode-I geometry (gui.cpp:1361-1371) */
#define DABGPU_TU     2048
#define DABGPU_TS     2552
#define DABGPU_TG     504
#define DABGPU_TNULL  2656
#define DABGPU_TF     196608
#define DABGPU_K      1536
#define DABGPU_L      76
#define DABGPU_CIF_BITS 55296

typedef struct dabgpu_ctx dabgpu_ctx;

/* Subchannel of the MSC, as produced by the FIB parser (dab-constants.h:151-176,
 * audiodata/packetdata: startAddr, length in CUs, uepFlag, protLevel, bitRate).
 * uepFlag == 0 selects UEP (deconvolve.cpp:130); otherwise protLevel carries
 * 0100|level (EEP-A) or 0200|level (EEP-B). */
typedef struct {
    int16_t startAddr;
    int16_t length;
    int16_t bitRate;
    int16_t protLevel;
    int16_t uepFlag;
    int16_t flags;          /* DABGPU_SUBCH_DABPLUS: feed the DAB+ superframe layer */
} dabgpu_subch;
#define DABGPU_SUBCH_DABPLUS 1
#define DABGPU_SUBCH_RAW     2   /* dabgpu_msc_deconvolve: no energy dispersal (the bare
                                    uep_/eep_deconvolve::deconvolve output) */

/* One CIF of one DAB+ subchannel through mp4Processor::addtoFrame
 * (mp4processor.cpp:107-145) and, when five blocks are buffered and the fire
 * code holds, processSuperframe (:146-292). */
typedef struct {
    int8_t  status;         /* -1 CIF not delivered (de-interleaver warm-up), 0 fewer than 5
                               blocks buffered, 1 fire code failed, 2 superframe rejected
                               (RS failure or impossible AU table), 3 superframe decoded */
    int8_t  num_aus;        /* AUs in the superframe (2, 3, 4 or 6) */
    int16_t n_corrected;    /* RS symbols corrected (sum over the RSDims codewords) */
    int16_t au_start[7];    /* au_start[0..num_aus] */
    uint8_t au_crc_ok;      /* bit i: AU i passed dabPlus_crc */
    uint8_t reserved;       /* compact output: the superframe's slot (0xFF: none); else 0 */
} dabgpu_superframe;

/* Per-frame front-end parameters (ofdm-processor.cpp:344-446), one per
 * (stream, frame).  Sample indices are relative to the stream's base.
 * The NCO follows getSamples: for the k-th sample read in a segment
 * (k = 1, 2, ...), localPhase = (lp - k*phase) mod 2048000 and the
 * sample is multiplied by oscillatorTable[localPhase]. */
typedef struct {
    int64_t iq_base;    /* sample offset of the stream in the IQ buffer */
    int64_t n_samples;  /* samples of this stream readable from iq_base (bounds check) */
    int64_t window;     /* first sample of the T_u sync window (SyncOnPhase) */
    int64_t block0;     /* first sample of block 0 = window + startIndex */
    int32_t lp_window;  /* localPhase before the window's first sample */
    int32_t phase_a;    /* coarse+fine while reading window and PRS (segment A) */
    int32_t lp_data;    /* localPhase before the first data-symbol sample */
    int32_t phase_b;    /* coarse+fine while reading symbols 1..75 (segment B) */
    int32_t out_slot;   /* output frame slot in the soft-bit buffer */
    int32_t flags;      /* bit0: run coarse AFC (f2Correction) in block0 */
} dabgpu_frame;

/* ---- host-side tables (no device needed; for pinning against the reference) --
 *   DABGPU_TABLE_PRS     float2[2048] refTable (phasereference.cpp:40-47), natural order
 *   DABGPU_TABLE_MAPPER  int16[1536]  permVector::mapIn (mapper.cpp:33-117)
 *   DABGPU_TABLE_REFARG  float[18]    refArg (ofdm-decoder.cpp:71-74)
 *   DABGPU_TABLE_OSC     float2[2048000] oscillatorTable (ofdm-processor.cpp:79-81)
 *   DABGPU_TABLE_NCO     double2[384] the factor tables the kernels rebuild
 *                        oscillatorTable from (128 e^{2pi i a/128}, 125 e^{2pi i b/16000},
 *                        128 e^{2pi i c/2048000}, 3 zero) */
#define DABGPU_TABLE_PRS    1
#define DABGPU_TABLE_MAPPER 2
#define DABGPU_TABLE_REFARG 3
#define DABGPU_TABLE_OSC    4
#define DABGPU_TABLE_NCO    5
int dabgpu_host_table(int which, void *out_h, size_t bytes);
/* The depuncturing profile the decoder uses for a subchannel (deconvolve.cpp:142-366;
 * uep_deconvolve's unknown-profile fallback to table row 1, :148-151): decoded bits,
 * fragment size consumed, and the non-empty (L_i blocks of 128, PI_i) segments in
 * order.  Returns 0, 1 when the UEP (bitRate, level) is not in the table (fallback),
 * DABGPU_E_UNSUP when the protection is undefined. */
int dabgpu_subch_profile(const dabgpu_subch *s, int32_t *nbits, int32_t *frag_size, int32_t *nseg,
                         int32_t *L /*[4]*/, int32_t *PI /*[4]*/);

/* ---- context ---------------------------------------------------------- */
int         dabgpu_abi_version(void);
const char *dabgpu_last_error(void);
int         dabgpu_device_count(void);
int         dabgpu_ctx_create(int device, dabgpu_ctx **out);
int         dabgpu_ctx_destroy(dabgpu_ctx *ctx);
int         dabgpu_sync(dabgpu_ctx *ctx);
int         dabgpu_alloc(dabgpu_ctx *ctx, size_t bytes, void **dptr);
int         dabgpu_free(dabgpu_ctx *ctx, void *dptr);
int         dabgpu_memcpy_h2d(dabgpu_ctx *ctx, void *dst_d, const void *src_h, size_t bytes);
int         dabgpu_memcpy_d2h(dabgpu_ctx *ctx, void *dst_h, const void *src_d, size_t bytes);
int         dabgpu_memset_d(dabgpu_ctx *ctx, void *dst_d, int value, size_t bytes);
/* page-locked host memory (DMA without the pageable bounce: dabgpu_pipe_fetch targets) */
int         dabgpu_host_alloc(dabgpu_ctx *ctx, size_t bytes, void **h);
int         dabgpu_host_free(dabgpu_ctx *ctx, void *h);
/* device-to-device copy on the context stream (asynchronous; regions must not overlap) */
int         dabgpu_memcpy_d2d(dabgpu_ctx *ctx, void *dst_d, const void *src_d, size_t bytes);
/* HIP events on the context stream, for timing (ms between two marks) */
int         dabgpu_event_record(dabgpu_ctx *ctx, int slot);
/* device-side bounds violations flagged by kernels since the last call (syncs; clears) */
int         dabgpu_kernel_errors(dabgpu_ctx *ctx);
int         dabgpu_event_elapsed(dabgpu_ctx *ctx, int slot_a, int slot_b, float *ms);

/* ---- recorded IQ formats ---------------------------- */
/* Convert device-resident recorded samples to the interleaved cf32 IQ every OFDM
 * entry point reads, with the reference file readers' scaling:
 *   DABGPU_IQ_U8   .raw: rawFiles::getSamples (rawfiles.cpp:100-118),
 *                  I/Q = float(x - 128) / 128.0
 *   DABGPU_IQ_S16  .sdr: 2-channel PCM16 WAV at 2.048 MHz, wavFiles (wavfiles.cpp:
 *                  64-69, readBuffer) through libsndfile's sf_readf_float: x / 32768
 * n_pairs I/Q pairs: src_d holds 2*n_pairs values, iq_d receives 2*n_pairs floats.
 * Asynchronous on the context stream (dabgpu_sync to wait). */
#define DABGPU_IQ_F32  0   /* interleaved cf32: what every entry point reads by default */
#define DABGPU_IQ_U8   1
#define DABGPU_IQ_S16  2
int dabgpu_iq_convert(dabgpu_ctx *ctx, int format, const void *src_d, int64_t n_pairs, float *iq_d);

/* ---- OFDM front end (L3) ---------------------------------------------- */

/* phaseReference::findIndex batched (phasereference.cpp:60-88): for each of n
 * frames, FFT of the NCO-mixed T_u window, x conj(PRS), IFFT, argmax |.|.
 * start_index[i] follows the reference: argmax, or -|Max/mean|-1 (truncated)
 * when Max < level*mean.  maxv/sumv (optional) receive Max and sum |.|. */
int dabgpu_prs_sync(dabgpu_ctx *ctx, const float *iq_d, const dabgpu_frame *frames_d, int n,
                    int16_t level, int32_t *start_index_d, float *maxv_d, float *sumv_d);

/* ofdmDecoder::processBlock_0 batched (ofdm-decoder.cpp:85-162): FFT of block 0,
 * snr_d[i] (optional) = get_snr (ofdm-decoder.cpp:212-230), and when
 * frames[i].flags&1 the coarse offset estimate of freqSyncMethod `method`
 * (0 getMiddle, 1 phase-difference correlation, 2 pattern match), else 0. */
int dabgpu_block0(dabgpu_ctx *ctx, const float *iq_d, const dabgpu_frame *frames_d, int n, int method,
                  int16_t *correction_d, int16_t *snr_d);

/* ofdmDecoder::processToken for symbols 1..75 of n frames (ofdm-decoder.cpp:167-190):
 * FFT, x conj(previous symbol), frequency de-interleave (mapper.cpp:115),
 * ibits = (int16)(-re/(|re|+|im|)*127).  Output layout
 *   softbits_d[out_slot][75][3072]  (FIC = symbols 1..3, CIF c = symbols 4+18c..21+18c)
 * softf_d (optional, same layout, float -re/|.|, -im/|.|) for parity tests.
 * freqcorr_d (optional) float2[n]: sum over the frame of x[i]*conj(x[i-T_u]),
 * i in [T_u, T_s) (ofdm-processor.cpp:424-438), in unspecified float order. */
int dabgpu_ofdm_demod(dabgpu_ctx *ctx, const float *iq_d, const dabgpu_frame *frames_d, int n,
                      int16_t *softbits_d, float *softf_d, float *freqcorr_d);

/* The north-star fused front end, one workgroup per frame (k_demod_wg<.., SYNC>):
 * findIndex on the frame's T_u window (phasereference.cpp:60-88, threshold `level`;
 * start_index_d[i] as dabgpu_prs_sync), the frame placed at block0 = window +
 * startIndex with lp_data following getSamples (ofdm-processor.cpp:344-368),
 * get_snr of block 0 (snr_d, optional, ofdm-decoder.cpp:93) and processToken x 75
 * as dabgpu_ofdm_demod.  frames[i].block0 / lp_data are ignored; a frame whose
 * findIndex fails or whose symbols lie past n_samples is skipped (no soft bits). */
int dabgpu_ofdm_sync_demod(dabgpu_ctx *ctx, const float *iq_d, const dabgpu_frame *frames_d, int n, int16_t level,
                           int32_t *start_index_d, int16_t *snr_d, int16_t *softbits_d, float *softf_d,
                           float *freqcorr_d);

/* The kernels' NCO: oscillatorTable[first .. first+n-1] as the front-end kernels
 * compute it (float2 into out_d) -- for checking it against the table exhaustively. */
int dabgpu_nco_eval(dabgpu_ctx *ctx, int32_t first, int32_t n, float *out_d);
/* Test hook of the fused demod's NCO and FFT (getSamples' v *= oscillatorTable[localPhase],
 * ofdm-processor.cpp:76-81,202-226; fft.cpp:53-121): the demod with `chunks` workgroups per
 * frame (1: one recurrence over all 75 symbols, as the pipeline runs C3) that also writes
 * every data symbol's mixed FFT input, mix_d[out_slot][75][2048] cf32 (the samples
 * [T_g, T_s) of symbol l after the NCO), and that FFT's output, spec_d[out_slot][75][2048]
 * in natural bin order, both in absolute units (format's scale taken out, exactly), for
 * comparison with the reference's table and with the transform restated.
 *   start_index_d == NULL: the operator form (dabgpu_ofdm_demod: cf32 in, frames give
 *     block0 / lp_data, int16 soft bits [out_slot][75][3072] into softbits_d);
 *   start_index_d != NULL: the streaming pipeline's instantiation -- findIndex on the
 *     window (threshold `level`, as dabgpu_ofdm_sync_demod), samples read as `format`
 *     (DABGPU_IQ_F32 / S16 / U8) and converted in the loads, RING8 soft-bit bytes
 *     (ibits + 127, [out_slot][75][3072]) into softbits_d. */
int dabgpu_ofdm_demod_mix(dabgpu_ctx *ctx, const void *iq_d, int format, const dabgpu_frame *frames_d, int n,
                          int chunks, int16_t level, int32_t *start_index_d, float *mix_d, float *spec_d,
                          void *softbits_d);

/* One symbol at a time (the reference's ofdmDecoder call pattern, ofdm-decoder.cpp:
 * 85-190), samples already mixed by the caller: kind 0 = block 0 (samples_d holds
 * T_u samples; its spectrum becomes the phase reference), kind 1 = a data symbol
 * (T_s samples; ibits_d[3072] = processToken's soft bits against the stored
 * spectrum, which then becomes this symbol's).  spectrum_d: cf32[2048] state. */
int dabgpu_ofdm_symbol(dabgpu_ctx *ctx, const float *samples_d, int kind, float *spectrum_d, int16_t *ibits_d);

/* ofdmDecoder::get_snr (ofdm-decoder.cpp:212-230) of a T_u-point spectrum in natural
 * bin order (cf32[2048], device): get_db(mean |X| of the signal bins) - get_db(mean |X|
 * of the noise bins) into snr_d[0]. */
int dabgpu_get_snr(dabgpu_ctx *ctx, const float *spectrum_d, int16_t *snr_d);

/* ---- channel decoding (L4) -------------------------------------------- */

/* viterbi::deconvolve batched (viterbi.cpp:225-242): n_cw codewords of
 * 4*(nbits+6) depunctured soft bits -> nbits decoded bits each. */
int dabgpu_viterbi(dabgpu_ctx *ctx, const int16_t *in_d, int n_cw, int nbits, uint8_t *out_d);

/* ficHandler::process_ficInput batched (fic-handler.cpp:241-321): n blocks of
 * 2304 soft bits (contiguous, block stride 2304) -> 768 bits after energy
 * dispersal, with each FIB's CRC field inverted by the check exactly as
 * check_CRC_bits leaves it (dab-constants.h:316-317); crc_ok_d[3*n]. */
int dabgpu_fic_decode(dabgpu_ctx *ctx, const int16_t *fic_soft_d, int n, uint8_t *bits_d,
                      uint8_t *crc_ok_d);

/* FIC blocks straight from a demod soft-bit buffer: frames slots[0..n_frames)
 * each give 4 blocks (symbols 1..3 of the slot). Output [n_frames][4][768]. */
int dabgpu_fic_decode_frames(dabgpu_ctx *ctx, const int16_t *softbits_d, const int32_t *slots_h,
                             int n_frames, uint8_t *bits_d, uint8_t *crc_ok_d);

/* uep_/eep_deconvolve::deconvolve + energy dispersal (deconvolve.cpp:172-237,
 * 325-366; dab-concurrent.cpp:183-190; no dispersal with DABGPU_SUBCH_RAW) for n_cw codewords whose
 * fragmentSize = length*64 soft bits are given contiguous (already
 * time-de-interleaved), one subchannel description per codeword.
 * Output bits_d[n_cw][24*max_bitRate] (row stride out_stride bytes). */
/* reedSolomon::dec(rsIn, rsOut, 135) batched (reed-solomon.cpp:129-141; the
 * RS(255,245) code of mp4processor.cpp:74 shortened to (120,110)): n codewords of
 * 120 bytes -> 110 corrected bytes each; ret_d[i] = symbols corrected or -1. */
int dabgpu_rs_decode(dabgpu_ctx *ctx, const uint8_t *in_d, int n, uint8_t *out_d, int16_t *ret_d);

int dabgpu_msc_deconvolve(dabgpu_ctx *ctx, const int16_t *frag_d, int64_t frag_stride,
                          const dabgpu_subch *subch_h, int n_cw, uint8_t *bits_d, int64_t out_stride);

/* ---- streaming pipeline (ofdmProcessor::run + ficHandler + mscHandler) ---
 * n_streams independent ensembles; each call decodes n_frames frames per
 * stream.  Sync, AFC, DQPSK references and the 16-CIF time de-interleaver
 * state (dab-concurrent.cpp:162-175: the first 16 CIFs are warm-up) are
 * carried across calls.  subch lists the subchannels decoded for every
 * stream (the reference decodes one selected subchannel; this decodes all). */
typedef struct dabgpu_pipe dabgpu_pipe;
typedef struct {
    int32_t n_streams;
    int32_t n_frames;          /* frames per dabgpu_pipe_run call */
    int32_t n_subch;
    int16_t threshold;         /* findIndex level (gui.cpp:98-99, default 3) */
    int16_t freq_sync_method;  /* processBlock_0's coarse AFC: 0 getMiddle, 1 phase-difference
                                  correlation (main.cpp:91 default), 2 pattern match
                                  (ofdm-decoder.cpp:103-161) */
    const dabgpu_subch *subch;
} dabgpu_pipe_cfg;

typedef struct {
    int64_t next_pos;          /* stream index of the next window (SyncOnPhase) */
    int32_t local_phase;
    int32_t coarse;            /* coarseCorrector */
    int16_t fine;              /* fineCorrector */
    int16_t f2correction;
    int16_t prev1, prev2;
    int32_t synced;
    int64_t cif_count;         /* CIFs delivered to the MSC so far */
    int32_t last_start_index;
    int32_t resyncs;           /* sync losses (findIndex failed: goto notSynced, ofdm-processor.cpp:354-357) */
    int32_t acquisitions;      /* null-symbol searches completed (SyncOnNull..SyncOnEndNull) */
    int32_t attempts;          /* the reference's `attempts` counter (ofdm-processor.cpp:274-314) */
    int32_t no_signal;         /* No_Signal_Found emissions (scan mode, > 5 failed attempts) */
    int32_t frames_run;        /* frames this stream committed in the last dabgpu_pipe_run */
    int32_t acquiring;         /* 1: a background null search (DABGPU_CTL_ACQ_ASYNC) is running */
} dabgpu_stream_state;

/* Per-frame record of the last run (the observables ofdmProcessor / ofdmDecoder
 * report to the GUI, ofdm-processor.cpp:172-175,344-446, ofdm-decoder.cpp:93-97). */
typedef struct {
    int64_t window;            /* first sample of the frame's T_u sync window */
    int32_t start_index;       /* findIndex result */
    int32_t coarse;            /* coarseCorrector used for symbols 1..75 */
    int16_t fine;              /* fineCorrector used for symbols 1..75 */
    int16_t correction;        /* processBlock_0's return (0 when f2Correction was off) */
    int16_t snr;               /* get_snr of block 0 (ofdm-decoder.cpp:212-230), before the IIR */
    int16_t committed;         /* 1: the frame was decoded in this run */
} dabgpu_frame_info;

int dabgpu_pipe_create(dabgpu_ctx *ctx, const dabgpu_pipe_cfg *cfg, dabgpu_pipe **out);
int dabgpu_pipe_destroy(dabgpu_pipe *p);
/* Acquire (notSynced/SyncOnNull/SyncOnEndNull, ofdm-processor.cpp:274-338)
 * every stream not yet synchronised from sample start_h[s] of its IQ (device,
 * stream s at sample stream_stride*s of iq_d, n_avail_h[s] samples).  Optional:
 * dabgpu_pipe_run acquires unsynchronised streams itself, from their current
 * position (sample 0 for a new pipeline). */
int dabgpu_pipe_acquire(dabgpu_pipe *p, const void *iq_d, int64_t stream_stride,
                        const int64_t *start_h, const int64_t *n_avail_h);
/* Decode the next n_frames frames of every stream, as ofdmProcessor::run does:
 * a stream whose findIndex fails goes back to the null-symbol search from where it
 * is (goto notSynced, ofdm-processor.cpp:354-357) and continues with the frames
 * after it.  Outputs (device memory, or dabgpu_host_alloc memory through its device
 * address: the decoders then write across PCIe themselves -- zero copy, slower than
 * dabgpu_pipe_fetch behind the decoding on MI355X; not for a pipeline with DAB+
 * subchannels, whose layer reads msc_bits_d back):
 *   fic_bits_d  [n_streams][n_frames][4][768] (DABGPU_PACK_FIC: [4][96] FIB bytes),
 *               fic_crc_d [n_streams][n_frames][12]
 *               (frame f of stream s: its f-th frame of this run; frames past
 *               dabgpu_stream_state.frames_run have CRC flags 0)
 *   msc_bits_d  [n_streams][4*n_frames][n_subch][msc_stride] (24*bitRate used)
 *   msc_valid_h [n_streams][4*n_frames] (host, optional): 1 where the stream
 *               delivered the CIF and it is past the 16-CIF warm-up.
 * Returns 0 when every stream decoded n_frames frames, DABGPU_E_STATE when one
 * ran out of samples (its decoded frames are still delivered; see
 * dabgpu_pipe_state). */
int dabgpu_pipe_run(dabgpu_pipe *p, const void *iq_d, int64_t stream_stride, const int64_t *n_avail_h,
                    uint8_t *fic_bits_d, uint8_t *fic_crc_d, uint8_t *msc_bits_d, int32_t msc_stride,
                    uint8_t *msc_valid_h);
/* DAB+ superframe layer for the CIFs of the last dabgpu_pipe_run (call once per
 * run, after it): mp4Processor::addtoFrame/processSuperframe
 * (mp4processor.cpp:107-292) for every subchannel flagged DABGPU_SUBCH_DABPLUS,
 * state (5-CIF byte ring, blockFillIndex, blocksInBuffer) carried across runs.
 * Outputs (device), DAB+ subchannels numbered in cfg order:
 *   sf_bytes_d [n_streams][4*n_frames][n_dabplus][sf_stride]: the 110*RSDims
 *              corrected superframe bytes where info.status == 3
 *   info_d     [n_streams][4*n_frames][n_dabplus] */
int dabgpu_pipe_dabplus(dabgpu_pipe *p, uint8_t *sf_bytes_d, int32_t sf_stride, dabgpu_superframe *info_d);
/* Compact superframe bytes for the following dabgpu_pipe_dabplus calls (on = 1): only the
 * superframes that complete in the run are stored, per (stream, DAB+ subchannel) in CIF
 * order -- sf_bytes_d [n_streams][n_dabplus][DABGPU_SF_SLOTS(n_frames)][sf_stride], the
 * k-th at slot k, and its info record's `reserved` byte is k (0xFF for records without
 * bytes).  One CIF in five carries a superframe, so this is the form to copy to the host
 * (dabgpu_pipe_fetch).  At most 512 frames per run. */
#define DABGPU_SF_SLOTS(n_frames) ((4 * (n_frames) + 4) / 5 + 1)
int dabgpu_pipe_set_dabplus_compact(dabgpu_pipe *p, int on);
/* Sample format of the streams dabgpu_pipe_acquire / dabgpu_pipe_run read (default
 * DABGPU_IQ_F32): DABGPU_IQ_S16 (interleaved int16, the .sdr recording's PCM16) or
 * DABGPU_IQ_U8 (interleaved u8, the .raw recording / dabstick) are converted exactly
 * in the kernels' sample loads, with the file readers' scaling (see dabgpu_iq_convert),
 * so the decode equals that of the converted cf32 stream; the stream stride and
 * n_avail stay in samples.  Takes effect at the next call. */
int dabgpu_pipe_set_iq_format(dabgpu_pipe *p, int format);
/* dabgpu_pipe_state takes a finished background null search's results first, so
 * st->acquiring is 0 once the search no longer reads iq_d. */
int dabgpu_pipe_state(dabgpu_pipe *p, int stream, dabgpu_stream_state *st);
/* [n_streams][n_frames] records of the last dabgpu_pipe_run */
int dabgpu_pipe_frame_info(dabgpu_pipe *p, dabgpu_frame_info *info_h);
/* ofdmProcessor's control methods, for one stream (stream = -1: every stream):
 *   DABGPU_CTL_RESET        reset(): fine = coarse = 0, f2Correction on (ofdm-processor.cpp:476-479)
 *   DABGPU_CTL_COARSE_ON    coarseCorrectorOn(): f2Correction on, coarse = 0 (:498-501)
 *   DABGPU_CTL_COARSE_OFF   coarseCorrectorOff() (:503-505)
 *   DABGPU_CTL_SCAN_ON/OFF  set_scanMode(bool) (:507-509): count No_Signal_Found
 *   DABGPU_CTL_RESYNC       drop sync: the next run searches the null symbol again from
 *                           the stream's current position (goto notSynced)
 *   DABGPU_CTL_ACQ_ASYNC    (default since ABI 6; stream ignored) a stream that needs the null
 *                           search after it had been synchronised -- a sync loss,
 *                           ofdm-processor.cpp:354-357 -- gets it in the background on a
 *                           low-priority stream while the run goes on without it; the first
 *                           run after the search finished continues that stream from where it
 *                           found the null (its frames are the same, delivered later: it
 *                           decodes fewer than n_frames in the runs it misses, with
 *                           DABGPU_OK).  A stream's first search (before any frame) stays
 *                           inside the run.  iq_d must stay valid until the search ends
 *                           (dabgpu_stream_state.acquiring, or dabgpu_pipe_acquire_wait).
 *                           dabgpu_pipe_sync does not wait for a background search; the
 *                           other control ops do (its result is applied first, so the
 *                           control is the last word)
 *   DABGPU_CTL_ACQ_SYNC     the reference's order: the run waits for every search and
 *                           delivers n_frames (a one-ensemble caller loses nothing by it)
 *   DABGPU_CTL_INJECT_BOUNDS fault injection (stream ignored): the next run's MSC decoder
 *                           is handed a subchannel offset past the soft-bit ring; its
 *                           kernels refuse it (erasures read instead: the depunctured
 *                           value 0, RING8 byte 127), and dabgpu_pipe_sync or
 *                           the next run reports DABGPU_E_BOUNDS once -- the error path of
 *                           the back-end streams, for tests */
#define DABGPU_CTL_RESET      1
#define DABGPU_CTL_COARSE_ON  2
#define DABGPU_CTL_COARSE_OFF 3
#define DABGPU_CTL_SCAN_ON    4
#define DABGPU_CTL_SCAN_OFF   5
#define DABGPU_CTL_RESYNC     6
#define DABGPU_CTL_ACQ_ASYNC  7
#define DABGPU_CTL_ACQ_SYNC   8
#define DABGPU_CTL_INJECT_BOUNDS 9
int dabgpu_pipe_control(dabgpu_pipe *p, int stream, int op);
/* Wait until everything the pipeline enqueued is done.  The FIC/MSC/DAB+ outputs
 * of run r are written by back-end stream r & 1 (overlapping run r+1's OFDM front
 * end and channel decoding): call this before reading them, and give run r+1
 * output buffers other than run r's unless this was called in between.  Also
 * reports a kernel that refused out-of-bounds work (DABGPU_E_BOUNDS). */
int dabgpu_pipe_sync(dabgpu_pipe *p);
/* Wait for a background null search (DABGPU_CTL_ACQ_ASYNC) in flight and apply its
 * result; afterwards no search reads iq_d.  0 when none is in flight. */
int dabgpu_pipe_acquire_wait(dabgpu_pipe *p);
/* per-stage kernel time (HIP events on each stage's stream, no synchronisation added):
 * dabgpu_pipe_set_profiling(p, 1) times the last dabgpu_pipe_run, (p, 2) every run
 * since the call (summed; launches counts them); 0 turns it off.  Mode 3 is mode 2
 * with every timed stage run alone (the device drained before and after its launch):
 * per-kernel times without the overlap of the front end and the channel decoders,
 * for rooflines -- slower, never for throughput.  set_profiling waits for the
 * pipeline's streams; dabgpu_pipe_timing waits for the recorded work. */
#define DABGPU_STAGE_PRS      0   /* k_prs_sync   (findIndex)          */
#define DABGPU_STAGE_BLOCK0   1   /* k_block0     (processBlock_0 AFC) */
#define DABGPU_STAGE_DEMOD    2   /* k_demod      (processToken x 75)  */
#define DABGPU_STAGE_FIC      3   /* FIC Viterbi + CRC (CRC only when the run also
                                     decodes MSC: the FIC's Viterbi then shares the
                                     MSC's ACS and traceback launches)  */
#define DABGPU_STAGE_MSC_ACS  4   /* MSC Viterbi add-compare-select    */
#define DABGPU_STAGE_MSC_TB   5   /* MSC chainback + energy dispersal  */
#define DABGPU_STAGE_DABPLUS  6   /* k_dabplus (superframe, RS, AU CRC) */
#define DABGPU_NSTAGE         7
int dabgpu_pipe_set_profiling(dabgpu_pipe *p, int on);
int dabgpu_pipe_timing(dabgpu_pipe *p, float *ms /*[DABGPU_NSTAGE]*/, int32_t *launches /*[DABGPU_NSTAGE] or NULL*/);
/* device soft-bit ring of the last run ([n_streams][ring][75][3072] bytes) and the slot
 * of (stream, frame) in it, for tests and the ofdmProcessor drop-in.  Each byte is the
 * ibits value v of processToken (ofdm-decoder.cpp:188-189, always in -127..127) plus 127:
 * the Viterbi's branch-metric input itself (viterbi.cpp:230-233), half the bytes of int16. */
int dabgpu_pipe_softbits(dabgpu_pipe *p, const uint8_t **soft_d, int32_t *ring_frames);
int dabgpu_pipe_frame_slot(dabgpu_pipe *p, int frame, int32_t *slot);
/* per-frame front-end record of the last run: [n_streams][n_frames] */
int dabgpu_pipe_frames(dabgpu_pipe *p, dabgpu_frame *frames_h, int32_t *start_index_h);
/* The constellation display of ofdmDecoder::processToken (ofdm-decoder.cpp:192-206,
 * displayToken 2): with on = 1 the demod keeps, for every frame it decodes, the FFT
 * of symbol 2 at bins [0, K/2) and [T_u-1-K/2, T_u-1) -- the K values processToken
 * pushes into iqBuffer, in that order; dabgpu_pipe_iq_display copies those of
 * (stream, frame) of the last dabgpu_pipe_run (a decoded frame) to carriers_h[K][2].
 * Which frames the GUI is shown (every 8th) is the caller's choice, as in the
 * reference.  Costs 12 KB of HBM writes per frame while on. */
int dabgpu_pipe_set_display(dabgpu_pipe *p, int on);
/* The symbol (1..75) the display feed keeps, ofdmDecoder::set_displayToken (declared in
 * ofdm-decoder.h:50, displayToken = 2 at ofdm-decoder.cpp:61); takes effect at the next run. */
int dabgpu_pipe_set_display_token(dabgpu_pipe *p, int token);
/* Output format of the following runs, a mask (0 = the default: one bit per byte, as
 * deconvolve / process_ficInput deliver them, viterbi.cpp:240-241, fic-handler.cpp:270-292):
 *   DABGPU_PACK_MSC  MSC eight bits per byte, msb first (the packing of
 *                    mp4Processor::addtoFrame, mp4processor.cpp:115-121 -- numpy packbits
 *                    order): msc_stride is then in bytes (>= 3 * bitRate).  The DAB+ layer
 *                    reads either.
 *   DABGPU_PACK_FIC  FIC as FIB bytes, msb first: fic_bits holds [n_frames][4][96] bytes per
 *                    stream (3 FIBs of 32 bytes per FIC block, the last 2 bytes of each FIB
 *                    its CRC, inverted in place as check_CRC_bits leaves it,
 *                    dab-constants.h:310-340) instead of [4][768] bits -- an eighth of the
 *                    bytes a host (or dabgpu_pipe_fetch) has to move; fic_crc unchanged.
 * Any other value: DABGPU_E_ARG. */
#define DABGPU_PACK_MSC 1
#define DABGPU_PACK_FIC 2
int dabgpu_pipe_set_packed(dabgpu_pipe *p, int on);
/* Copy bytes from an output buffer of the last dabgpu_pipe_run (or dabgpu_pipe_dabplus)
 * to host memory, asynchronously, behind that run's channel decoding on its back-end
 * stream: the results reach the host while the next run decodes.  Complete after
 * dabgpu_pipe_sync (the run after next does not wait for it; its channel decoding, which
 * may reuse the output buffers, is queued behind it).  dst_h should be dabgpu_host_alloc
 * memory: with it (and 16-byte aligned pointers and size) a kernel of a few waves writes
 * the mapped host buffer directly; other memory goes through the runtime's copy, which
 * may synchronise. */
int dabgpu_pipe_fetch(dabgpu_pipe *p, void *dst_h, const void *src_d, size_t bytes);
int dabgpu_pipe_iq_display(dabgpu_pipe *p, int stream, int frame, float *carriers_h);

#ifdef __cplusplus
}
#endif
#endif
