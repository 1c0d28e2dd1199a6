/*
 * dab_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the sdr-j-dab (v0.997) DAB Mode-I receive hot path,
 * used as the parity checker for the MI355X path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product path (sdr-j-dab_amd/) never links or calls it.
 *
 * Every function cites the reference file:line whose behaviour it restates
 * (paths relative to the reference tree).  The restatement is pinned by
 *   (1) golden vectors produced by the reference's own compilable sources
 *       (oracle/_ref, see oracle/Makefile and tests/golden/make_golden.py),
 *   (2) the reference's intrinsic checks (FIB CRC, fire code, RS, AU CRC).
 * FFT parity is unpinned by construction: the reference links FFTW3f (an
 * un-vendored third-party dependency absent from this image); the oracle
 * uses a double-precision DFT rounded to float (an "ideal" fp32 FFT); an fp32
 * radix-4 transform (orc_fft2048_f32, FFTW3f's precision class) measures the
 * soft values' fp32 floor and serves the CPU baseline.
 */
#ifndef DAB_ORACLE_H
#define DAB_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Mode-I geometry (gui.cpp:1361-1371, dab-constants.h:137-149) */
#define ORC_TU     2048
#define ORC_TS     2552
#define ORC_TG     504
#define ORC_TNULL  2656
#define ORC_TF     196608
#define ORC_K      1536
#define ORC_L      76
#define ORC_CARRIER_DIFF 1000
#define ORC_INPUT_RATE   2048000

/* ---- tables ---- */
void    orc_init(void);          /* builds the lazily initialised tables (thread-safe use after) */
void    orc_mapper(int16_t *perm /*[1536]*/);                  /* mapper.cpp:33-55,84-86 */
void    orc_ref_table(float *ref /*[2*2048] cf32*/);          /* phasereference.cpp:40-47 */
float   orc_get_phi(int32_t k);                                /* phasetable.cpp:261-274 */
void    orc_osc_entry(int32_t i, float *re, float *im);        /* ofdm-processor.cpp:79-81 */
void    orc_prbs(int n, uint8_t *out);                         /* fic-handler.cpp:100-108 */
void    orc_pcode(int idx /*1..24*/, int8_t *out /*[32]*/);    /* protTables.cpp:28-58 */
int     orc_uep_profile(int bitRate, int protLevel, int16_t *L /*[4]*/, int16_t *PI /*[4]*/); /* deconvolve.cpp:39-114 */
int     orc_eep_profile(int bitRate, int protLevel, int16_t *L /*[2]*/, int16_t *PI /*[2]*/); /* deconvolve.cpp:244-314 */
int     orc_interleave_delay(int i);                           /* dab-concurrent.cpp:42-43 */

/* ---- OFDM front end ---- */
void    orc_fft2048(const float *in /*cf32[2048]*/, float *out, int inverse); /* fft.cpp:53,109 */
int32_t orc_find_index(const float *v /*cf32[T_u]*/, int16_t level, float *maxv, float *sumv); /* phasereference.cpp:60-88 */
int16_t orc_process_block0(const float *v /*cf32[T_u]*/, float *phase_ref /*cf32[T_u] out*/,
                           int flag, int method);             /* ofdm-decoder.cpp:85-162 */
int16_t orc_get_snr(const float *X /*cf32[T_u] spectrum*/);      /* ofdm-decoder.cpp:212-230 */
void    orc_process_token(const float *v /*cf32[T_s]*/, float *phase_ref /*cf32[T_u] in/out*/,
                          int16_t *ibits /*[3072]*/, float *softf /*[3072] or NULL*/); /* ofdm-decoder.cpp:167-190 */
/* the same with the fp32 radix-4 FFT (fft_kind 1: FFTW3f's precision class, the soft
 * values' fp32 floor and the CPU baseline) or the double-precision one (0) */
void    orc_fft2048_f32(const float *in /*cf32[2048]*/, float *out, int inverse);
/* kind 0 double, 1 fp32 radix-4 Stockham, 2 fp32 radix-2 DIT, 3 fp32 radix-2 DIF */
void    orc_fft2048_kind(const float *in, float *out, int inverse, int kind);
void    orc_process_token_fft(const float *v, float *phase_ref, int16_t *ibits, float *softf, int fft_kind);
int16_t orc_process_block0_fft(const float *v, float *phase_ref, int flag, int method, int fft_kind);
void    orc_freqcorr(const float *v /*cf32[T_s]*/, double *acc_re, double *acc_im,
                     float *facc /*cf32 running, reference float order*/); /* ofdm-processor.cpp:424-425 */

/* Whole-stream restatement of ofdmProcessor::run (ofdm-processor.cpp:247-474)
 * over an in-memory cf32 stream.  Per decoded frame f it records the PRS
 * window start, startIndex, coarse/fine corrector values and the 75x3072
 * soft bits.  Returns the number of complete frames decoded. */
typedef struct {
    int64_t window_start;   /* stream index of the first sample of the T_u window (SyncOnPhase) */
    int32_t start_index;    /* findIndex result */
    int32_t coarse;         /* coarseCorrector used for the data symbols */
    int16_t fine;           /* fineCorrector used for the data symbols */
    int16_t correction;     /* processBlock_0 return (or 0 when f2Correction off) */
    int32_t lp_window;      /* localPhase before the window's first sample */
} orc_frame_info;

/* ofdmProcessor::run's null search in scan mode: attempts / No_Signal_Found count when
 * the samples run out (0) or where a null's end is found (1, pos) */
int     orc_null_scan(const float *iq, int64_t n, int scan, int32_t *attempts, int32_t *no_signal, int64_t *pos);
int     orc_ofdm_run(const float *iq /*cf32[n]*/, int64_t n, int16_t threshold, int method,
                     int max_frames, orc_frame_info *info, int16_t *softbits /*[max_frames][75][3072]*/);
int     orc_ofdm_run_fft(const float *iq, int64_t n, int16_t threshold, int method, int max_frames,
                         orc_frame_info *info, int16_t *softbits, int fft_kind);
/* ... and the two display feeds of the reference's OFDM classes:
 *   iqBuffer (ofdmDecoder::processToken, ofdm-decoder.cpp:192-206): every 8th call with
 *     blkno == displayToken (2), fft_buffer[0, K/2) then [T_u-1-K/2, T_u-1): iq_disp[k]
 *     holds K cf32 values, disp_frame[k] the frame they came from;
 *   spectrumBuffer (ofdmProcessor::getSample(s), ofdm-processor.cpp:161-180,220-238):
 *     spec_start[k] = stream index of the first of the 32768 raw (pre-NCO) samples of
 *     the k-th emission.
 * n_disp / n_spec count every emission (entries past max_* are not stored). */
typedef struct {
    float   *iq_disp;       /* [max_disp][K][2] */
    int32_t *disp_frame;    /* [max_disp] */
    int32_t  max_disp, n_disp;
    int64_t *spec_start;    /* [max_spec] */
    int32_t  max_spec, n_spec;
    int32_t  token;         /* displayToken (ofdm-decoder.cpp:61; 0 means the reference's 2) */
} orc_display;
int     orc_ofdm_run_display(const float *iq, int64_t n, int16_t threshold, int method, int max_frames,
                             orc_frame_info *info, int16_t *softbits, orc_display *disp);

/* ---- backend ---- */
void    orc_viterbi(const int16_t *in /*[4*(nbits+6)]*/, int nbits, uint8_t *out /*[nbits]*/); /* viterbi.cpp:225-242 */
void    orc_fic_depuncture(const int16_t *in /*[2304]*/, int16_t *out /*[3096]*/); /* fic-handler.cpp:254-288 */
void    orc_fic_process(const int16_t *in /*[2304]*/, uint8_t *bits /*[768]*/, uint8_t *crc_ok /*[3]*/); /* fic-handler.cpp:241-321 */
int     orc_check_crc_bits(uint8_t *in, int16_t size);        /* dab-constants.h:310-340 (mutates like the reference) */
int     orc_msc_depuncture(int uep, int bitRate, int protLevel, const int16_t *in, int16_t *out /*[4*(24*bitRate)+24]*/); /* deconvolve.cpp:142-237,325-366 */
/* dabConcurrent (dab-concurrent.cpp:144-193) restated for one subchannel over ncif CIFs:
 * cif_frag[c][fragmentSize] -> outputs for CIF c >= 16 (warm-up skipped, like the reference)
 * in out[c][24*bitRate] (1 bit per byte, after energy dispersal).  out rows for c < 16 are zeroed. */
int     orc_msc_stream(int uep, int bitRate, int protLevel, int fragmentSize, int ncif,
                       const int16_t *cif_frag, uint8_t *out);

/* ---- DAB+ ---- */
int16_t orc_rs_dec(const uint8_t *in /*[120]*/, uint8_t *out /*[110]*/); /* reed-solomon.cpp:129-141 */
void    orc_rs_enc(const uint8_t *in /*[110]*/, uint8_t *out /*[120]*/); /* reed-solomon.cpp:110-126 */
int     orc_firecode_check(const uint8_t *x /*[11]*/);        /* firecode-checker.cpp:76-94 */
int     orc_dabplus_crc(const uint8_t *msg, int16_t len);      /* mp4processor.cpp:40-61 */
/* mp4Processor::processSuperframe (mp4processor.cpp:146-230) minus faad:
 * returns 1 on success, 0 on failure; fills out[110*RSDims], n_corrected,
 * num_aus, au_start[num_aus+1], au_crc[num_aus]. */
int     orc_superframe(const uint8_t *frame /*[120*RSDims]*/, int base, int bitRate,
                       uint8_t *out, int16_t *n_corrected, int *num_aus, int16_t *au_start, uint8_t *au_crc);

/* mp4Processor::addtoFrame (mp4processor.cpp:107-145): 5-CIF byte ring,
 * fire-code check at the oldest block, processSuperframe on success.
 * Returns 0 (fewer than 5 blocks buffered), 1 (fire code failed),
 * 2 (processSuperframe returned false), 3 (superframe decoded); the
 * orc_superframe outputs are filled for 2 and 3. */
typedef struct {
    int bitRate, fill, blocks;
    uint8_t ring[120 * 48];
} orc_mp4;
void orc_mp4_init(orc_mp4 *m, int bitRate);
int  orc_mp4_add(orc_mp4 *m, const uint8_t *bits /*[24*bitRate], 1 bit per byte*/, uint8_t *out,
                 int16_t *n_corrected, int *num_aus, int16_t *au_start, uint8_t *au_crc);

#ifdef __cplusplus
}
#endif
#endif
