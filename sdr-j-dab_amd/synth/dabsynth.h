/*
 * dabsynth.h -- synthetic DAB Mode-I transmitter (input generator for the
 * tests and bench; not part of the decode path).
 *
 * sdr-j-dab has no signal generator (its GENERATOR device id is declared
 * but unimplemented, virtual-input.h:41), so this is the build's own
 * ETSI EN 300 401 Mode-I modulator: FIBs with CRC, energy dispersal,
 * k=7 R=1/4 convolutional code, FIC/MSC puncturing (UEP and EEP), time
 * interleaving, CIF assembly, frequency interleaving, DQPSK against the
 * phase reference symbol, IFFT, cyclic prefix, null symbol, AWGN and CFO.
 * Its conventions are the inverse of the reference receiver's:
 *   soft bit i of a symbol  -> carrier i real part, bit 1536+i -> imag part
 *   QPSK  (1-2b_re) + j(1-2b_im), DQPSK z_l[k] = z_{l-1}[k] * q
 *   time interleaving delay 15 - d(i) so the receiver's d(i) makes 15
 *   (receiver CIF n decodes encoder CIF n-15).
 */
#ifndef DABSYNTH_H
#define DABSYNTH_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int16_t startAddr;   /* CU address 0..863 */
    int16_t length;      /* subchannel size in CUs */
    int16_t bitRate;     /* kbit/s */
    int16_t protLevel;   /* UEP level 1..5, or EEP 0100|lvl (A) / 0200|lvl (B) */
    int16_t uep;         /* 1 = UEP (uepFlag 0 in the reference), 0 = EEP */
    int16_t dabplus;     /* 1+k: DAB+ superframe stream (valid RS/fire code/AU CRCs), grid shifted by k CIFs */
    int16_t content;     /* with dabplus 0: 0 random bits; DABSYNTH_MP2: one MPEG-1 layer II frame per
                            CIF (48 kHz, sync + header, payload bytes < 0x80 so only headers carry
                            12 ones in a row); DABSYNTH_PACKET: packet mode, 24..96-byte packets with
                            CRCs carrying MSC data groups (address 0x100 + subchannel index, some
                            padding packets), announced as DSCTy 60 by FIG 0/2 (TMid 3) + FIG 0/3;
                            with dabplus: 0 every superframe dacRate 0 / SBR 0 (4 AUs),
                            DABSYNTH_AU_MIX the superframes cycle through the four (dacRate, SBR)
                            layouts of mp4processor.cpp:163-195 (4, 2, 6, 3 AUs) */
} dabsynth_subch;
#define DABSYNTH_MP2 2
#define DABSYNTH_PACKET 3
#define DABSYNTH_AU_MIX 4

typedef struct {
    int32_t n_frames;    /* frames after the pre-roll */
    int32_t pre_offset;  /* stream starts this many samples into a pre-roll frame */
    float   snr_db;      /* >= 200: noiseless */
    float   cfo_hz;      /* carrier frequency offset */
    float   amplitude;   /* RMS of the OFDM signal */
    int32_t n_subch;
    const dabsynth_subch *subch;
    int32_t figs;        /* 0: FIBs of random bytes (with CRC); 1: FIGs describing the
                            ensemble -- FIG 1/0 label "SYNTH ENSEMBLE", per subchannel i
                            FIG 0/1 (sub-channel i), FIG 0/2 (service 0xC000+i, one audio
                            component, ASCTy 63 for DAB+), FIG 1/1 label "SERVICE ii" --
                            cycled one item per FIB */
} dabsynth_cfg;

/* total stream length in samples */
int64_t dabsynth_stream_len(const dabsynth_cfg *cfg);
/* Generate one ensemble.  iq: cf32[stream_len].  Optional truth outputs:
 *   fic_bits   [n_frames][4][768]     FIB bits (CRC field as transmitted)
 *   msc_bits   [4*n_frames][n_subch][24*max_bitRate]  info bits the receiver
 *              must output at CIF n (valid for n >= 16)
 *   coded_bits [n_frames][75][3072]  hard bits carried by each data symbol
 *   frame0_start  stream index of frame 0's null symbol start
 * returns 0 on success. */
int dabsynth_generate(const dabsynth_cfg *cfg, uint64_t seed, float *iq,
                      uint8_t *fic_bits, uint8_t *msc_bits, uint8_t *coded_bits,
                      int64_t *frame0_start);

/* Many ensembles in parallel (host threads).  iq: [n_ens][stream_len]; the
 * truth pointers may be NULL; seeds are seed0 + ensemble index. */
int dabsynth_generate_many(const dabsynth_cfg *cfg, uint64_t seed0, int n_ens, int n_threads,
                           float *iq, uint8_t *fic_bits, uint8_t *msc_bits);

/* One period of a cyclic stream: P frames (P >= 4) of TF samples, frame 0's null
 * symbol first.  The time interleaver (and the DAB+ superframe grid: 4P must then be a
 * multiple of 5) wraps around the period, so the period repeated end to end is a valid
 * stream anywhere.  A stream of any length with the linear generator's layout (frame 0
 * at TF - pre_offset) is iq_stream[p] = iq[(p - (TF - pre_offset)) mod (P * TF)].
 * Truth: fic_bits [P][4][768] by frame; msc_bits [4P][n_subch][24*max_bitRate] by
 * receiver CIF n mod 4P (receiver CIF n decodes encoder CIF (n - 15) mod 4P).
 * DABSYNTH_PACKET subchannels are refused (-4): a data group in flight and the packet
 * continuity counter would not wrap at the seam. */
int dabsynth_generate_period(const dabsynth_cfg *cfg, uint64_t seed, int period, float *iq,
                             uint8_t *fic_bits, uint8_t *msc_bits);
/* periods of n_ens ensembles (seeds seed0 + e) in parallel: iq [n_ens][2 * period * TF] */
int dabsynth_period_many(const dabsynth_cfg *cfg, uint64_t seed0, int period, int n_ens, int n_threads,
                         float *iq);

/* building blocks exposed for tests */
void dabsynth_conv_encode(const uint8_t *bits, int nbits, uint8_t *coded /*[4*(nbits+6)]*/);
int  dabsynth_puncture_msc(int uep, int bitRate, int protLevel, const uint8_t *mother, uint8_t *out);
void dabsynth_puncture_fic(const uint8_t *mother /*[3096]*/, uint8_t *out /*[2304]*/);
void dabsynth_make_fib(uint64_t *rng_state, uint8_t *fib /*[256]*/);
void dabsynth_rs_encode(const uint8_t *data /*[110]*/, uint8_t *cw /*[120]*/);

#ifdef __cplusplus
}
#endif
#endif
