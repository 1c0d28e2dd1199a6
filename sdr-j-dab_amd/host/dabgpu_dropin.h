// dabgpu_dropin.h -- C++ host classes with the interfaces of sdr-j-dab's hot-path
// classes, running on MI355X through the C ABI (include/dabgpu.h).
//
// Same class names, constructor arguments, method signatures and argument
// meaning as the reference (paths relative to the sdr-j-dab v0.997 tree), minus
// Qt: where the reference emits a Qt signal or calls into the GUI, these classes
// take a std::function callback instead.  They live in namespace dabgpu so a
// build can switch with a using-declaration.
//
// Errors: the reference signals hard errors by `throw int` out of its worker
// threads (ofdm-processor.cpp:200-240); here a failing GPU call throws
// dabgpu::error (std::runtime_error with dabgpu_last_error()).  Decoding
// outcomes (CRC failures, RS failures) are return values, as in the reference.
//
// Threading: one HIP context per calling thread (thread_local), as the
// reference runs OFDM, FIC and MSC on separate threads.
#pragma once
#include <complex>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <vector>

#include <atomic>
#include <cstdio>
#include <memory>
#include <mutex>
#include <thread>

#ifdef DABGPU_HAVE_SNDFILE
#include <sndfile.h>          // a build with libsndfile (the reference's gui.cpp / wavfiles)
#endif

#include "dabgpu.h"
#include "fib_processor.h"
#include "msc_consumers.h"
#include "ringbuffer.h"

namespace dabgpu {

typedef std::complex<float> DSPCOMPLEX;   // dab-constants.h: DSPCOMPLEX

// ---- reference data types (dab-constants.h:72-73,137-176) -------------------------
#define DAB      0100
#define DAB_PLUS 0101
struct DabParams {
    uint8_t dabMode;
    int16_t L, K, T_null;
    int32_t T_F;
    int16_t T_s, T_u, guardLength, carrierDiff;
};
// RadioInterface::setModeParameters (gui.cpp:1361-1371); the GPU path is Mode I only
void setModeParameters(DabParams *p, uint8_t mode = 1);
// packetdata / audiodata (dab-constants.h:152-177): fib_processor.h

// virtualInput (src/input/virtual-input.h:51-70): the device the front end pulls
// samples from; getSamples copies up to n cf32 samples scaled to about +-1.
class virtualInput {
public:
    virtual ~virtualInput() = default;
    virtual int32_t getSamples(DSPCOMPLEX *v, int32_t n) = 0;
    virtual int32_t Samples() = 0;
    virtual bool restartReader() { return true; }
    virtual void stopReader() {}
    virtual int16_t bitDepth() { return 10; }
};

struct error : std::runtime_error {
    int code;
    error(int c, const std::string &what) : std::runtime_error(what), code(c) {}
};

// HIP device used by contexts created from now on in this process (default 0)
void set_device(int device);
// this thread's context (created on first use)
dabgpu_ctx *thread_context();

// device buffer owned by the calling thread's context
class devbuf {
public:
    devbuf() = default;
    explicit devbuf(size_t bytes) { resize(bytes); }
    ~devbuf();
    devbuf(const devbuf &) = delete;
    devbuf &operator=(const devbuf &) = delete;
    void resize(size_t bytes);
    void *get() const { return p_; }
    size_t size() const { return n_; }
    void upload(const void *h, size_t bytes);
    void download(void *h, size_t bytes) const;
private:
    void *p_ = nullptr;
    size_t n_ = 0;
};

// viterbi.h:66-85 -- k=7 R=1/4 decoder for wordlength info bits
class viterbi {
public:
    explicit viterbi(int16_t wordlength);
    virtual ~viterbi() = default;
    // input: 4*(wordlength+6) soft bits in [-127, 127]; output: wordlength bits (one per byte)
    void deconvolve(int16_t *input, uint8_t *output);
protected:
    int16_t wordlength_;
    devbuf in_, out_;
};

// deconvolve.h: uep_deconvolve (deconvolve.cpp:142-237)
class uep_deconvolve : public viterbi {
public:
    uep_deconvolve(int16_t bitRate, int16_t protLevel);
    // v: fragmentSize punctured soft bits; out: 24*bitRate bits (no energy dispersal,
    // exactly what the reference's deconvolve delivers). False for an undefined profile.
    bool deconvolve(int16_t *v, int32_t size, uint8_t *outBuffer);
private:
    dabgpu_subch sub_;
};

// deconvolve.h: eep_deconvolve (deconvolve.cpp:238-366), protLevel = 0100|n (A) or 0200|n (B)
class eep_deconvolve : public viterbi {
public:
    eep_deconvolve(int16_t bitRate, int16_t protLevel);
    bool deconvolve(int16_t *v, int32_t size, uint8_t *outBuffer);
private:
    dabgpu_subch sub_;
};

// reed-solomon.h -- only the DAB+ code (8, 0435, 0, 1, 10) is supported on the GPU
class reedSolomon {
public:
    reedSolomon(uint16_t symsize = 8, uint16_t gfpoly = 0435, uint16_t fcr = 0, uint16_t prim = 1,
                uint16_t nroots = 10);
    // cutlen must be 135 (RS(120,110), mp4processor.cpp:171); returns corrected symbols or -1
    int16_t dec(const uint8_t *data_in, uint8_t *data_out, int16_t cutlen);
private:
    devbuf in_, out_, ret_;
};

// phasereference.h -- findIndex on T_u samples already mixed by getSamples
class phaseReference {
public:
    explicit phaseReference(int16_t threshold);
    int32_t findIndex(DSPCOMPLEX *v);
private:
    int16_t threshold_;
    devbuf iq_, fr_, si_;
};

// ficHandler without Qt (fic-handler.cpp:143-321, fic-handler.h:44-52): process_ficBlock
// accumulates symbols 1..3 of a frame into the 4 FIC blocks and decodes each on the GPU
// (depuncture, Viterbi, energy dispersal, CRC); every CRC-good FIB goes to the owned
// fib_processor under the fibHandling lock, as process_ficInput does (:304-320), so the
// GUI's service lookups (kindofService, dataforAudioService, dataforDataService,
// clearEnsemble) work on this class as on the reference's.  QString& arguments are
// std::string (UTF-8, the 16 characters of the label as transmitted).  Signals are
// callbacks: show_ficCRC per FIB, nameofEnsemble / addtoEnsemble from the FIG parser.
// Optionally every FIB (256 bits, CRC field inverted as check_CRC_bits leaves it) with
// its CRC verdict goes to a raw callback as well.
// The reference runs the decoding on its own thread behind a 3-slot queue and stop()
// ends that thread; here decoding happens in the caller's thread (the GPU is the
// parallel part) and after stop() process_ficBlock drops its input.
class ficHandler {
public:
    using fib_cb = std::function<void(const uint8_t *fib /*256 bits*/, bool crc_ok, int16_t ficno)>;
    struct signals {
        std::function<void(bool)> show_ficCRC;
        fib_processor::ensemble_cb nameofEnsemble;
        fib_processor::service_cb addtoEnsemble;
    };
    explicit ficHandler(signals sig, int16_t bitsperBlock = 2 * DABGPU_K);
    explicit ficHandler(fib_cb cb, int16_t bitsperBlock = 2 * DABGPU_K);
    void process_ficBlock(int16_t *data, int16_t blkno);   // blkno 1..3
    void clearEnsemble();
    int16_t get_ficRatio() const;                           // % of FIBs with a good CRC (*)
    uint8_t kindofService(const std::string &s);
    void dataforDataService(const std::string &s, packetdata *d);
    void dataforAudioService(const std::string &s, audiodata *d);
    void stop();
    void on_fib(fib_cb cb) { cb_ = std::move(cb); }
    // (*) the reference's ficRatio is never updated in v0.997 (fic-handler.cpp:186-188)
    // the database, for callers that want more than the reference's lookups (under the lock)
    template <class F> auto with_fib_processor(F f) {
        std::lock_guard<std::mutex> g(fibHandling_);
        return f(fibProcessor_);
    }
private:
    void init(int16_t bitsperBlock);
    fib_cb cb_;
    signals sig_;
    std::vector<int16_t> ofdm_input_;
    int index_ = 0, ficno_ = 0;
    int good_ = 0, total_ = 0;
    std::atomic<bool> running_{true};
    std::mutex fibHandling_;
    fib_processor fibProcessor_;
    std::vector<std::function<void()>> pending_;   // GUI signals raised under fibHandling_, fired after it
    devbuf in_, bits_, crc_;
};

// ---- MSC back end ----------------------------------------------------------------
// mp4Processor::addtoFrame / processSuperframe (mp4processor.cpp:107-292) minus faad:
// 5-CIF superframe window, fire code, RS(120,110) of the RSDims columns on the GPU
// (one dabgpu_rs_decode launch per superframe), AU table and AU CRCs; each AU goes to
// the callback where the reference hands it to the AAC decoder.
class mp4Processor : public dabProcessor {
public:
    struct au_info {
        uint8_t dacRate, sbrFlag, aacChannelMode, mpegSurround;
        int16_t n_corrected;           // RS symbols corrected in the superframe
    };
    using au_cb = std::function<void(const uint8_t *au, int16_t len, bool crc_ok, const au_info &)>;
    mp4Processor(int16_t bitRate, au_cb cb);
    void addtoFrame(uint8_t *v, int16_t nbits) override;
    int32_t superframes() const { return superframes_; }
    int32_t frameErrors() const { return frameErrors_; }
private:
    bool processSuperframe(int base);
    int16_t bitRate_, RSDims_;
    au_cb cb_;
    std::vector<uint8_t> frameBytes_, outVector_;
    int16_t blockFillIndex_ = 0, blocksInBuffer_ = 0;
    int32_t superframes_ = 0, frameErrors_ = 0;
    devbuf rsin_, rsout_, rsret_;
};

// dabConcurrent (dab-concurrent.cpp:34-202) without its thread: each CIF fragment is
// time-de-interleaved (16 branches, delays 15 - brev4(i), the first 16 CIFs are warm-up),
// then depunctured + Viterbi-decoded + energy-dispersed on the GPU
// (dabgpu_msc_deconvolve) and handed to the dabProcessor.  (The reference's thread hands
// CIF n over when CIF n+1 arrives; here it is decoded on arrival.)
class dabConcurrent : public dabVirtual {
public:
    dabConcurrent(uint8_t dabModus, int16_t fragmentSize, int16_t bitRate, int16_t uepFlag, int16_t protLevel,
                  std::unique_ptr<dabProcessor> processor);
    int32_t process(int16_t *v, int16_t cnt) override;
    void setFiles(FILE *mp2, FILE *mp4) override;   // dab-concurrent.cpp:196-200
    dabProcessor *processor() { return proc_.get(); }
protected:
    bool deinterleave(const int16_t *v);       // false during the warm-up
    uint8_t dabModus_;
    int16_t fragmentSize_, bitRate_;
    dabgpu_subch sub_;
    std::vector<int16_t> delay_;               // [16][fragmentSize] ring of past fragments
    std::vector<int16_t> data_;
    int32_t countforInterleaver_ = 0, cif_ = 0;
    std::vector<uint8_t> outV_;
    std::unique_ptr<dabProcessor> proc_;
    devbuf in_, out_;
};

// mscDatagroup (msc-datagroup.cpp:44-339) without its thread: the same de-interleave and
// GPU decode, then packets -> MSC data groups (packetAssembler) for the data handler.
class mscDatagroup : public dabConcurrent {
public:
    mscDatagroup(uint8_t DSCTy, int16_t packetAddress, int16_t fragmentSize, int16_t bitRate, int16_t uepFlag,
                 int16_t protLevel, uint8_t DGflag, int16_t FEC_scheme, packetAssembler::datagroup_cb cb);
    int32_t process(int16_t *v, int16_t cnt) override;
    const packetAssembler &assembler() const { return pa_; }
private:
    packetAssembler pa_;
};

// mscHandler (msc-handler.cpp:41-193): collects the 18 MSC symbols of a CIF
// (process_mscBlock with blkno 4..75), and for the selected subchannel hands the
// CIF's slice [startAddr * 64, + Length * 64) to a dabConcurrent (audio: mp2Processor
// for DAB, mp4Processor for DAB+ (ASCTy 077)) or an mscDatagroup (data).  The channel
// set by set_audioChannel / set_dataChannel (any thread, under the lock) takes effect
// at the next process_mscBlock.  The decoded output goes to the callbacks; setFiles
// (msc-handler.cpp:208-212) dumps the DAB audio's MPEG frames into the mp2 file instead
// (see mp2Processor), and keeps both files for the channels selected later
// (msc-handler.cpp:147-150).
class mscHandler {
public:
    struct outputs {
        mp2Processor::frame_cb mp2;            // MPEG-1/2 layer II frames (DAB)
        mp4Processor::au_cb aac;               // AAC access units (DAB+)
        packetAssembler::datagroup_cb datagroup;
    };
    mscHandler(DabParams *p, outputs out, uint8_t concurrent = 1);
    void process_mscBlock(int16_t *fbits, int16_t blkno);
    void set_audioChannel(audiodata *d);
    void set_dataChannel(packetdata *d);
    int16_t getLanguage();
    int16_t getType();
    void stop();
    void stopProcessing();
    void setFiles(FILE *mp2, FILE *mp4);
    dabVirtual *handler() { return dabHandler_.get(); }
private:
    std::mutex locker_;
    outputs out_;
    FILE *mp2File_ = nullptr, *mp4File_ = nullptr;
    int16_t BitsperBlock_, numberofblocksperCIF_;
    std::vector<int16_t> cifVector_;
    std::unique_ptr<dabVirtual> dabHandler_;
    bool audioService_ = true, work_to_be_done_ = false, newChannel_ = false;
    int16_t startAddr_ = 0, Length_ = 0;
    audiodata na_{};
    packetdata np_{};
    int16_t new_language_ = 0, new_type_ = 0;
};

// ---- libsndfile (the .sdr dump) -------------------------------------------------------
// gui.cpp:861-893 opens the dump with sf_open (path, SFM_WRITE, {INPUT_RATE, 2 channels,
// SF_FORMAT_WAV | SF_FORMAT_PCM_16}) and hands the SNDFILE* to ofdmProcessor::startDumping,
// which writes interleaved PCM16 frames with sf_writef_short (ofdm-processor.cpp:150-157).
// Built with -DDABGPU_HAVE_SNDFILE (and -lsndfile), dabgpu:: names libsndfile's own types
// and calls, so the GUI's ::SNDFILE* binds to startDumping unchanged.  Without it (this
// image has no libsndfile) a stand-in with the subset those calls use writes the same
// RIFF/WAVE PCM16 file (the header's sizes are filled in by sf_close).
#ifdef DABGPU_HAVE_SNDFILE
using ::SF_INFO;
using ::SNDFILE;
using ::sf_close;
using ::sf_open;
using ::sf_writef_short;
using ::SFM_WRITE;
using ::SF_FORMAT_WAV;
using ::SF_FORMAT_PCM_16;
#else
struct SF_INFO {
    int64_t frames;
    int samplerate, channels, format, sections, seekable;
};
struct SNDFILE;
constexpr int SFM_WRITE = 0x20;
constexpr int SF_FORMAT_WAV = 0x010000, SF_FORMAT_PCM_16 = 0x0002;
SNDFILE *sf_open(const char *path, int mode, SF_INFO *info);   // SFM_WRITE, WAV PCM16 only (else nullptr)
int64_t sf_writef_short(SNDFILE *f, const int16_t *ptr, int64_t frames);
int sf_close(SNDFILE *f);
#endif

// ---- OFDM front end ----------------------------------------------------------------
// ofdmDecoder (ofdm-decoder.cpp:37-230, ofdm-decoder.h:40-48) one symbol per call on the
// GPU: processBlock_0 = get_snr (IIR 0.7/0.3, show_snr every 11 blocks) + coarse offset of
// freqSyncMethod 0/1/2 + the spectrum as phase reference; processToken = FFT + DQPSK +
// frequency de-interleave -> 3072 soft bits, and every 8th displayToken (blkno 2) the
// carriers fft_buffer[0, K/2) and [T_u-1-K/2, T_u-1) into iqBuffer + showIQ(K)
// (ofdm-decoder.cpp:192-206; the counter is shared by every decoder, as the reference's
// function-static cnt).  Samples are the caller's, already NCO-mixed.  The reference's
// RadioInterface* is the signals struct; refTable (phaseReference::getTable) only feeds
// refArg (ofdm-decoder.cpp:71-74), which the device tables hold already.
class ofdmDecoder {
public:
    struct signals {
        std::function<void(int)> show_snr, showIQ;
    };
    ofdmDecoder(DabParams *p, RingBuffer<DSPCOMPLEX> *iqBuffer, DSPCOMPLEX *refTable, signals sig,
                uint8_t freqSyncMethod);
    ofdmDecoder(DabParams *p, uint8_t freqSyncMethod = 1, std::function<void(int)> show_snr = nullptr);
    int16_t processBlock_0(DSPCOMPLEX *vi, bool flag);
    void processToken(DSPCOMPLEX *inv, int16_t *ibits, int32_t blkno);
    // get_snr (ofdm-decoder.cpp:212-230) of a T_u-point spectrum (natural bin order)
    int16_t get_snr(DSPCOMPLEX *v);
    int16_t snr() const { return snr_; }
    // the symbol whose carriers feed iqBuffer (ofdm-decoder.cpp:61,197; the reference
    // declares set_displayToken, ofdm-decoder.h:50, without defining it: here it works)
    void set_displayToken(int16_t t) { displayToken = t; }
    // processToken's `static int cnt` (ofdm-decoder.cpp:171): one count per process
    static std::atomic<int> iq_count;
    static constexpr int16_t defaultDisplayToken = 2;          // ofdm-decoder.cpp:61
    int16_t displayToken = defaultDisplayToken;
private:
    uint8_t method_;
    RingBuffer<DSPCOMPLEX> *iqBuffer_ = nullptr;
    signals sig_;
    int16_t snr_ = 0, snrCount_ = 0;
    devbuf smp_, spec_, fr_, corr_, snrd_, bits_;
};

// ofdmProcessor (ofdm-processor.cpp:34-509, ofdm-processor.h:49-59): the constructor
// starts the thread that pulls samples from the virtualInput into a sliding window in
// HBM and runs the GPU front end (the dabgpu_pipe_* engine for one stream: null search,
// findIndex, coarse/fine AFC, demod); every decoded frame's symbols go to
// ficHandler::process_ficBlock (blkno 1..3) and mscHandler::process_mscBlock (4..75) with
// the reference's soft bits.  The GUI signals are callbacks (the RadioInterface* of the
// reference): show_avgTokenLength (every 11 frames), setSynced, No_Signal_Found (scan
// mode), show_snr, and at the reference's sample positions -- the end of the getSample /
// getSamples call that takes the sample count past INPUT_RATE/7, replayed from the
// frames the GPU decoded -- show_fineCorrector / show_coarseCorrector and, with a
// spectrumBuffer (HAVE_SPECTRUM), the 32768 raw samples read since the previous one
// into the ring + showSpectrum(32768) (ofdm-processor.cpp:161-180,220-238).  With an
// iqBuffer every 8th frame's symbol-2 carriers go into it + showIQ(K), as the
// reference's ofdmDecoder does (ofdm-decoder.cpp:192-206; the GPU demod exports them,
// dabgpu_pipe_iq_display).  startDumping writes the raw samples as interleaved PCM16
// (the .sdr payload, ofdm-processor.cpp:150-157) with the reference's scaling, through
// sf_writef_short (SNDFILE*) or as bare PCM16 into a FILE*.
class ficHandler;
class ofdmProcessor {
public:
    struct signals {
        std::function<void(int)> show_fineCorrector, show_coarseCorrector, show_avgTokenLength, show_snr;
        std::function<void(char)> setSynced;
        std::function<void()> No_Signal_Found;
        std::function<void(int)> showSpectrum, showIQ;
    };
    // the reference's argument list (spectrumBuffer: HAVE_SPECTRUM builds; either ring may be null)
    ofdmProcessor(virtualInput *theRig, DabParams *p, signals sig, mscHandler *msc, ficHandler *fic,
                  int16_t threshold, RingBuffer<DSPCOMPLEX> *spectrumBuffer, RingBuffer<DSPCOMPLEX> *iqBuffer,
                  uint8_t freqSyncMethod);
    // without display rings (a build without HAVE_SPECTRUM and no IQ scope)
    ofdmProcessor(virtualInput *theRig, DabParams *p, signals sig, mscHandler *msc, ficHandler *fic,
                  int16_t threshold = 3, uint8_t freqSyncMethod = 1);
    ~ofdmProcessor();
    void reset();
    void stop();
    void coarseCorrectorOn();
    void coarseCorrectorOff();
    void set_scanMode(bool b);
    void startDumping(SNDFILE *f);
    void startDumping(FILE *f);
    void stopDumping();
    // the display symbol of the decoder this processor drives (ofdmDecoder::set_displayToken,
    // ofdm-decoder.h:50; the reference's ofdmProcessor owns its ofdmDecoder): 1..75, from
    // the next frame on.  A value outside 1..75 selects no symbol: in the reference such a
    // token never matches blkno (ofdm-decoder.cpp:192-195), so the display feed stops and the
    // decode goes on -- the setter keeps the last valid token and turns the feed off
    void set_displayToken(int16_t t) {
        if (t >= 1 && t <= 75) { displayToken_ = t; displayOff_ = false; }
        else displayOff_ = true;
    }
    int64_t frames() const { return frames_.load(); }
    static constexpr int32_t spectrumSize = 32768;          // bufferSize (ofdm-processor.cpp:97)
private:
    void run();
    void emit_frame(const dabgpu_frame_info &fi);
    // the reference's getSample / getSamples calls, replayed for the spectrum feed
    void consume_singles(int64_t to, const dabgpu_frame_info *fi);
    void consume_block(int64_t n, const dabgpu_frame_info *fi);
    void spectrum_emit(const dabgpu_frame_info *fi);
    void write_dump(const DSPCOMPLEX *v, int32_t n);
    virtualInput *theRig_;
    signals sig_;
    mscHandler *msc_;
    ficHandler *fic_;
    int16_t threshold_;
    uint8_t method_;
    RingBuffer<DSPCOMPLEX> *spectrumBuffer_ = nullptr, *iqBuffer_ = nullptr;
    std::thread thread_;
    std::atomic<bool> running_{false};
    std::atomic<int64_t> frames_{0};
    std::mutex ctl_;
    std::vector<int> pending_ops_;
    std::atomic<FILE *> dumpFile_{nullptr};
    std::atomic<SNDFILE *> dumpSnd_{nullptr};
    int16_t dumpScaler_ = 512;
    std::atomic<int16_t> displayToken_{ofdmDecoder::defaultDisplayToken};
    std::atomic<bool> displayOff_{false};
    // observables state
    int64_t last_block0_ = -1;
    int32_t avgTokenLength_ = 196608, tokenCount_ = 0;
    int16_t snr_ = 0, snrCount_ = 0;
    int32_t no_signal_ = 0, resyncs_ = 0;
    bool synced_ = false;
    // spectrum feed replay: samples consumed, sampleCnt, first sample of localBuffer
    int64_t consumed_ = 0, spec_cnt_ = 0, spec_start_ = 0;
    int16_t last_fine_ = 0;
    int32_t last_coarse_ = 0;
    // the device sample window (run()): the spectrum block is read back from it
    const float *win_ = nullptr;
    int64_t win_base_ = 0;
    std::vector<DSPCOMPLEX> specbuf_;
};

// The streaming engine: ofdmProcessor::run + ficHandler + mscHandler (+ DAB+
// mp4Processor layer) for many ensembles at once (dabgpu_pipe_*).  Each stream's
// cf32 samples are handed over as host arrays (a recorded or synthetic
// virtualInput); they are uploaded once and decoded n_frames at a time.
class ensembleDecoder {
public:
    struct config {
        int n_streams = 1;
        int n_frames = 8;                    // frames per step
        int16_t threshold = 3;               // gui.cpp:98-99
        std::vector<dabgpu_subch> subch;     // decoded in every stream
    };
    using fib_cb = std::function<void(int stream, int64_t frame, int ficno, const uint8_t *bits256, bool crc_ok)>;
    using msc_cb = std::function<void(int stream, int64_t cif, int subch, const uint8_t *bits, int nbits)>;
    using sf_cb = std::function<void(int stream, int64_t cif, int subch, const dabgpu_superframe &info,
                                     const uint8_t *bytes, int nbytes)>;
    explicit ensembleDecoder(const config &cfg);
    ~ensembleDecoder();
    void on_fib(fib_cb f) { fib_cb_ = std::move(f); }
    void on_msc(msc_cb f) { msc_cb_ = std::move(f); }
    void on_superframe(sf_cb f) { sf_cb_ = std::move(f); }
    // samples[s] -> n[s] cf32 samples of stream s (copied to HBM)
    void load(const std::vector<const DSPCOMPLEX *> &samples, const std::vector<int64_t> &n);
    // the streams as recorded: format DABGPU_IQ_S16 (.sdr PCM16 I/Q pairs) or DABGPU_IQ_U8
    // (.raw bytes), n[s] pairs each, copied to HBM as they are -- the pipeline converts them
    // in its sample loads with the readers' scaling (wavfiles.cpp:172, rawfiles.cpp:115-117)
    void load_recorded(int format, const std::vector<const void *> &samples, const std::vector<int64_t> &n);
    // one recording file per stream, all .sdr (RIFF/WAVE PCM16, 2 channels, 2048000 Hz, as
    // wavFiles accepts them: wavfiles.cpp:56-69) or all .raw (u8 I/Q): read in pieces straight
    // into HBM, unconverted.  Throws dabgpu::error for any other file.
    void load_files(const std::vector<std::string> &paths);
    // null search (ofdm-processor.cpp:274-338) for every unsynchronised stream from its
    // current position (optional: step() acquires such streams itself)
    void acquire();
    // decode the next n_frames frames of every stream (a stream that loses sync searches
    // the next null symbol and continues, as ofdmProcessor::run); false when a stream
    // ran out of samples (the frames it decoded were delivered)
    bool step();
    dabgpu_stream_state state(int stream) const;
private:
    config cfg_;
    dabgpu_pipe *pipe_ = nullptr;
    devbuf iq_, fic_, crc_, msc_, sf_, sfi_;
    int64_t stride_ = 0;
    std::vector<int64_t> navail_;
    int msc_stride_ = 0, sf_stride_ = 0, ndp_ = 0, maxbits_ = 0;
    std::vector<int> dp_index_;
    std::vector<int64_t> frames_done_;     // frames delivered per stream
    fib_cb fib_cb_;
    msc_cb msc_cb_;
    sf_cb sf_cb_;
};

}  // namespace dabgpu
