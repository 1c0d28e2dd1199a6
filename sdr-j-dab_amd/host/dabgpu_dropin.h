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

#include "dabgpu.h"

namespace dabgpu {

typedef std::complex<float> DSPCOMPLEX;   // dab-constants.h: DSPCOMPLEX

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

// ficHandler without Qt (fic-handler.cpp:143-321): process_ficBlock accumulates
// symbols 1..3 of a frame into the 4 FIC blocks, decodes each on the GPU and
// hands every FIB (256 bits, CRC field inverted as check_CRC_bits leaves it)
// with its CRC verdict to the callback that stands in for fibProcessor::process_FIB.
class ficHandler {
public:
    using fib_cb = std::function<void(const uint8_t *fib /*256 bits*/, bool crc_ok, int16_t ficno)>;
    explicit ficHandler(fib_cb cb, int16_t bitsperBlock = 2 * DABGPU_K);
    void process_ficBlock(int16_t *data, int16_t blkno);   // blkno 1..3
    int16_t get_ficRatio() const;                           // % of FIBs with a good CRC
private:
    fib_cb cb_;
    std::vector<int16_t> ofdm_input_;
    int index_ = 0, ficno_ = 0;
    int good_ = 0, total_ = 0;
    devbuf in_, bits_, crc_;
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
    int msc_stride_ = 0, sf_stride_ = 0, ndp_ = 0;
    std::vector<int> dp_index_;
    std::vector<int64_t> frames_done_;     // frames delivered per stream
    fib_cb fib_cb_;
    msc_cb msc_cb_;
    sf_cb sf_cb_;
};

}  // namespace dabgpu
