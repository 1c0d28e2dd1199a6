// dabgpu_frontend.cpp -- the OFDM side of the drop-in (dabgpu_dropin.h):
// setModeParameters, ofdmDecoder (one symbol per call) and ofdmProcessor (the
// reference's thread: samples from a virtualInput, the GPU front end, soft bits to the
// FIC and MSC handlers, the GUI's observables as callbacks).
#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>

#include "dabgpu_dropin.h"

namespace dabgpu {

namespace {
void chk(int rc, const char *what) {
    if (rc != DABGPU_OK) throw error(rc, std::string(what) + ": " + dabgpu_last_error());
}
constexpr int32_t INPUT_RATE = 2048000;
}  // namespace

void setModeParameters(DabParams *p, uint8_t mode) {              // gui.cpp:1361-1371
    if (mode != 1) throw error(DABGPU_E_UNSUP, "DAB mode " + std::to_string(mode) + ": the GPU path is Mode I");
    p->dabMode = 1;
    p->L = 76;
    p->K = 1536;
    p->T_null = 2656;
    p->T_F = 196608;
    p->T_s = 2552;
    p->T_u = 2048;
    p->guardLength = 504;
    p->carrierDiff = 1000;
}

// ---- libsndfile stand-in (a build with -DDABGPU_HAVE_SNDFILE uses libsndfile itself) --
#ifndef DABGPU_HAVE_SNDFILE
struct SNDFILE {
    FILE *f = nullptr;
    int channels = 2, samplerate = 0;
    int64_t frames = 0;                             // frames written
};
static void put_le(FILE *f, uint32_t v, int bytes) {
    for (int i = 0; i < bytes; i++) std::fputc((int)((v >> (8 * i)) & 0xFF), f);
}
static void wav_header(SNDFILE *s) {                          // RIFF/WAVE, fmt (PCM 16), data
    const uint32_t samplerate = (uint32_t)s->samplerate;
    const uint32_t data = (uint32_t)(s->frames * 2 * s->channels);
    std::fseek(s->f, 0, SEEK_SET);
    std::fwrite("RIFF", 1, 4, s->f);
    put_le(s->f, 36 + data, 4);
    std::fwrite("WAVEfmt ", 1, 8, s->f);
    put_le(s->f, 16, 4);
    put_le(s->f, 1, 2);                                       // PCM
    put_le(s->f, (uint32_t)s->channels, 2);
    put_le(s->f, samplerate, 4);
    put_le(s->f, samplerate * 2 * s->channels, 4);
    put_le(s->f, 2 * s->channels, 2);
    put_le(s->f, 16, 2);
    std::fwrite("data", 1, 4, s->f);
    put_le(s->f, data, 4);
}
SNDFILE *sf_open(const char *path, int mode, SF_INFO *info) {
    if (mode != SFM_WRITE || !info || info->format != (SF_FORMAT_WAV | SF_FORMAT_PCM_16) || info->channels < 1)
        return nullptr;
    FILE *f = std::fopen(path, "w+b");
    if (!f) return nullptr;
    SNDFILE *s = new SNDFILE;
    s->f = f;
    s->channels = info->channels;
    s->samplerate = info->samplerate;
    wav_header(s);
    return s;
}
int64_t sf_writef_short(SNDFILE *s, const int16_t *ptr, int64_t frames) {
    if (!s || frames <= 0) return 0;
    const size_t w = std::fwrite(ptr, sizeof(int16_t) * s->channels, (size_t)frames, s->f);
    s->frames += (int64_t)w;
    return (int64_t)w;
}
int sf_close(SNDFILE *s) {
    if (!s) return 0;
    wav_header(s);
    const int r = std::fclose(s->f);
    delete s;
    return r;
}
#endif

// ---- ofdmDecoder ------------------------------------------------------------------
std::atomic<int> ofdmDecoder::iq_count{0};

ofdmDecoder::ofdmDecoder(DabParams *p, RingBuffer<DSPCOMPLEX> *iqBuffer, DSPCOMPLEX *refTable, signals sig,
                         uint8_t freqSyncMethod)
    : ofdmDecoder(p, freqSyncMethod, sig.show_snr) {
    (void)refTable;                                  // refArg: in the device tables (ofdm-decoder.cpp:71-74)
    iqBuffer_ = iqBuffer;
    sig_ = std::move(sig);
}

ofdmDecoder::ofdmDecoder(DabParams *p, uint8_t freqSyncMethod, std::function<void(int)> show_snr)
    : method_(freqSyncMethod) {
    sig_.show_snr = std::move(show_snr);
    if (p->dabMode != 1) throw error(DABGPU_E_UNSUP, "ofdmDecoder: Mode I only");
    if (freqSyncMethod > 2) throw error(DABGPU_E_UNSUP, "ofdmDecoder: freqSyncMethod 0, 1 or 2");
    smp_.resize(sizeof(float) * 2 * DABGPU_TS);
    spec_.resize(sizeof(float) * 2 * DABGPU_TU);
    fr_.resize(sizeof(dabgpu_frame));
    corr_.resize(16);
    snrd_.resize(16);
    bits_.resize(sizeof(int16_t) * 2 * DABGPU_K);
}

int16_t ofdmDecoder::processBlock_0(DSPCOMPLEX *vi, bool flag) {   // ofdm-decoder.cpp:85-162
    dabgpu_ctx *c = thread_context();
    smp_.upload(vi, sizeof(float) * 2 * DABGPU_TU);
    dabgpu_frame f;
    std::memset(&f, 0, sizeof f);
    f.n_samples = DABGPU_TU;                      // the samples are mixed already: NCO phase 0
    f.flags = flag ? 1 : 0;
    fr_.upload(&f, sizeof f);
    chk(dabgpu_block0(c, (const float *)smp_.get(), (const dabgpu_frame *)fr_.get(), 1, method_,
                      (int16_t *)corr_.get(), (int16_t *)snrd_.get()), "dabgpu_block0");
    chk(dabgpu_ofdm_symbol(c, (const float *)smp_.get(), 0, (float *)spec_.get(), nullptr), "dabgpu_ofdm_symbol");
    int16_t corr = 0, s = 0;
    corr_.download(&corr, sizeof corr);
    snrd_.download(&s, sizeof s);
    snr_ = (int16_t)(0.7 * snr_ + 0.3 * s);       // ofdm-decoder.cpp:93-97
    if (++snrCount_ > 10) {
        if (sig_.show_snr) sig_.show_snr(snr_);
        snrCount_ = 0;
    }
    return flag ? corr : 0;
}

void ofdmDecoder::processToken(DSPCOMPLEX *inv, int16_t *ibits, int32_t blkno) {   // ofdm-decoder.cpp:167-206
    dabgpu_ctx *c = thread_context();
    smp_.upload(inv, sizeof(float) * 2 * DABGPU_TS);
    chk(dabgpu_ofdm_symbol(c, (const float *)smp_.get(), 1, (float *)spec_.get(), (int16_t *)bits_.get()),
        "dabgpu_ofdm_symbol");
    bits_.download(ibits, sizeof(int16_t) * 2 * DABGPU_K);
    // spec_ now holds this symbol's spectrum (natural bin order): the display carriers
    if (blkno == displayToken && ++iq_count > 7) {
        iq_count = 0;
        if (iqBuffer_) {
            std::vector<DSPCOMPLEX> x(DABGPU_TU);
            spec_.download(x.data(), sizeof(DSPCOMPLEX) * DABGPU_TU);
            iqBuffer_->putDataIntoBuffer(&x[0], DABGPU_K / 2);
            iqBuffer_->putDataIntoBuffer(&x[DABGPU_TU - 1 - DABGPU_K / 2], DABGPU_K / 2);
            if (sig_.showIQ) sig_.showIQ(DABGPU_K);
        }
    }
}

int16_t ofdmDecoder::get_snr(DSPCOMPLEX *v) {                        // ofdm-decoder.cpp:212-230
    dabgpu_ctx *c = thread_context();
    devbuf x(sizeof(DSPCOMPLEX) * DABGPU_TU), r(16);
    x.upload(v, sizeof(DSPCOMPLEX) * DABGPU_TU);
    chk(dabgpu_get_snr(c, (const float *)x.get(), (int16_t *)r.get()), "dabgpu_get_snr");
    int16_t out = 0;
    r.download(&out, sizeof out);
    return out;
}

// ---- ofdmProcessor ----------------------------------------------------------------
static int16_t valueFor(int16_t b) {              // ofdm-processor.cpp:26-32 (dumpScaler)
    int16_t res = 1;
    while (--b > 1) res <<= 1;
    return res;
}

ofdmProcessor::ofdmProcessor(virtualInput *theRig, DabParams *p, signals sig, mscHandler *msc, ficHandler *fic,
                             int16_t threshold, uint8_t freqSyncMethod)
    : ofdmProcessor(theRig, p, std::move(sig), msc, fic, threshold, nullptr, nullptr, freqSyncMethod) {}

ofdmProcessor::ofdmProcessor(virtualInput *theRig, DabParams *p, signals sig, mscHandler *msc, ficHandler *fic,
                             int16_t threshold, RingBuffer<DSPCOMPLEX> *spectrumBuffer,
                             RingBuffer<DSPCOMPLEX> *iqBuffer, uint8_t freqSyncMethod)
    : theRig_(theRig), sig_(std::move(sig)), msc_(msc), fic_(fic), threshold_(threshold), method_(freqSyncMethod),
      spectrumBuffer_(spectrumBuffer), iqBuffer_(iqBuffer) {
    if (p->dabMode != 1) throw error(DABGPU_E_UNSUP, "ofdmProcessor: Mode I only");
    dumpScaler_ = valueFor(theRig->bitDepth());
    running_ = true;
    thread_ = std::thread([this] {                // ofdm-processor.cpp:107: the constructor starts the thread
        try {
            run();
        } catch (const std::exception &e) {
            std::fprintf(stderr, "ofdmProcessor: %s\n", e.what());   // the reference's catch (int) ends the thread
        }
        running_ = false;
    });
}

ofdmProcessor::~ofdmProcessor() {
    stop();
    if (thread_.joinable()) thread_.join();
}

void ofdmProcessor::stop() { running_ = false; }
void ofdmProcessor::reset() {
    std::lock_guard<std::mutex> g(ctl_);
    pending_ops_.push_back(DABGPU_CTL_RESET);
}
void ofdmProcessor::coarseCorrectorOn() {
    std::lock_guard<std::mutex> g(ctl_);
    pending_ops_.push_back(DABGPU_CTL_COARSE_ON);
}
void ofdmProcessor::coarseCorrectorOff() {
    std::lock_guard<std::mutex> g(ctl_);
    pending_ops_.push_back(DABGPU_CTL_COARSE_OFF);
}
void ofdmProcessor::set_scanMode(bool b) {
    std::lock_guard<std::mutex> g(ctl_);
    pending_ops_.push_back(b ? DABGPU_CTL_SCAN_ON : DABGPU_CTL_SCAN_OFF);
}
void ofdmProcessor::startDumping(SNDFILE *f) { dumpSnd_ = f; }       // ofdm-processor.cpp:486-493
void ofdmProcessor::startDumping(FILE *f) { dumpFile_ = f; }
void ofdmProcessor::stopDumping() {
    dumpSnd_ = nullptr;
    dumpFile_ = nullptr;
}

// raw samples * dumpScaler as interleaved PCM16 (ofdm-processor.cpp:150-157, 204-213)
void ofdmProcessor::write_dump(const DSPCOMPLEX *v, int32_t n) {
    SNDFILE *sf = dumpSnd_.load();
    FILE *f = dumpFile_.load();
    if (!sf && !f) return;
    std::vector<int16_t> d(2 * (size_t)n);
    for (int i = 0; i < n; i++) {
        d[2 * i] = (int16_t)(v[i].real() * dumpScaler_);
        d[2 * i + 1] = (int16_t)(v[i].imag() * dumpScaler_);
    }
    if (sf) sf_writef_short(sf, d.data(), n);
    if (f) std::fwrite(d.data(), sizeof(int16_t), d.size(), f);
}

// The observables of one decoded frame, as ofdmProcessor::run / ofdmDecoder emit them:
// token length (samples between successive block-0 starts, averaged when within 10% of
// T_F, ofdm-processor.cpp:368-378), get_snr IIR (ofdm-decoder.cpp:93-97).
void ofdmProcessor::emit_frame(const dabgpu_frame_info &fi) {
    const int64_t block0 = fi.window + fi.start_index;
    if (last_block0_ >= 0) {
        const int64_t tokenLength = block0 - last_block0_;
        if (0.9 * DABGPU_TF <= tokenLength && tokenLength <= 1.1 * DABGPU_TF)
            avgTokenLength_ = (int32_t)(0.8 * avgTokenLength_ + 0.2 * tokenLength);
        if (++tokenCount_ > 10) {
            tokenCount_ = 0;
            if (sig_.show_avgTokenLength) sig_.show_avgTokenLength(avgTokenLength_);
        }
    }
    last_block0_ = block0;
    snr_ = (int16_t)(0.7 * snr_ + 0.3 * fi.snr);
    if (++snrCount_ > 10) {
        if (sig_.show_snr) sig_.show_snr(snr_);
        snrCount_ = 0;
    }
}

// sampleCnt past INPUT_RATE / 7 at the end of a getSample(s) call (ofdm-processor.cpp:170-180,
// 229-238): the corrector displays and, with a spectrumBuffer, the localBuffer -- the
// first 32768 raw samples read since the previous emission, read back from the device
// window -- into the ring + showSpectrum.  The correctors shown are the frame's.
void ofdmProcessor::spectrum_emit(const dabgpu_frame_info *fi) {
    if (fi) {
        last_fine_ = fi->fine;
        last_coarse_ = fi->coarse;
    }
    if (sig_.show_fineCorrector) sig_.show_fineCorrector(last_fine_);
    if (sig_.show_coarseCorrector) sig_.show_coarseCorrector(last_coarse_ / 1000);
    if (spectrumBuffer_ && win_) {
        specbuf_.resize(spectrumSize);
        chk(dabgpu_memcpy_d2h(thread_context(), specbuf_.data(), win_ + 2 * (spec_start_ - win_base_),
                              sizeof(DSPCOMPLEX) * spectrumSize), "spectrum samples");
        spectrumBuffer_->putDataIntoBuffer(specbuf_.data(), spectrumSize);
        if (sig_.showSpectrum) sig_.showSpectrum(spectrumSize);
    }
    spec_cnt_ = 0;
    spec_start_ = consumed_;                        // localCounter = 0
}
// getSample calls, one sample each, up to stream index `to` (null search, the T_u window)
void ofdmProcessor::consume_singles(int64_t to, const dabgpu_frame_info *fi) {
    constexpr int64_t LIM = INPUT_RATE / 7;
    while (consumed_ < to) {
        const int64_t need = LIM + 1 - spec_cnt_;   // samples until sampleCnt > LIM
        if (consumed_ + need <= to) {
            consumed_ += need;
            spec_cnt_ += need;
            spectrum_emit(fi);
        } else {
            spec_cnt_ += to - consumed_;
            consumed_ = to;
        }
    }
}
// one getSamples call of n samples
void ofdmProcessor::consume_block(int64_t n, const dabgpu_frame_info *fi) {
    consumed_ += n;
    spec_cnt_ += n;
    if (spec_cnt_ > INPUT_RATE / 7) spectrum_emit(fi);
}

void ofdmProcessor::run() {                                        // ofdm-processor.cpp:247-474
    dabgpu_ctx *c = thread_context();
    dabgpu_pipe_cfg pc;
    std::memset(&pc, 0, sizeof pc);
    pc.n_streams = 1;
    pc.n_frames = 1;
    pc.threshold = threshold_;
    pc.freq_sync_method = method_;
    dabgpu_pipe *pipe = nullptr;
    chk(dabgpu_pipe_create(c, &pc, &pipe), "dabgpu_pipe_create");
    struct PipeGuard {
        dabgpu_pipe *p;
        ~PipeGuard() { dabgpu_pipe_destroy(p); }
    } guard{pipe};
    // one ensemble: nothing decodes beside a null search, so it runs inside the run, in the
    // reference's order (the engine's default background search pays off for batches)
    chk(dabgpu_pipe_control(pipe, -1, DABGPU_CTL_ACQ_SYNC), "dabgpu_pipe_control");
    if (iqBuffer_) chk(dabgpu_pipe_set_display(pipe, 1), "dabgpu_pipe_set_display");
    // the stream in HBM: samples [base, end) of the device's sample sequence in one of
    // two buffers (the kernels index absolute sample numbers from buf - 2 * base);
    // when the decoder has moved past half of it, the tail moves to the other one (from
    // the spectrum feed's pending localBuffer start if that is earlier)
    const int64_t CAP = 24 * (int64_t)DABGPU_TF;
    devbuf bufs[2];
    bufs[0].resize(sizeof(float) * 2 * CAP);
    bufs[1].resize(sizeof(float) * 2 * CAP);
    int cur = 0;
    int64_t base = 0, end = 0, last_run = -1;
    const uint8_t *ring = nullptr;                  // RING8 bytes: ibits + 127
    int32_t R = 0;
    chk(dabgpu_pipe_softbits(pipe, &ring, &R), "dabgpu_pipe_softbits");
    std::vector<DSPCOMPLEX> chunk(1 << 16);
    std::vector<int16_t> soft((size_t)75 * 3072);
    std::vector<uint8_t> soft8(soft.size());
    std::vector<DSPCOMPLEX> carriers(DABGPU_K);
    while (running_) {
        {
            std::lock_guard<std::mutex> g(ctl_);
            for (int op : pending_ops_) chk(dabgpu_pipe_control(pipe, 0, op), "dabgpu_pipe_control");
            pending_ops_.clear();
        }
        dabgpu_stream_state st;
        chk(dabgpu_pipe_state(pipe, 0, &st), "dabgpu_pipe_state");
        if (st.next_pos - base > CAP / 2) {        // slide the window
            const int64_t from = spectrumBuffer_ ? std::min(st.next_pos, spec_start_) : st.next_pos;
            const int64_t keep = end - from;
            chk(dabgpu_memcpy_d2d(c, bufs[cur ^ 1].get(), (const float *)bufs[cur].get() + 2 * (from - base),
                                   sizeof(float) * 2 * keep), "slide");
            cur ^= 1;
            base = from;
        }
        const int32_t avail = theRig_->Samples();
        const int64_t room = CAP - (end - base);
        if (avail > 0 && room > 0) {
            const int32_t n = (int32_t)std::min<int64_t>({(int64_t)avail, (int64_t)chunk.size(), room});
            const int32_t got = theRig_->getSamples(chunk.data(), n);
            if (got > 0) {
                write_dump(chunk.data(), got);
                chk(dabgpu_memcpy_h2d(c, (float *)bufs[cur].get() + 2 * (end - base), chunk.data(),
                                      sizeof(float) * 2 * got), "upload");
                end += got;
            }
            if (end - last_run < DABGPU_TF / 4 && end - base < CAP) continue;   // gather more first
        } else if (end == last_run) {
            std::this_thread::sleep_for(std::chrono::milliseconds(1));          // getSample's wait
            continue;
        }
        last_run = end;
        // decode every frame the samples so far allow, one per pipeline run
        for (;;) {
            // token 0 (display off: an out-of-range set_displayToken) matches no blkno below
            const int16_t token = displayOff_.load() ? 0 : displayToken_.load();
            if (iqBuffer_ && token) chk(dabgpu_pipe_set_display_token(pipe, token), "dabgpu_pipe_set_display_token");
            const float *iq = (const float *)bufs[cur].get() - 2 * base;
            win_ = (const float *)bufs[cur].get();
            win_base_ = base;
            const int rc = dabgpu_pipe_run(pipe, iq, 0, &end, nullptr, nullptr, nullptr, 0, nullptr);
            if (rc != DABGPU_OK && rc != DABGPU_E_STATE) chk(rc, "dabgpu_pipe_run");
            dabgpu_stream_state s2;
            chk(dabgpu_pipe_state(pipe, 0, &s2), "dabgpu_pipe_state");
            while (no_signal_ < s2.no_signal) {
                no_signal_++;
                if (sig_.No_Signal_Found) sig_.No_Signal_Found();
            }
            if (s2.resyncs > resyncs_) {           // goto notSynced: setSynced (false)
                resyncs_ = s2.resyncs;
                synced_ = false;
                if (sig_.setSynced) sig_.setSynced(false);
            }
            if (s2.frames_run == 0) {
                consume_singles(s2.next_pos, nullptr);   // the null search so far: getSample calls
                break;
            }
            if (!synced_) {
                synced_ = true;
                if (sig_.setSynced) sig_.setSynced(true);
            }
            dabgpu_frame_info fi;
            chk(dabgpu_pipe_frame_info(pipe, &fi), "dabgpu_pipe_frame_info");
            int32_t slot = 0;
            chk(dabgpu_pipe_frame_slot(pipe, 0, &slot), "dabgpu_pipe_frame_slot");
            chk(dabgpu_memcpy_d2h(c, soft8.data(), ring + (size_t)slot * 75 * 3072, soft8.size()), "soft bits");
            for (size_t i = 0; i < soft.size(); i++) soft[i] = (int16_t)(soft8[i] - 127);   // processToken's ibits
            // the frame's getSample(s) calls (ofdm-processor.cpp:344-453): the null search and
            // the T_u window one sample at a time, the rest of block 0, 75 symbols, the null
            consume_singles(fi.window + DABGPU_TU, &fi);
            consume_block(fi.start_index, &fi);
            for (int l = 1; l < 76; l++) consume_block(DABGPU_TS, &fi);
            consume_block(DABGPU_TNULL, &fi);
            emit_frame(fi);
            for (int16_t blk = 1; blk < 76; blk++) {   // ofdm-processor.cpp:421-442
                int16_t *ib = &soft[(size_t)(blk - 1) * 3072];
                if (blk < 4) {
                    if (fic_) fic_->process_ficBlock(ib, blk);
                } else if (msc_) {
                    msc_->process_mscBlock(ib, blk);
                }
                // processToken's display token (ofdm-decoder.cpp:192-206), exported by the demod
                if (blk == token && ++ofdmDecoder::iq_count > 7) {
                    ofdmDecoder::iq_count = 0;
                    if (iqBuffer_) {
                        chk(dabgpu_pipe_iq_display(pipe, 0, 0, (float *)carriers.data()), "dabgpu_pipe_iq_display");
                        iqBuffer_->putDataIntoBuffer(carriers.data(), DABGPU_K / 2);
                        iqBuffer_->putDataIntoBuffer(carriers.data() + DABGPU_K / 2, DABGPU_K / 2);
                        if (sig_.showIQ) sig_.showIQ(DABGPU_K);
                    }
                }
            }
            frames_++;
        }
    }
}

}  // namespace dabgpu
