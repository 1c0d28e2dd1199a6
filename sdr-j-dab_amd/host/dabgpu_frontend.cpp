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

// ---- ofdmDecoder ------------------------------------------------------------------
ofdmDecoder::ofdmDecoder(DabParams *p, uint8_t freqSyncMethod, std::function<void(int)> show_snr)
    : method_(freqSyncMethod), show_snr_(std::move(show_snr)) {
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
        if (show_snr_) show_snr_(snr_);
        snrCount_ = 0;
    }
    return flag ? corr : 0;
}

void ofdmDecoder::processToken(DSPCOMPLEX *inv, int16_t *ibits, int32_t blkno) {   // ofdm-decoder.cpp:167-190
    (void)blkno;
    dabgpu_ctx *c = thread_context();
    smp_.upload(inv, sizeof(float) * 2 * DABGPU_TS);
    chk(dabgpu_ofdm_symbol(c, (const float *)smp_.get(), 1, (float *)spec_.get(), (int16_t *)bits_.get()),
        "dabgpu_ofdm_symbol");
    bits_.download(ibits, sizeof(int16_t) * 2 * DABGPU_K);
}

// ---- ofdmProcessor ----------------------------------------------------------------
static int16_t valueFor(int16_t b) {              // ofdm-processor.cpp:26-32 (dumpScaler)
    int16_t res = 1;
    while (--b > 1) res <<= 1;
    return res;
}

ofdmProcessor::ofdmProcessor(virtualInput *theRig, DabParams *p, signals sig, mscHandler *msc, ficHandler *fic,
                             int16_t threshold, uint8_t freqSyncMethod)
    : theRig_(theRig), sig_(std::move(sig)), msc_(msc), fic_(fic), threshold_(threshold), method_(freqSyncMethod) {
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
void ofdmProcessor::startDumping(FILE *f) { dumpFile_ = f; }
void ofdmProcessor::stopDumping() { dumpFile_ = nullptr; }

// The observables of one decoded frame, as ofdmProcessor::run / ofdmDecoder emit them:
// token length (samples between successive block-0 starts, averaged when within 10% of
// T_F, ofdm-processor.cpp:368-378), get_snr IIR, the corrector displays every
// INPUT_RATE / 7 samples (here checked once per frame).
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
    if (prev_window_ >= 0) sampleCnt_ += fi.window - prev_window_;
    prev_window_ = fi.window;
    if (sampleCnt_ > INPUT_RATE / 7) {
        if (sig_.show_fineCorrector) sig_.show_fineCorrector(fi.fine);
        if (sig_.show_coarseCorrector) sig_.show_coarseCorrector(fi.coarse / 1000);
        sampleCnt_ = 0;
    }
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
    // the stream in HBM: samples [base, end) of the device's sample sequence in one of
    // two buffers (the kernels index absolute sample numbers from buf - 2 * base);
    // when the decoder has moved past half of it, the tail moves to the other one
    const int64_t CAP = 24 * (int64_t)DABGPU_TF;
    devbuf bufs[2];
    bufs[0].resize(sizeof(float) * 2 * CAP);
    bufs[1].resize(sizeof(float) * 2 * CAP);
    int cur = 0;
    int64_t base = 0, end = 0, last_run = -1;
    const int16_t *ring = nullptr;
    int32_t R = 0;
    chk(dabgpu_pipe_softbits(pipe, &ring, &R), "dabgpu_pipe_softbits");
    std::vector<DSPCOMPLEX> chunk(1 << 16);
    std::vector<int16_t> dump;
    std::vector<int16_t> soft((size_t)75 * 3072);
    while (running_) {
        {
            std::lock_guard<std::mutex> g(ctl_);
            for (int op : pending_ops_) chk(dabgpu_pipe_control(pipe, 0, op), "dabgpu_pipe_control");
            pending_ops_.clear();
        }
        dabgpu_stream_state st;
        chk(dabgpu_pipe_state(pipe, 0, &st), "dabgpu_pipe_state");
        if (st.next_pos - base > CAP / 2) {        // slide the window
            const int64_t keep = end - st.next_pos;
            chk(dabgpu_memcpy_d2d(c, bufs[cur ^ 1].get(), (const float *)bufs[cur].get() + 2 * (st.next_pos - base),
                                   sizeof(float) * 2 * keep), "slide");
            cur ^= 1;
            base = st.next_pos;
        }
        const int32_t avail = theRig_->Samples();
        const int64_t room = CAP - (end - base);
        if (avail > 0 && room > 0) {
            const int32_t n = (int32_t)std::min<int64_t>({(int64_t)avail, (int64_t)chunk.size(), room});
            const int32_t got = theRig_->getSamples(chunk.data(), n);
            if (got > 0) {
                if (FILE *f = dumpFile_.load()) {  // ofdm-processor.cpp:150-157: raw samples * dumpScaler
                    dump.resize(2 * (size_t)got);
                    for (int i = 0; i < got; i++) {
                        dump[2 * i] = (int16_t)(chunk[i].real() * dumpScaler_);
                        dump[2 * i + 1] = (int16_t)(chunk[i].imag() * dumpScaler_);
                    }
                    std::fwrite(dump.data(), sizeof(int16_t), dump.size(), f);
                }
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
            const float *iq = (const float *)bufs[cur].get() - 2 * base;
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
            if (s2.frames_run == 0) break;
            if (!synced_) {
                synced_ = true;
                if (sig_.setSynced) sig_.setSynced(true);
            }
            dabgpu_frame_info fi;
            chk(dabgpu_pipe_frame_info(pipe, &fi), "dabgpu_pipe_frame_info");
            int32_t slot = 0;
            chk(dabgpu_pipe_frame_slot(pipe, 0, &slot), "dabgpu_pipe_frame_slot");
            chk(dabgpu_memcpy_d2h(c, soft.data(), ring + (size_t)slot * 75 * 3072, sizeof(int16_t) * soft.size()),
                "soft bits");
            emit_frame(fi);
            for (int16_t blk = 1; blk < 76; blk++) {   // ofdm-processor.cpp:421-442
                int16_t *ib = &soft[(size_t)(blk - 1) * 3072];
                if (blk < 4) {
                    if (fic_) fic_->process_ficBlock(ib, blk);
                } else if (msc_) {
                    msc_->process_mscBlock(ib, blk);
                }
            }
            frames_++;
        }
    }
}

}  // namespace dabgpu
