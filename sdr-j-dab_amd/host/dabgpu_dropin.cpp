// dabgpu_dropin.cpp -- see dabgpu_dropin.h.  Every class is a thin host shell over
// the C ABI: buffers are allocated once per object, each call is one upload, one
// (or a few) kernel launches and one download on the thread's HIP stream.
#include "dabgpu_dropin.h"

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>

namespace dabgpu {

namespace {
int g_device = 0;

struct ctx_holder {
    dabgpu_ctx *c = nullptr;
    ~ctx_holder() {
        if (c) dabgpu_ctx_destroy(c);
    }
};
thread_local ctx_holder t_ctx;

void chk(int rc, const char *what) {
    if (rc != DABGPU_OK) throw error(rc, std::string(what) + ": " + dabgpu_last_error());
}
}  // namespace

void set_device(int device) { g_device = device; }

dabgpu_ctx *thread_context() {
    if (!t_ctx.c) chk(dabgpu_ctx_create(g_device, &t_ctx.c), "dabgpu_ctx_create");
    return t_ctx.c;
}

devbuf::~devbuf() {
    if (p_ && t_ctx.c) dabgpu_free(t_ctx.c, p_);
}

void devbuf::resize(size_t bytes) {
    if (bytes <= n_) return;
    dabgpu_ctx *c = thread_context();
    if (p_) dabgpu_free(c, p_);
    p_ = nullptr;
    n_ = 0;
    chk(dabgpu_alloc(c, bytes, &p_), "dabgpu_alloc");
    n_ = bytes;
}

void devbuf::upload(const void *h, size_t bytes) {
    resize(bytes);
    chk(dabgpu_memcpy_h2d(thread_context(), p_, h, bytes), "dabgpu_memcpy_h2d");
}

void devbuf::download(void *h, size_t bytes) const {
    chk(dabgpu_memcpy_d2h(thread_context(), h, p_, bytes), "dabgpu_memcpy_d2h");
}

// ---- viterbi family --------------------------------------------------------
viterbi::viterbi(int16_t wordlength) : wordlength_(wordlength) {
    in_.resize(sizeof(int16_t) * 4 * (wordlength + 6));
    out_.resize(wordlength + 16);
}

void viterbi::deconvolve(int16_t *input, uint8_t *output) {
    in_.upload(input, sizeof(int16_t) * 4 * (wordlength_ + 6));
    chk(dabgpu_viterbi(thread_context(), (const int16_t *)in_.get(), 1, wordlength_, (uint8_t *)out_.get()),
        "dabgpu_viterbi");
    out_.download(output, wordlength_);
}

namespace {
bool msc_one(const dabgpu_subch &sub, devbuf &in, devbuf &out, int16_t *v, int32_t size, uint8_t *outBuffer) {
    const int nbits = 24 * sub.bitRate;
    in.upload(v, sizeof(int16_t) * size);
    const int rc = dabgpu_msc_deconvolve(thread_context(), (const int16_t *)in.get(), size, &sub, 1,
                                         (uint8_t *)out.get(), nbits);
    if (rc == DABGPU_E_UNSUP || rc == DABGPU_E_ARG) return false;   // profile undefined / fragment too short
    chk(rc, "dabgpu_msc_deconvolve");
    out.download(outBuffer, nbits);
    return true;
}
}  // namespace

uep_deconvolve::uep_deconvolve(int16_t bitRate, int16_t protLevel) : viterbi(24 * bitRate) {
    sub_ = dabgpu_subch{0, 0, bitRate, protLevel, 0, DABGPU_SUBCH_RAW};
}

bool uep_deconvolve::deconvolve(int16_t *v, int32_t size, uint8_t *outBuffer) {
    return msc_one(sub_, in_, out_, v, size, outBuffer);
}

eep_deconvolve::eep_deconvolve(int16_t bitRate, int16_t protLevel) : viterbi(24 * bitRate) {
    sub_ = dabgpu_subch{0, 0, bitRate, protLevel, 1, DABGPU_SUBCH_RAW};
}

bool eep_deconvolve::deconvolve(int16_t *v, int32_t size, uint8_t *outBuffer) {
    return msc_one(sub_, in_, out_, v, size, outBuffer);
}

// ---- reedSolomon -------------------------------------------------------------
reedSolomon::reedSolomon(uint16_t symsize, uint16_t gfpoly, uint16_t fcr, uint16_t prim, uint16_t nroots) {
    if (symsize != 8 || gfpoly != 0435 || fcr != 0 || prim != 1 || nroots != 10)
        throw error(DABGPU_E_UNSUP, "reedSolomon: only the DAB+ code (8, 0435, 0, 1, 10) runs on the GPU");
    in_.resize(120);
    out_.resize(112);
    ret_.resize(16);
}

int16_t reedSolomon::dec(const uint8_t *data_in, uint8_t *data_out, int16_t cutlen) {
    if (cutlen != 135) throw error(DABGPU_E_UNSUP, "reedSolomon::dec: only cutlen 135 (RS(120,110))");
    in_.upload(data_in, 120);
    chk(dabgpu_rs_decode(thread_context(), (const uint8_t *)in_.get(), 1, (uint8_t *)out_.get(), (int16_t *)ret_.get()),
        "dabgpu_rs_decode");
    int16_t r = 0;
    out_.download(data_out, 110);
    ret_.download(&r, sizeof r);
    return r;
}

// ---- phaseReference ------------------------------------------------------------
phaseReference::phaseReference(int16_t threshold) : threshold_(threshold) {
    iq_.resize(sizeof(float) * 2 * DABGPU_TU);
    fr_.resize(sizeof(dabgpu_frame));
    si_.resize(16);
}

int32_t phaseReference::findIndex(DSPCOMPLEX *v) {
    iq_.upload(v, sizeof(float) * 2 * DABGPU_TU);
    dabgpu_frame f;
    std::memset(&f, 0, sizeof f);
    f.n_samples = DABGPU_TU;                      // samples already mixed: NCO phase 0
    fr_.upload(&f, sizeof f);
    chk(dabgpu_prs_sync(thread_context(), (const float *)iq_.get(), (const dabgpu_frame *)fr_.get(), 1, threshold_,
                        (int32_t *)si_.get(), nullptr, nullptr),
        "dabgpu_prs_sync");
    int32_t r = 0;
    si_.download(&r, sizeof r);
    return r;
}

// ---- ficHandler -------------------------------------------------------------------
// The reference's signals are queued to the GUI thread (Qt); here the FIG parser's
// events are collected under fibHandling_ and fired after it is released, so a slot may
// call back into kindofService / dataforAudioService / clearEnsemble without deadlock.
ficHandler::ficHandler(signals sig, int16_t bitsperBlock) : sig_(std::move(sig)) {
    init(bitsperBlock);
    if (sig_.nameofEnsemble)
        fibProcessor_.on_ensemble([this](uint32_t id, const std::string &name) {
            pending_.push_back([this, id, name] { sig_.nameofEnsemble(id, name); });
        });
    if (sig_.addtoEnsemble)
        fibProcessor_.on_service([this](const std::string &label) {
            pending_.push_back([this, label] { sig_.addtoEnsemble(label); });
        });
}

ficHandler::ficHandler(fib_cb cb, int16_t bitsperBlock) : cb_(std::move(cb)) { init(bitsperBlock); }

void ficHandler::init(int16_t bitsperBlock) {
    if (bitsperBlock != 2 * DABGPU_K) throw error(DABGPU_E_UNSUP, "ficHandler: Mode I (3072 bits per block) only");
    ofdm_input_.assign(2304, 0);
    in_.resize(sizeof(int16_t) * 2304);
    bits_.resize(768);
    crc_.resize(16);
}

void ficHandler::process_ficBlock(int16_t *data, int16_t blkno) {   // fic-handler.cpp:192-224
    if (!running_.load()) return;
    if (blkno == 1) {
        index_ = 0;
        ficno_ = 0;
    }
    for (int i = 0; i < 2 * DABGPU_K; i++) {
        ofdm_input_[index_++] = data[i];
        if (index_ >= 2304) {
            // process_ficInput (fic-handler.cpp:241-321) on the GPU
            in_.upload(ofdm_input_.data(), sizeof(int16_t) * 2304);
            chk(dabgpu_fic_decode(thread_context(), (const int16_t *)in_.get(), 1, (uint8_t *)bits_.get(),
                                  (uint8_t *)crc_.get()),
                "dabgpu_fic_decode");
            uint8_t bits[768], ok[3];
            bits_.download(bits, 768);
            crc_.download(ok, 3);
            std::vector<std::function<void()>> events;
            {
                std::lock_guard<std::mutex> g(fibHandling_);          // fic-handler.cpp:304-320
                for (int k = 0; k < 3; k++) {
                    total_++;
                    good_ += ok[k] ? 1 : 0;
                    if (sig_.show_ficCRC) {
                        const bool b = ok[k] != 0;
                        pending_.push_back([this, b] { sig_.show_ficCRC(b); });
                    }
                    if (ok[k]) fibProcessor_.process_FIB(bits + 256 * k, (uint16_t)ficno_);
                }
                events.swap(pending_);
            }
            for (auto &e : events) e();                               // outside the lock
            for (int k = 0; k < 3; k++)
                if (cb_) cb_(bits + 256 * k, ok[k] != 0, (int16_t)ficno_);
            index_ = 0;
            ficno_++;
        }
    }
}

int16_t ficHandler::get_ficRatio() const { return total_ ? (int16_t)(100 * good_ / total_) : 0; }

void ficHandler::clearEnsemble() {                                   // fic-handler.cpp:159-163
    std::lock_guard<std::mutex> g(fibHandling_);
    fibProcessor_.clearEnsemble();
}

uint8_t ficHandler::kindofService(const std::string &s) {           // fic-handler.cpp:165-171
    std::lock_guard<std::mutex> g(fibHandling_);
    return fibProcessor_.kindofService(s);
}

void ficHandler::dataforAudioService(const std::string &s, audiodata *d) {   // :174-178
    std::lock_guard<std::mutex> g(fibHandling_);
    (void)fibProcessor_.dataforAudioService(s, d);
}

void ficHandler::dataforDataService(const std::string &s, packetdata *d) {   // :180-184
    std::lock_guard<std::mutex> g(fibHandling_);
    (void)fibProcessor_.dataforDataService(s, d);
}

void ficHandler::stop() { running_.store(false); }                  // fic-handler.cpp:155-157

// ---- ensembleDecoder -------------------------------------------------------------
ensembleDecoder::ensembleDecoder(const config &cfg) : cfg_(cfg) {
    dabgpu_pipe_cfg pc;
    std::memset(&pc, 0, sizeof pc);
    pc.n_streams = cfg.n_streams;
    pc.n_frames = cfg.n_frames;
    pc.n_subch = (int32_t)cfg.subch.size();
    pc.threshold = cfg.threshold;
    pc.freq_sync_method = 1;
    pc.subch = cfg.subch.data();
    chk(dabgpu_pipe_create(thread_context(), &pc, &pipe_), "dabgpu_pipe_create");
    int maxbits = 768, maxrs = 0;
    for (size_t i = 0; i < cfg.subch.size(); i++) {
        maxbits = std::max(maxbits, 24 * (int)cfg.subch[i].bitRate);
        if (cfg.subch[i].flags & DABGPU_SUBCH_DABPLUS) {
            dp_index_.push_back((int)i);
            maxrs = std::max(maxrs, cfg.subch[i].bitRate / 8);
        }
    }
    ndp_ = (int)dp_index_.size();
    // the MSC and the FIBs leave the GPU packed (8 bits per byte, 1/8 of the bytes over
    // PCIe) and are unpacked here for the one-bit-per-byte consumers (dab-concurrent.cpp:191,
    // fibProcessor::process_FIB)
    chk(dabgpu_pipe_set_packed(pipe_, DABGPU_PACK_MSC | DABGPU_PACK_FIC), "dabgpu_pipe_set_packed");
    msc_stride_ = ((maxbits + 7) / 8 + 15) / 16 * 16;
    maxbits_ = maxbits;
    sf_stride_ = std::max(16, 110 * maxrs);
    const size_t SF = (size_t)cfg.n_streams * cfg.n_frames;
    // only the superframes a run completes cross PCIe (DABGPU_SF_SLOTS per subchannel)
    if (ndp_) chk(dabgpu_pipe_set_dabplus_compact(pipe_, 1), "dabgpu_pipe_set_dabplus_compact");
    fic_.resize(SF * 4 * 96);
    crc_.resize(SF * 12);
    msc_.resize(std::max<size_t>(1, SF * 4 * cfg.subch.size() * msc_stride_));
    if (ndp_) {
        sf_.resize(SF * 4 * ndp_ * sf_stride_);
        sfi_.resize(SF * 4 * ndp_ * sizeof(dabgpu_superframe));
    }
}

ensembleDecoder::~ensembleDecoder() {
    if (pipe_) dabgpu_pipe_destroy(pipe_);
}

void ensembleDecoder::load(const std::vector<const DSPCOMPLEX *> &samples, const std::vector<int64_t> &n) {
    if ((int)samples.size() != cfg_.n_streams || (int)n.size() != cfg_.n_streams)
        throw error(DABGPU_E_ARG, "ensembleDecoder::load: one sample array per stream");
    stride_ = 0;
    for (int64_t k : n) stride_ = std::max(stride_, k);
    iq_.resize(sizeof(float) * 2 * (size_t)stride_ * cfg_.n_streams);
    for (int s = 0; s < cfg_.n_streams; s++)
        chk(dabgpu_memcpy_h2d(thread_context(), (float *)iq_.get() + 2 * stride_ * s, samples[s],
                              sizeof(float) * 2 * n[s]),
            "dabgpu_memcpy_h2d");
    navail_ = n;
    frames_done_.assign(cfg_.n_streams, 0);
    chk(dabgpu_pipe_set_iq_format(pipe_, DABGPU_IQ_F32), "dabgpu_pipe_set_iq_format");
}

void ensembleDecoder::load_recorded(int format, const std::vector<const void *> &samples, const std::vector<int64_t> &n) {
    if ((int)samples.size() != cfg_.n_streams || (int)n.size() != cfg_.n_streams)
        throw error(DABGPU_E_ARG, "ensembleDecoder::load_recorded: one sample array per stream");
    if (format != DABGPU_IQ_S16 && format != DABGPU_IQ_U8)
        throw error(DABGPU_E_ARG, "ensembleDecoder::load_recorded: format DABGPU_IQ_S16 or DABGPU_IQ_U8");
    const size_t bps = format == DABGPU_IQ_S16 ? 4 : 2;      // bytes per I/Q pair
    stride_ = 0;
    for (int64_t k : n) stride_ = std::max(stride_, k);
    iq_.resize(bps * (size_t)stride_ * cfg_.n_streams);
    for (int s = 0; s < cfg_.n_streams; s++)
        chk(dabgpu_memcpy_h2d(thread_context(), (char *)iq_.get() + bps * stride_ * s, samples[s], bps * n[s]),
            "dabgpu_memcpy_h2d");
    navail_ = n;
    frames_done_.assign(cfg_.n_streams, 0);
    chk(dabgpu_pipe_set_iq_format(pipe_, format), "dabgpu_pipe_set_iq_format");
}

namespace {
// the data chunk of an .sdr recording: what wavFiles accepts (wavfiles.cpp:56-69 via
// libsndfile: 2 channels, 2048000 Hz, 16-bit PCM; WAVE_FORMAT_EXTENSIBLE with the PCM
// subformat too).  Returns the payload's byte offset and size.
std::pair<int64_t, int64_t> sdr_payload(std::FILE *f, const std::string &path) {
    auto u32 = [](const uint8_t *b) { return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24; };
    auto u16 = [](const uint8_t *b) { return (uint32_t)b[0] | (uint32_t)b[1] << 8; };
    uint8_t h[12];
    if (std::fread(h, 1, 12, f) != 12 || std::memcmp(h, "RIFF", 4) || std::memcmp(h + 8, "WAVE", 4))
        throw error(DABGPU_E_ARG, path + ": not a RIFF/WAVE file");
    int64_t off = 12;
    bool fmt_ok = false, have_fmt = false;
    for (;;) {
        uint8_t ck[8];
        if (std::fread(ck, 1, 8, f) != 8) throw error(DABGPU_E_ARG, path + ": no data chunk");
        const int64_t n = u32(ck + 4);
        off += 8;
        if (!std::memcmp(ck, "fmt ", 4)) {
            std::vector<uint8_t> b((size_t)n);
            if (n < 16 || std::fread(b.data(), 1, (size_t)n, f) != (size_t)n) throw error(DABGPU_E_ARG, path + ": bad fmt chunk");
            uint32_t tag = u16(&b[0]);
            if (tag == 0xFFFE && n >= 26) tag = u16(&b[24]);       // WAVE_FORMAT_EXTENSIBLE: the subformat
            fmt_ok = tag == 1 && u16(&b[2]) == 2 && u32(&b[4]) == 2048000 && u16(&b[14]) == 16;
            have_fmt = true;
            if (n & 1) std::fseek(f, 1, SEEK_CUR);
        } else if (!std::memcmp(ck, "data", 4)) {
            if (!have_fmt || !fmt_ok)
                throw error(DABGPU_E_ARG, path + ": not a recorded DAB file (need PCM16, 2 channels, 2048000 Hz)");
            return {off, n};
        } else {
            std::fseek(f, (long)(n + (n & 1)), SEEK_CUR);
        }
        off += n + (n & 1);
    }
}
}  // namespace

void ensembleDecoder::load_files(const std::vector<std::string> &paths) {
    if ((int)paths.size() != cfg_.n_streams) throw error(DABGPU_E_ARG, "ensembleDecoder::load_files: one file per stream");
    auto is_raw = [](const std::string &p) { return p.size() >= 4 && p.compare(p.size() - 4, 4, ".raw") == 0; };
    const bool raw = !paths.empty() && is_raw(paths[0]);
    for (const std::string &p : paths)
        if (is_raw(p) != raw) throw error(DABGPU_E_ARG, "ensembleDecoder::load_files: .raw and .sdr files mixed");
    const int format = raw ? DABGPU_IQ_U8 : DABGPU_IQ_S16;
    const size_t bps = raw ? 2 : 4;
    struct closer { void operator()(std::FILE *f) const { if (f) std::fclose(f); } };
    std::vector<std::unique_ptr<std::FILE, closer>> files;
    std::vector<std::pair<int64_t, int64_t>> payload;
    std::vector<int64_t> n;
    for (const std::string &p : paths) {
        std::unique_ptr<std::FILE, closer> f(std::fopen(p.c_str(), "rb"));
        if (!f) throw error(DABGPU_E_ARG, p + ": cannot open");
        std::pair<int64_t, int64_t> pl{0, 0};
        if (raw) {
            std::fseek(f.get(), 0, SEEK_END);
            pl = {0, (int64_t)std::ftell(f.get())};
        } else {
            pl = sdr_payload(f.get(), p);
            std::fseek(f.get(), 0, SEEK_END);
            pl.second = std::min<int64_t>(pl.second, (int64_t)std::ftell(f.get()) - pl.first);   // a truncated recording
        }
        n.push_back(pl.second / (int64_t)bps);
        payload.push_back(pl);
        files.push_back(std::move(f));
    }
    stride_ = 0;
    for (int64_t k : n) stride_ = std::max(stride_, k);
    iq_.resize(bps * (size_t)stride_ * cfg_.n_streams);
    std::vector<char> piece((size_t)1 << 24);
    for (int s = 0; s < cfg_.n_streams; s++) {
        std::FILE *f = files[s].get();
        std::fseek(f, (long)payload[s].first, SEEK_SET);
        for (int64_t done = 0, total = n[s] * (int64_t)bps; done < total;) {
            const size_t want = (size_t)std::min<int64_t>((int64_t)piece.size(), total - done);
            if (std::fread(piece.data(), 1, want, f) != want) throw error(DABGPU_E_ARG, paths[s] + ": short read");
            chk(dabgpu_memcpy_h2d(thread_context(), (char *)iq_.get() + bps * stride_ * s + done, piece.data(), want),
                "dabgpu_memcpy_h2d");
            done += (int64_t)want;
        }
    }
    navail_ = n;
    frames_done_.assign(cfg_.n_streams, 0);
    chk(dabgpu_pipe_set_iq_format(pipe_, format), "dabgpu_pipe_set_iq_format");
}

void ensembleDecoder::acquire() {
    // unsynchronised streams search from where they are (sample 0 for a new decoder,
    // the position after a sync loss otherwise: notSynced continues, ofdm-processor.cpp:274)
    std::vector<int64_t> start(cfg_.n_streams, 0);
    for (int s = 0; s < cfg_.n_streams; s++) {
        dabgpu_stream_state st;
        chk(dabgpu_pipe_state(pipe_, s, &st), "dabgpu_pipe_state");
        start[s] = st.next_pos;
    }
    const int rc = dabgpu_pipe_acquire(pipe_, (const float *)iq_.get(), stride_, start.data(), navail_.data());
    if (rc != DABGPU_OK && rc != DABGPU_E_STATE) chk(rc, "dabgpu_pipe_acquire");
}

bool ensembleDecoder::step() {
    const int S = cfg_.n_streams, F = cfg_.n_frames, NS = (int)cfg_.subch.size();
    std::vector<uint8_t> valid((size_t)S * 4 * F);
    const int rc = dabgpu_pipe_run(pipe_, (const float *)iq_.get(), stride_, navail_.data(), (uint8_t *)fic_.get(),
                                   (uint8_t *)crc_.get(), NS ? (uint8_t *)msc_.get() : nullptr, msc_stride_,
                                   valid.data());
    if (rc != DABGPU_OK && rc != DABGPU_E_STATE) chk(rc, "dabgpu_pipe_run");
    const bool ok = rc == DABGPU_OK;
    chk(dabgpu_pipe_sync(pipe_), "dabgpu_pipe_sync");
    // frames committed per stream (a stream that lost sync re-acquired inside the run;
    // one that ran out of samples committed fewer): FIC and MSC for those
    std::vector<dabgpu_frame_info> fr((size_t)S * F);
    chk(dabgpu_pipe_frame_info(pipe_, fr.data()), "dabgpu_pipe_frame_info");
    std::vector<uint8_t> fic((size_t)S * F * 4 * 96), crc((size_t)S * F * 12);
    fic_.download(fic.data(), fic.size());
    crc_.download(crc.data(), crc.size());
    uint8_t fib[256];
    for (int s = 0; s < S && fib_cb_; s++)
        for (int f = 0; f < F; f++) {
            if (!fr[(size_t)s * F + f].committed) continue;
            for (int b = 0; b < 4; b++)
                for (int k = 0; k < 3; k++) {
                    const uint8_t *pk = fic.data() + (((size_t)s * F + f) * 4 + b) * 96 + 32 * k;   // FIB bytes
                    for (int i = 0; i < 256; i++) fib[i] = (uint8_t)((pk[i >> 3] >> (7 - (i & 7))) & 1);
                    fib_cb_(s, frames_done_[s] + f, b, fib, crc[((size_t)s * F + f) * 12 + 3 * b + k] != 0);
                }
        }
    if (NS && msc_cb_) {
        std::vector<uint8_t> msc((size_t)S * 4 * F * NS * msc_stride_), bits(maxbits_);
        msc_.download(msc.data(), msc.size());
        for (int s = 0; s < S; s++)
            for (int c = 0; c < 4 * F; c++) {
                if (!valid[(size_t)s * 4 * F + c]) continue;
                for (int k = 0; k < NS; k++) {
                    const uint8_t *pk = msc.data() + (((size_t)s * 4 * F + c) * NS + k) * msc_stride_;
                    const int nbits = 24 * cfg_.subch[k].bitRate;
                    for (int i = 0; i < nbits; i++) bits[i] = (uint8_t)((pk[i >> 3] >> (7 - (i & 7))) & 1);
                    msc_cb_(s, 4 * frames_done_[s] + c, k, bits.data(), nbits);
                }
            }
    }
    if (NS && ndp_) {
        chk(dabgpu_pipe_dabplus(pipe_, (uint8_t *)sf_.get(), sf_stride_, (dabgpu_superframe *)sfi_.get()),
            "dabgpu_pipe_dabplus");
        chk(dabgpu_pipe_sync(pipe_), "dabgpu_pipe_sync");
        if (sf_cb_) {
            std::vector<dabgpu_superframe> info((size_t)S * 4 * F * ndp_);
            const int slots = DABGPU_SF_SLOTS(F);
            std::vector<uint8_t> bytes((size_t)S * ndp_ * slots * sf_stride_);
            sfi_.download(info.data(), info.size() * sizeof(dabgpu_superframe));
            sf_.download(bytes.data(), bytes.size());
            for (size_t r = 0; r < info.size(); r++) {
                if (info[r].status < 0) continue;
                const int d = (int)(r % ndp_);
                const int c = (int)((r / ndp_) % (4 * F));
                const int s = (int)(r / ndp_ / (4 * F));
                const int k = dp_index_[d];
                const int slot = info[r].reserved;           // compact output: the superframe's slot
                const bool has = info[r].status == 3 && slot < slots;
                sf_cb_(s, 4 * frames_done_[s] + c, k, info[r],
                       bytes.data() + (((size_t)s * ndp_ + d) * slots + (has ? slot : 0)) * sf_stride_,
                       has ? 110 * (cfg_.subch[k].bitRate / 8) : 0);
            }
        }
    }
    for (int s = 0; s < S; s++) {
        dabgpu_stream_state st;
        chk(dabgpu_pipe_state(pipe_, s, &st), "dabgpu_pipe_state");
        frames_done_[s] += st.frames_run;
    }
    return ok;
}

dabgpu_stream_state ensembleDecoder::state(int stream) const {
    dabgpu_stream_state st;
    chk(dabgpu_pipe_state(pipe_, stream, &st), "dabgpu_pipe_state");
    return st;
}

}  // namespace dabgpu
