// dabgpu_backend.cpp -- the MSC side of the drop-in (dabgpu_dropin.h): mp4Processor,
// dabConcurrent, mscDatagroup, mscHandler.  Viterbi / depuncturing / energy dispersal
// and the Reed-Solomon decoding run on the GPU through the C ABI; the bookkeeping
// around them is the reference's, on the host.
#include <algorithm>
#include <cstring>
#include <string>

#include "dabgpu_dropin.h"

namespace dabgpu {

namespace {
void chk(int rc, const char *what) {
    if (rc != DABGPU_OK) throw error(rc, std::string(what) + ": " + dabgpu_last_error());
}

// firecode_checker (firecode-checker.cpp:31-94): g(x) = (x^11 + 1)(x^5 + x^3 + x^2 + x + 1)
// over bytes 2..10 followed by the two check bytes 0..1, table driven
struct FireTab {
    uint16_t tab[256];
    FireTab() {
        static const uint8_t g[16] = {1, 1, 1, 1, 0, 1, 0, 0, 0, 0, 0, 1, 1, 1, 1, 0};
        uint16_t itab[8];
        for (int i = 0; i < 8; i++) {
            uint8_t regs[16] = {};
            regs[8 + i] = 1;
            for (int r = 0; r < 8; r++) {
                const uint8_t z = regs[15];
                for (int j = 15; j > 0; j--) regs[j] = regs[j - 1] ^ (z & g[j]);
                regs[0] = z;
            }
            uint16_t v = 0;
            for (int j = 15; j >= 0; j--) v = (uint16_t)((v << 1) | regs[j]);
            itab[i] = v;
        }
        for (int i = 0; i < 256; i++) {
            tab[i] = 0;
            for (int j = 0; j < 8; j++)
                if (i & (1 << j)) tab[i] ^= itab[j];
        }
    }
};
bool fire_check(const uint8_t *x) {
    static const FireTab ft;
    uint16_t state = (uint16_t)((x[2] << 8) | x[3]);
    for (int i = 4; i < 13; i++) {
        const uint8_t b = i < 11 ? x[i] : x[i - 11];
        const uint16_t is = ft.tab[state >> 8];
        state = (uint16_t)(((is & 0x00ff) ^ b) | ((is ^ state << 8) & 0xff00));
    }
    return state == 0;
}

// dabPlus_crc (mp4processor.cpp:40-61): CRC-CCITT from all ones, the AU's last two
// bytes the inverted CRC
bool dabPlus_crc(const uint8_t *msg, int16_t len) {
    uint16_t acc = 0xFFFF;
    for (int i = 0; i < len; i++) {
        uint16_t data = (uint16_t)(msg[i] << 8);
        for (int j = 8; j > 0; j--) {
            acc = ((data ^ acc) & 0x8000) ? (uint16_t)((acc << 1) ^ 0x1021) : (uint16_t)(acc << 1);
            data = (uint16_t)(data << 1);
        }
    }
    const uint16_t crc = (uint16_t)~((msg[len] << 8) | msg[len + 1]);
    return crc == acc;
}

int16_t interleave_delay(int i) {                  // dab-concurrent.cpp:42-43: 15 - brev4(i & 15)
    const int b = i & 15;
    return (int16_t)(15 - (((b & 1) << 3) | ((b & 2) << 1) | ((b & 4) >> 1) | ((b & 8) >> 3)));
}
}  // namespace

// ---- mp4Processor ---------------------------------------------------------------
mp4Processor::mp4Processor(int16_t bitRate, au_cb cb)
    : bitRate_(bitRate), RSDims_((int16_t)(bitRate / 8)), cb_(std::move(cb)),
      frameBytes_((size_t)RSDims_ * 120, 0), outVector_((size_t)RSDims_ * 110, 0) {
    if (bitRate < 8 || bitRate % 8 || bitRate > 384) throw error(DABGPU_E_UNSUP, "mp4Processor: bitRate");
    rsin_.resize((size_t)RSDims_ * 120);
    rsout_.resize((size_t)RSDims_ * 110 + 16);
    rsret_.resize(2 * (size_t)RSDims_ + 16);
}

void mp4Processor::addtoFrame(uint8_t *V, int16_t nbits) {        // mp4processor.cpp:107-145
    const int nbytes = nbits / 8;
    for (int i = 0; i < nbytes; i++) {
        uint8_t temp = 0;
        for (int j = 0; j < 8; j++) temp = (uint8_t)((temp << 1) | (V[i * 8 + j] & 1));
        frameBytes_[blockFillIndex_ * nbytes + i] = temp;
    }
    blocksInBuffer_++;
    blockFillIndex_ = (int16_t)((blockFillIndex_ + 1) % 5);
    if (blocksInBuffer_ >= 5) {
        if (fire_check(&frameBytes_[blockFillIndex_ * nbytes]) && processSuperframe(blockFillIndex_ * nbytes)) {
            blocksInBuffer_ = 0;
        } else {                                   // virtual shift left by one block
            blocksInBuffer_ = 4;
            frameErrors_++;
        }
    }
}

bool mp4Processor::processSuperframe(int base) {                 // mp4processor.cpp:146-292
    const int RS = RSDims_;
    std::vector<uint8_t> rsIn((size_t)RS * 120), rsOut((size_t)RS * 110);
    std::vector<int16_t> ret(RS);
    for (int j = 0; j < RS; j++)
        for (int k = 0; k < 120; k++) rsIn[(size_t)j * 120 + k] = frameBytes_[(base + j + k * RS) % (RS * 120)];
    rsin_.upload(rsIn.data(), rsIn.size());
    chk(dabgpu_rs_decode(thread_context(), (const uint8_t *)rsin_.get(), RS, (uint8_t *)rsout_.get(),
                         (int16_t *)rsret_.get()), "dabgpu_rs_decode");
    rsout_.download(rsOut.data(), rsOut.size());
    rsret_.download(ret.data(), sizeof(int16_t) * RS);
    int16_t nErrors = 0;
    for (int j = 0; j < RS; j++) {                 // the reference stops at the first failing column
        if (ret[j] > 0) nErrors = (int16_t)(nErrors + ret[j]);
        if (ret[j] < 0) return false;
        for (int k = 0; k < 110; k++) outVector_[j + k * RS] = rsOut[(size_t)j * 110 + k];
    }
    const uint8_t *o = outVector_.data();
    au_info info;
    info.dacRate = (o[2] >> 6) & 1;
    info.sbrFlag = (o[2] >> 5) & 1;
    info.aacChannelMode = (o[2] >> 4) & 1;
    info.mpegSurround = o[2] & 7;
    info.n_corrected = nErrors;
    int num_aus, a[7];
    const int end = 110 * RS;
    switch (2 * info.dacRate + info.sbrFlag) {
    default:
    case 0: num_aus = 4; a[0] = 8; a[1] = o[3] * 16 + (o[4] >> 4); a[2] = (o[4] & 0xf) * 256 + o[5];
            a[3] = o[6] * 16 + (o[7] >> 4); a[4] = end; break;
    case 1: num_aus = 2; a[0] = 5; a[1] = o[3] * 16 + (o[4] >> 4); a[2] = end; break;
    case 2: num_aus = 6; a[0] = 11; a[1] = o[3] * 16 + (o[4] >> 4); a[2] = (o[4] & 0xf) * 256 + o[5];
            a[3] = o[6] * 16 + (o[7] >> 4); a[4] = (o[7] & 0xf) * 256 + o[8]; a[5] = o[9] * 16 + (o[10] >> 4);
            a[6] = end; break;
    case 3: num_aus = 3; a[0] = 6; a[1] = o[3] * 16 + (o[4] >> 4); a[2] = (o[4] & 0xf) * 256 + o[5]; a[3] = end; break;
    }
    for (int i = 0; i < num_aus; i++) {
        if (a[i + 1] < a[i]) return false;
        const int len = a[i + 1] - a[i] - 2;
        if (len >= 960 || len < 0) return false;
        const bool ok = dabPlus_crc(&outVector_[a[i]], (int16_t)len);
        if (cb_) cb_(&outVector_[a[i]], (int16_t)len, ok, info);
    }
    superframes_++;
    return true;
}

// ---- dabConcurrent / mscDatagroup ---------------------------------------------------
dabConcurrent::dabConcurrent(uint8_t dabModus, int16_t fragmentSize, int16_t bitRate, int16_t uepFlag,
                             int16_t protLevel, std::unique_ptr<dabProcessor> processor)
    : dabModus_(dabModus), fragmentSize_(fragmentSize), bitRate_(bitRate), delay_((size_t)16 * fragmentSize, 0),
      data_(fragmentSize), outV_((size_t)24 * bitRate), proc_(std::move(processor)) {
    sub_ = dabgpu_subch{0, (int16_t)(fragmentSize / 64), bitRate, protLevel, uepFlag, 0};
    int32_t nb, fr, ns, L[4], PI[4];
    chk(dabgpu_subch_profile(&sub_, &nb, &fr, &ns, L, PI) < 0 ? DABGPU_E_UNSUP : DABGPU_OK,
        "dabConcurrent: protection undefined");
    if (fr > fragmentSize) throw error(DABGPU_E_ARG, "dabConcurrent: fragment shorter than the profile consumes");
    in_.resize(sizeof(int16_t) * fragmentSize);
    out_.resize(outV_.size() + 16);
}

bool dabConcurrent::deinterleave(const int16_t *v) {              // dab-concurrent.cpp:162-175
    // out_n[i] = in_{n - d(i)}[i]: the last 16 fragments in a ring, zeros before the first
    std::memcpy(&delay_[(size_t)(cif_ & 15) * fragmentSize_], v, sizeof(int16_t) * fragmentSize_);
    for (int i = 0; i < fragmentSize_; i++) {
        const int d = interleave_delay(i);
        data_[i] = cif_ - d >= 0 ? delay_[(size_t)((cif_ - d) & 15) * fragmentSize_ + i] : 0;
    }
    cif_++;
    if (countforInterleaver_ <= 15) {              // only continue when the de-interleaver is filled
        countforInterleaver_++;
        return false;
    }
    // uep_/eep_deconvolve + the inline energy dispersal (:177-190) on the GPU
    in_.upload(data_.data(), sizeof(int16_t) * fragmentSize_);
    chk(dabgpu_msc_deconvolve(thread_context(), (const int16_t *)in_.get(), fragmentSize_, &sub_, 1,
                              (uint8_t *)out_.get(), (int64_t)outV_.size()),
        "dabgpu_msc_deconvolve");
    out_.download(outV_.data(), outV_.size());
    return true;
}

int32_t dabConcurrent::process(int16_t *v, int16_t cnt) {
    if (cnt != fragmentSize_) throw error(DABGPU_E_ARG, "dabConcurrent::process: fragment size");
    if (deinterleave(v) && proc_) proc_->addtoFrame(outV_.data(), (int16_t)(24 * bitRate_));
    return cnt;
}

void dabConcurrent::setFiles(FILE *mp2, FILE *mp4) {                // dab-concurrent.cpp:196-200
    (void)mp4;
    if (dabModus_ == DAB && proc_) proc_->setFile(mp2);
}

mscDatagroup::mscDatagroup(uint8_t DSCTy, int16_t packetAddress, int16_t fragmentSize, int16_t bitRate,
                           int16_t uepFlag, int16_t protLevel, uint8_t DGflag, int16_t FEC_scheme,
                           packetAssembler::datagroup_cb cb)
    : dabConcurrent(DAB, fragmentSize, bitRate, uepFlag, protLevel, nullptr), pa_(DSCTy, DGflag, std::move(cb)) {
    (void)packetAddress;                           // the reference follows the first address it sees
    (void)FEC_scheme;
}

int32_t mscDatagroup::process(int16_t *v, int16_t cnt) {          // msc-datagroup.cpp:149-206
    if (cnt != fragmentSize_) throw error(DABGPU_E_ARG, "mscDatagroup::process: fragment size");
    if (deinterleave(v)) pa_.add(outV_.data(), (int16_t)(24 * bitRate_));
    return cnt;
}

// ---- mscHandler -------------------------------------------------------------------
mscHandler::mscHandler(DabParams *p, outputs out, uint8_t concurrent)
    : out_(std::move(out)), BitsperBlock_((int16_t)(2 * p->K)), cifVector_(55296, 0), dabHandler_(new dabVirtual) {
    (void)concurrent;                              // the reference always builds dabConcurrent (msc-handler.cpp:143)
    numberofblocksperCIF_ = p->dabMode == 4 ? 36 : p->dabMode == 2 ? 72 : 18;
    if (p->dabMode != 1) throw error(DABGPU_E_UNSUP, "mscHandler: Mode I only");
}

void mscHandler::set_audioChannel(audiodata *d) {                 // msc-handler.cpp:91-105
    std::lock_guard<std::mutex> g(locker_);
    audioService_ = true;
    na_ = *d;
    new_language_ = d->language;
    new_type_ = d->programType;
    newChannel_ = true;
}

void mscHandler::set_dataChannel(packetdata *d) {                 // msc-handler.cpp:107-121
    std::lock_guard<std::mutex> g(locker_);
    audioService_ = false;
    np_ = *d;
    newChannel_ = true;
}

void mscHandler::process_mscBlock(int16_t *fbits, int16_t blkno) { // msc-handler.cpp:125-193
    if (!work_to_be_done_ && !newChannel_) return;
    const int16_t currentblk = (int16_t)((blkno - 4) % numberofblocksperCIF_);
    if (newChannel_) {
        std::lock_guard<std::mutex> g(locker_);
        newChannel_ = false;
        dabHandler_->stopRunning();
        if (audioService_) {
            const uint8_t modus = na_.ASCTy == 077 ? DAB_PLUS : DAB;
            std::unique_ptr<dabProcessor> proc;
            if (modus == DAB_PLUS) proc.reset(new mp4Processor(na_.bitRate, out_.aac));
            else proc.reset(new mp2Processor(na_.bitRate, out_.mp2, mp2File_));   // msc-handler.cpp:147-150
            dabHandler_.reset(new dabConcurrent(modus, (int16_t)(na_.length * 64), na_.bitRate, na_.uepFlag,
                                                na_.protLevel, std::move(proc)));
            startAddr_ = na_.startAddr;
            Length_ = na_.length;
        } else {
            dabHandler_.reset(new mscDatagroup((uint8_t)np_.DSCTy, np_.packetAddress, (int16_t)(np_.length * 64),
                                               np_.bitRate, np_.uepFlag, np_.protLevel, (uint8_t)np_.DGflag,
                                               np_.FEC_scheme, out_.datagroup));
            startAddr_ = np_.startAddr;
            Length_ = np_.length;
        }
        work_to_be_done_ = true;
    }
    std::memcpy(&cifVector_[(size_t)currentblk * BitsperBlock_], fbits, sizeof(int16_t) * BitsperBlock_);
    if (currentblk < numberofblocksperCIF_ - 1) return;
    // a full CIF: the selected subchannel's slice
    (void)dabHandler_->process(&cifVector_[(size_t)startAddr_ * 64], (int16_t)(Length_ * 64));
}

int16_t mscHandler::getLanguage() { return new_language_; }
int16_t mscHandler::getType() { return new_type_; }
void mscHandler::stop() {
    work_to_be_done_ = false;
    dabHandler_->stop();
}
void mscHandler::stopProcessing() { work_to_be_done_ = false; }
void mscHandler::setFiles(FILE *mp2, FILE *mp4) {                  // msc-handler.cpp:208-212
    std::lock_guard<std::mutex> g(locker_);
    mp2File_ = mp2;
    mp4File_ = mp4;
    dabHandler_->setFiles(mp2, mp4);
}

}  // namespace dabgpu
