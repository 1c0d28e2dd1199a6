// msc_consumers.cpp -- see msc_consumers.h.
#include "msc_consumers.h"

#include <algorithm>
#include <cstring>

namespace dabgpu {

bool check_CRC_bits(uint8_t *in, int16_t size) {
    // CRC-CCITT x^16 + x^12 + x^5 + 1 from all ones over the bits, the received CRC
    // field (last 16 bits) inverted first (dab-constants.h:310-340)
    for (int i = size - 16; i < size; i++) in[i] ^= 1;
    uint32_t reg = 0xFFFF;
    for (int i = 0; i < size; i++) {
        const uint32_t top = (reg >> 15) & 1u;
        reg = (reg << 1) & 0xFFFFu;
        if (top ^ (in[i] & 1u)) reg ^= 0x1021u;
    }
    return reg == 0;
}

// ---- mp2Processor ---------------------------------------------------------------
mp2Processor::mp2Processor(int16_t bitRate, frame_cb cb, FILE *mp2file)
    : cb_(std::move(cb)), mp2File_(mp2file), MP2framesize_(24 * bitRate), MP2frame_(2 * 24 * bitRate, 0) {}

void mp2Processor::addbit(uint8_t b, int16_t nm) {                  // mp2processor.cpp:619-629
    uint8_t byte = MP2frame_[nm / 8];
    const uint8_t bit = (uint8_t)(1u << (7 - (nm & 7)));
    byte = b ? (uint8_t)(byte | bit) : (uint8_t)(byte & ~bit);
    MP2frame_[nm / 8] = byte;
}

void mp2Processor::addtoFrame(uint8_t *v, int16_t amount) {         // mp2processor.cpp:572-617
    const int32_t lf = baudRate_ == 48000 ? MP2framesize_ : 2 * MP2framesize_;
    for (int i = 0; i < amount; i++) {
        if (MP2Header_OK_ == 2) {
            addbit(v[i], MP2bitCount_++);
            if (MP2bitCount_ >= lf) {
                frames_++;
                if (FILE *f = mp2File_.load())
                    (void)std::fwrite(MP2frame_.data(), sizeof(uint8_t), (size_t)lf, f);   // :581-582
                else if (cb_)
                    cb_(MP2frame_.data(), lf, baudRate_);
                MP2Header_OK_ = 0;
                MP2headerCount_ = 0;
                MP2bitCount_ = 0;
            }
        } else if (MP2Header_OK_ == 0) {                            // not in sync yet
            if (v[i] == 1) {
                if (++MP2headerCount_ == 12) {
                    MP2bitCount_ = 0;
                    for (int j = 0; j < 12; j++) addbit(1, MP2bitCount_++);
                    MP2Header_OK_ = 1;
                }
            } else {
                MP2headerCount_ = 0;
            }
        } else if (MP2Header_OK_ == 1) {
            addbit(v[i], MP2bitCount_++);
            if (MP2bitCount_ == 24) {
                // mp2sampleRate (mp2processor.cpp:276-285) + setSamplerate (:262-269)
                static const int32_t rates[8] = {44100, 48000, 32000, 0, 22050, 24000, 16000, 0};
                const uint8_t *f = MP2frame_.data();
                int32_t rate = 0;
                if (f[0] == 0xFF && (f[1] & 0xF6) == 0xF4 && (int)f[2] - 0x10 < 0xE0)
                    rate = rates[(((f[1] & 0x08) >> 1) ^ 4) + ((f[2] >> 2) & 3)];
                if (rate == 48000 || rate == 24000) baudRate_ = rate;
                MP2Header_OK_ = 2;
            }
        }
    }
}

// ---- packet-mode data groups ----------------------------------------------------
static inline uint16_t bits_n(const uint8_t *d, int off, int n) {     // getBits (dab-constants.h:182-190)
    uint16_t r = 0;
    for (int i = 0; i < n; i++) r = (uint16_t)((r << 1) | d[off + i]);
    return r;
}

packetAssembler::packetAssembler(uint8_t DSCTy, uint8_t DGflag, datagroup_cb cb)
    : DSCTy_(DSCTy), DGflag_(DGflag), cb_(std::move(cb)) {}

void packetAssembler::add(uint8_t *data, int16_t length) {
    if (DSCTy_ == 5 && DGflag_) {                                      // handleTDCAsyncstream (:321-339)
        const int16_t packetLength = (int16_t)((bits_n(data, 0, 2) + 1) * 24);
        (void)check_CRC_bits(data, (int16_t)(packetLength * 8));
        return;
    }
    while (true) {                                                     // handlePackets (:221-234)
        const int16_t pLength = (int16_t)((bits_n(data, 0, 2) + 1) * 24 * 8);
        if (length < pLength) return;
        handlePacket(data, length);
        length = (int16_t)(length - pLength);
        if (length < 2) return;
        data = &data[pLength];
    }
}

// avail: bits of the CIF from this packet on.  The reference copies 8 * usefulLength
// bits from bit 24 whatever the packet length (msc-datagroup.cpp:276-283): a CRC-good
// packet whose useful length exceeds it reads on into the next packets, and past the
// CIF's buffer at its end -- here the copy stops at the buffer's end (defined behaviour;
// the same bits wherever the reference's read is defined).
void packetAssembler::handlePacket(uint8_t *data, int avail) {          // msc-datagroup.cpp:241-319
    const int16_t packetLength = (int16_t)((bits_n(data, 0, 2) + 1) * 24);
    const int16_t firstLast = (int16_t)bits_n(data, 4, 2);
    const int16_t address = (int16_t)bits_n(data, 6, 10);
    const int16_t usefulLength = (int16_t)bits_n(data, 17, 7);
    handledPackets_++;
    if (!check_CRC_bits(data, (int16_t)(packetLength * 8))) {
        crcErrors_++;
        return;
    }
    if (address == 0) return;                                          // padding packet
    if (streamAddress_ == -1) streamAddress_ = address;                // the first stream only
    if (streamAddress_ != address) return;
    auto take = [&](bool append) {
        const size_t cur = append ? series_.size() : 0;
        const int n = std::max(0, std::min(8 * (int)usefulLength, avail - 24));
        series_.resize(cur + (size_t)n);
        for (int i = 0; i < n; i++) series_[cur + i] = data[24 + i];
    };
    auto deliver = [&]() {
        datagroups_++;
        if (cb_) cb_(series_);
    };
    if (packetState_ == 0) {                                           // waiting for a start
        if (firstLast == 2) {
            packetState_ = 1;
            take(false);
        } else if (firstLast == 3) {                                   // single packet
            take(false);
            deliver();
        } else {
            series_.resize(0);
        }
    } else {                                                           // within a series
        if (firstLast == 0) {
            take(true);
        } else if (firstLast == 1) {
            take(true);
            deliver();
            packetState_ = 0;
        } else if (firstLast == 2) {                                   // new first: previous lost
            packetState_ = 1;
            take(false);
        } else {
            packetState_ = 0;
            series_.resize(0);
        }
    }
}

}  // namespace dabgpu
