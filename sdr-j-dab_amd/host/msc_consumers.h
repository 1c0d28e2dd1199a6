// msc_consumers.h -- what the reference does with the decoded MSC bits of a
// subchannel, minus the codecs: the plug-in interfaces (dabVirtual, dabProcessor),
// the MPEG-1/2 layer II frame synchroniser of mp2Processor (mp2processor.cpp:572-629)
// and the packet-mode data-group assembly of mscDatagroup (msc-datagroup.cpp:221-339).
// Host code (a few bit operations per decoded bit, after the GPU's Viterbi): no Qt,
// no kjmp2 / faad / MOT / IP handlers -- complete frames and data groups go to
// callbacks instead.  Same state machines and quirks as the reference.
#pragma once
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <vector>

namespace dabgpu {

// dabProcessor (includes/backend/audio/dab-processor.h): addtoFrame(bits, nbits),
// one bit per byte as the deconvolver delivers them
class dabProcessor {
public:
    virtual ~dabProcessor() = default;
    virtual void addtoFrame(uint8_t *v, int16_t nbits) { (void)v; (void)nbits; }
    // mp2Processor::setFile (mp2processor.cpp:631-633); the other processors ignore it
    virtual void setFile(FILE *f) { (void)f; }
};

// dabVirtual (includes/backend/dab-virtual.h:36-47): a subchannel's CIF fragments
class dabVirtual {
public:
    virtual ~dabVirtual() = default;
    virtual int32_t process(int16_t *v, int16_t cnt) { (void)v; (void)cnt; return 0; }
    virtual void stopRunning() {}
    virtual void stop() {}
    // dab-virtual.h:43: the mp2 / mp4 dump files (dabConcurrent hands the mp2 file to an
    // mp2Processor, dab-concurrent.cpp:196-200; the mp4 file is never written in v0.997)
    virtual void setFiles(FILE *mp2, FILE *mp4) { (void)mp2; (void)mp4; }
};

// check_CRC_bits (dab-constants.h:310-340): CRC-16 over size bits (1 per byte) whose
// last 16 are the inverted CRC; inverts those 16 bits in place, as the reference does
bool check_CRC_bits(uint8_t *in, int16_t size);

// mp2Processor::addtoFrame (mp2processor.cpp:572-629): sync on 12 consecutive 1 bits,
// read the 24-bit header (sample rate: 48 or 24 kHz, else unchanged), collect the frame
// (24 * bitRate bits at 48 kHz, twice that at 24 kHz) and hand it over -- where the
// reference writes it to the mp2 file or decodes it with kjmp2.  With a file set
// (setFile, mscHandler::setFiles) the frame is written INSTEAD of handed to the callback,
// exactly as mp2processor.cpp:581-586 writes instead of decoding -- including the
// reference's count: fwrite of lf BYTES where lf is the frame's length in bits, i.e.
// the frame's lf / 8 bytes followed by the rest of the (2 * 24 * bitRate byte) frame
// buffer, which the reference leaves uninitialised and this class zero-fills.
class mp2Processor : public dabProcessor {
public:
    using frame_cb = std::function<void(const uint8_t *frame, int32_t nbits, int32_t sampleRate)>;
    mp2Processor(int16_t bitRate, frame_cb cb, FILE *mp2file = nullptr);
    void addtoFrame(uint8_t *v, int16_t nbits) override;
    void setFile(FILE *f) override { mp2File_ = f; }
    int32_t sampleRate() const { return baudRate_; }
    int32_t frames() const { return frames_; }
private:
    void addbit(uint8_t b, int16_t nm);
    frame_cb cb_;
    std::atomic<FILE *> mp2File_{nullptr};   // setFile from the GUI thread, read by the decoding thread
    int32_t baudRate_ = 48000;
    int32_t MP2framesize_;                  // bits
    std::vector<uint8_t> MP2frame_;
    int16_t MP2Header_OK_ = 0, MP2headerCount_ = 0, MP2bitCount_ = 0;
    int32_t frames_ = 0;
};

// mscDatagroup's packet handling (msc-datagroup.cpp:221-339): the decoded bits of a CIF
// are a sequence of DAB packets (24, 48, 72 or 96 bytes); each is CRC-checked, padding
// packets (address 0) dropped, and the packets of the first address seen are assembled
// into MSC data groups by their first/last flags.  A data group (bits, one per byte) goes
// to the callback that stands in for the DSCTy's data handler (MOT, IP, journaline).
// DSCTy 5 with DGflag set: the transparent data channel of handleTDCAsyncstream, which
// only checks the first packet's CRC.
class packetAssembler {
public:
    using datagroup_cb = std::function<void(const std::vector<uint8_t> &bits)>;
    packetAssembler(uint8_t DSCTy, uint8_t DGflag, datagroup_cb cb);
    void add(uint8_t *data, int16_t length);           // one CIF's decoded bits (24 * bitRate)
    int32_t crcErrors() const { return crcErrors_; }
    int32_t packets() const { return handledPackets_; }
    int32_t datagroups() const { return datagroups_; }
private:
    void handlePacket(uint8_t *data, int avail);
    uint8_t DSCTy_, DGflag_;
    datagroup_cb cb_;
    int16_t packetState_ = 0;
    int32_t streamAddress_ = -1;
    std::vector<uint8_t> series_;
    int32_t crcErrors_ = 0, handledPackets_ = 0, datagroups_ = 0;
};

}  // namespace dabgpu
