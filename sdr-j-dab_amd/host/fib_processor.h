// fib_processor.h -- the FIG parser and service database behind a functional
// drop-in ficHandler: fib_processor of sdr-j-dab
// (includes/backend/fib-processor.h, src/backend/fib-processor.cpp), without Qt.
//
// Host code, scalar and tiny: a FIB is 30 bytes of FIGs once a frame, nothing to
// put on a GPU.  It consumes the CRC-good FIBs the GPU FIC decoder delivers
// (ficHandler / ensembleDecoder::on_fib) and answers the service lookups that
// configure the MSC decoder (kindofService, dataforAudioService,
// dataforDataService).
//
// Parsed as the reference does (same bit positions, same tables, same quirks):
//   FIG 0/1  sub-channel organisation (short form via the UEP table, long form EEP
//            A/B with the reference's bit-rate formulas)          fib-processor.cpp:278-354
//   FIG 0/2  service organisation (audio TMid 0, packet TMid 3)    :356-422, 1077-1140
//   FIG 0/3  packet-mode service components                        :424-453
//   FIG 0/14 FEC scheme (the reference matches ficList[i].SubChId, which FIG 0/1
//            never sets: only sub-channel id 0 takes effect, for every entry)  :688-705
//   FIG 0/17 programme type and language                           :726-752
//   FIG 0/16 programme number: only its service-table side effect (a new entry per
//            unknown SId, which orders later lookups)              :707-724
//   FIG 1/0  ensemble label, FIG 1/1 service label, FIG 1/5 data service label
//            (" (data)" appended)                                  :850-997
//   FIG 2/5  data service label, as FIG 1/5 without the suffix     :998-1037
// clearEnsemble keeps a service entry's language and programme type, as the
// reference's does (:1149-1163): an entry reused for a new service without FIG 0/17
// reports the old values.
// Labels are converted from the EBU Latin repertoire (charsets.cpp) or taken as
// UTF-8 (charset 15) and returned as UTF-8 strings, 16 characters as transmitted
// (trailing spaces included: the reference compares the full label).
// The remaining FIG 0 extensions (0, 5, 6, 8, 9, 10, 13, 18, 19, 21, 22) carry
// nothing the service lookups read and are skipped.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace dabgpu {

// dab-constants.h:75-77
constexpr uint8_t UNKNOWN_SERVICE = 0100;
constexpr uint8_t AUDIO_SERVICE = 0101;
constexpr uint8_t PACKET_SERVICE = 0102;

// dab-constants.h:152-177
struct packetdata {
    int16_t subchId;
    int16_t startAddr;
    uint8_t uepFlag;
    int16_t protLevel;
    int16_t DSCTy;
    int16_t length;
    int16_t bitRate;
    int16_t FEC_scheme;
    int16_t DGflag;
    int16_t packetAddress;
};
struct audiodata {
    int16_t subchId;
    int16_t startAddr;
    uint8_t uepFlag;
    int16_t protLevel;
    int16_t length;
    int16_t bitRate;
    int16_t ASCTy;
    int16_t language;
    int16_t programType;
};

class fib_processor {
public:
    // stand-ins for the Qt signals nameofEnsemble / addtoEnsemble
    using ensemble_cb = std::function<void(uint32_t EId, const std::string &name)>;
    using service_cb = std::function<void(const std::string &label)>;
    fib_processor();
    void on_ensemble(ensemble_cb f) { ens_cb_ = std::move(f); }
    void on_service(service_cb f) { svc_cb_ = std::move(f); }

    // fib: 256 bits, one per byte (as ficHandler hands them over); fib number unused
    void process_FIB(const uint8_t *fib, uint16_t ficno);
    void setupforNewFrame();
    void clearEnsemble();
    uint8_t kindofService(const std::string &label);
    // false (and *d untouched) where the reference returns without filling it in
    bool dataforAudioService(const std::string &label, audiodata *d);
    bool dataforDataService(const std::string &label, packetdata *d);

    std::string ensembleName() const { return ensemble_; }
    std::vector<std::string> serviceLabels() const;

private:
    struct service {
        int32_t serviceId = -1;
        std::string label;
        bool hasName = false, inUse = false, hasLanguage = false;
        int16_t language = 0, programType = 0;
    };
    struct component {
        bool inUse = false;
        int8_t TMid = 0;
        int service = -1;                      // index into services_
        int16_t componentNr = 0, ASCTy = 0, PS_flag = 0, subchannelId = 0;
        uint16_t SCId = 0;
        uint8_t CAflag = 0;
        int16_t DSCTy = 0;
        int8_t DGflag = 0;
        int16_t packetAddress = 0;
    };
    struct subchannel {
        int32_t SubChId = 0, StartAddr = 0, Length = 0, uepFlag = 0, protLevel = 0, BitRate = 0;
        int16_t language = 0, FEC_scheme = 0;
    };
    void fig0(const uint8_t *d);
    void fig1(const uint8_t *d);
    int fig0_1(const uint8_t *d, int used);
    int fig0_2(const uint8_t *d, int used, int pd);
    int fig0_3(const uint8_t *d, int used);
    void fig0_14(const uint8_t *d);
    void fig0_16(const uint8_t *d);
    void fig0_17(const uint8_t *d);
    void fig2(const uint8_t *d);
    int find_service(int32_t sid);
    int find_packet_component(int16_t scid) const;
    int bind(int8_t TMid, int32_t sid, int16_t compnr);
    int lookup(const std::string &label) const;       // first named service with this label

    service services_[64];
    component components_[64];
    subchannel sub_[64];
    std::string ensemble_;
    bool firstTime_ = true;
    ensemble_cb ens_cb_;
    service_cb svc_cb_;
};

}  // namespace dabgpu
