// TEST INFRASTRUCTURE: FIG parser (sdr-j-dab_amd/host/fib_processor.*) on FIBs built
// here field by field after ETSI EN 300 401 (FIG 0/1, 0/2, 0/3, 0/14, 0/17, 1/0,
// 1/1, 1/5), as the reference's fib_processor reads them.  The expected service
// records follow from the fields written; the reference class itself needs Qt and
// cannot be built here, so this parity is unpinned.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dabsynth.h"
#include "fib_processor.h"

using namespace dabgpu;

static int failures = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            failures++;                                                       \
        }                                                                     \
    } while (0)

// one FIB: FIGs appended as bytes, then end marker 0xFF up to 30 bytes, then a
// 16-bit CRC field (not checked by process_FIB); returned as 256 bits, one per byte
struct Fib {
    std::vector<uint8_t> bytes;
    void fig(int type, const std::vector<uint8_t> &field) {
        bytes.push_back((uint8_t)((type << 5) | (int)field.size()));
        bytes.insert(bytes.end(), field.begin(), field.end());
    }
    std::vector<uint8_t> bits() const {
        std::vector<uint8_t> b8(bytes);
        if (b8.size() > 30) std::fprintf(stderr, "FIB overflow %zu\n", b8.size()), failures++;
        b8.resize(30, 0xFF);
        b8.push_back(0);
        b8.push_back(0);
        std::vector<uint8_t> out(256);
        for (int i = 0; i < 256; i++) out[i] = (b8[i >> 3] >> (7 - (i & 7))) & 1;
        return out;
    }
};

// MSB-first field writer
struct Fields {
    std::vector<uint8_t> bits;
    Fields &put(uint32_t v, int n) {
        for (int i = n - 1; i >= 0; i--) bits.push_back((v >> i) & 1);
        return *this;
    }
    std::vector<uint8_t> bytes() const {
        std::vector<uint8_t> b((bits.size() + 7) / 8, 0);
        for (size_t i = 0; i < bits.size(); i++) b[i >> 3] |= bits[i] << (7 - (i & 7));
        return b;
    }
};

static Fields fig0_head(int ext, int pd = 0) { return Fields().put(0, 1).put(0, 1).put(pd, 1).put(ext, 5); }
static Fields label(Fields f, const char *l16) {
    for (int i = 0; i < 16; i++) f.put((uint8_t)l16[i], 8);
    return f.put(0xFF00, 16);                                   // character flag field
}

int main() {
    fib_processor fp;
    std::string ens_seen;
    std::vector<std::string> svc_seen;
    fp.on_ensemble([&](uint32_t eid, const std::string &n) { ens_seen = n; CHECK(eid == 0xE123); });
    fp.on_service([&](const std::string &n) { svc_seen.push_back(n); });
    std::vector<std::vector<uint8_t>> fibs;

    {   // FIG 1/0 ensemble label + FIG 0/14 (FEC 1 for sub-channel id 0)
        Fib f;
        f.fig(1, label(Fields().put(0, 4).put(0, 1).put(0, 3).put(0xE123, 16), "TEST ENSEMBLE   ").bytes());
        // two entries: the reference's loop (used < Length) stops before the last one
        f.fig(0, fig0_head(14).put(0, 6).put(1, 2).put(7, 6).put(2, 2).bytes());
        fibs.push_back(f.bits());
    }
    {   // FIG 0/1: id 3 short form (table index 35: 96 CUs, level 3, 128 kbit/s) at CU 104;
        // id 5 EEP-A level 3, 48 CUs at 200; id 6 EEP-B level 1, 54 CUs at 300
        // FIG 0/2: service 0xA001 audio (ASCTy 63) on sub-channel 5, 0xA002 audio on 3
        Fib f;
        f.fig(0, fig0_head(1)
                     .put(3, 6).put(104, 10).put(0, 1).put(0, 1).put(35, 6)
                     .put(5, 6).put(200, 10).put(1, 1).put(0, 3).put(2, 2).put(48, 10)
                     .put(6, 6).put(300, 10).put(1, 1).put(1, 3).put(0, 2).put(54, 10)
                     .bytes());
        f.fig(0, fig0_head(2)
                     .put(0xA001, 16).put(0, 1).put(0, 3).put(1, 4).put(0, 2).put(63, 6).put(5, 6).put(1, 1).put(0, 1)
                     .put(0xA002, 16).put(0, 1).put(0, 3).put(1, 4).put(0, 2).put(0, 6).put(3, 6).put(1, 1).put(0, 1)
                     .bytes());
        fibs.push_back(f.bits());
    }
    {   // FIG 0/2: packet service 0xA003 (SCId 0x123); FIG 0/3: SCId 0x123 on
        // sub-channel 6, DSCTy 5, packet address 1000, DG 1 (7-byte entry as the
        // reference steps); FIG 0/17: 0xA001 language 9, programme type 10
        Fib f;
        f.fig(0, fig0_head(2).put(0xA003, 16).put(0, 1).put(0, 3).put(1, 4).put(3, 2).put(0x123, 12).put(1, 1).put(0, 1)
                     .bytes());
        f.fig(0, fig0_head(3).put(0x123, 12).put(0, 3).put(1, 1).put(1, 1).put(0, 1).put(5, 6).put(6, 6).put(1000, 10)
                     .put(0xBEEF, 16).bytes());
        f.fig(0, fig0_head(17).put(0xA001, 16).put(0, 1).put(0, 1).put(1, 1).put(0, 1).put(0, 4).put(9, 8).put(0, 3)
                     .put(10, 5).bytes());
        fibs.push_back(f.bits());
    }
    const char labB[17] = {'S', 'T', 'R', 'A', (char)0x8D, 'E', ' ', (char)0x24, ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ', 0};
    for (auto [sid, lab] : std::vector<std::pair<int, const char *>>{{0xA001, "RADIO ONE       "}, {0xA002, labB},
                                                                       {0xA003, "DATA ONE        "}}) {
        Fib f;                                                    // FIG 1/1 service labels
        f.fig(1, label(Fields().put(0, 4).put(0, 1).put(1, 3).put(sid, 16), lab).bytes());
        fibs.push_back(f.bits());
    }
    {   // FIG 1/5: data service label with a 32-bit SId (no components)
        Fib f;
        f.fig(1, label(Fields().put(0, 4).put(0, 1).put(5, 3).put(0xE0A00004u, 32), "EPG             ").bytes());
        fibs.push_back(f.bits());
    }
    {   // a second FIG 1/1 for 0xA001 (the first name stays) and a repeated FIG 0/2
        Fib f;
        f.fig(1, label(Fields().put(0, 4).put(0, 1).put(1, 3).put(0xA001, 16), "OTHER NAME      ").bytes());
        fibs.push_back(f.bits());
    }
    for (auto &b : fibs) fp.process_FIB(b.data(), 0);
    for (auto &b : fibs) fp.process_FIB(b.data(), 0);          // repeated FIGs change nothing

    CHECK(fp.ensembleName() == "TEST ENSEMBLE   ");
    CHECK(ens_seen == "TEST ENSEMBLE   ");
    const std::string nameB = "STRA\xC3\x9F" "E \xC2\xA4        ";    // 0x8D -> U+00DF, 0x24 -> U+00A4
    CHECK(svc_seen.size() == 3);
    CHECK(fp.kindofService("RADIO ONE       ") == AUDIO_SERVICE);
    CHECK(fp.kindofService(nameB) == AUDIO_SERVICE);
    CHECK(fp.kindofService("DATA ONE        ") == PACKET_SERVICE);
    CHECK(fp.kindofService("EPG              (data)") == UNKNOWN_SERVICE);   // label known, no component
    CHECK(fp.kindofService("OTHER NAME      ") == UNKNOWN_SERVICE);
    CHECK(fp.kindofService("NOBODY") == UNKNOWN_SERVICE);

    audiodata a;
    std::memset(&a, 0, sizeof a);
    CHECK(fp.dataforAudioService("RADIO ONE       ", &a));
    CHECK(a.subchId == 5 && a.startAddr == 200 && a.uepFlag == 1 && a.protLevel == 0103 && a.length == 48);
    CHECK(a.bitRate == 64 && a.ASCTy == 63 && a.language == 9 && a.programType == 10);
    std::memset(&a, 0, sizeof a);
    CHECK(fp.dataforAudioService(nameB, &a));
    CHECK(a.subchId == 3 && a.startAddr == 104 && a.uepFlag == 0 && a.protLevel == 3 && a.length == 96);
    CHECK(a.bitRate == 128 && a.ASCTy == 0 && a.language == 0 && a.programType == 0);
    CHECK(!fp.dataforAudioService("DATA ONE        ", &a));      // a packet service

    packetdata p;
    std::memset(&p, 0, sizeof p);
    CHECK(fp.dataforDataService("DATA ONE        ", &p));
    CHECK(p.subchId == 6 && p.startAddr == 300 && p.uepFlag == 1 && p.protLevel == 0201 && p.length == 54);
    CHECK(p.bitRate == 64 && p.DSCTy == 5 && p.DGflag == 1 && p.packetAddress == 1000);
    CHECK(p.FEC_scheme == 1);                                   // FIG 0/14 quirk: id 0 matches every entry
    CHECK(!fp.dataforDataService("RADIO ONE       ", &p));

    // EEP-A/B bit-rate formulas of fib-processor.cpp:318-347 for every level
    {
        fib_processor q;
        const int sizes[8] = {72, 48, 36, 24, 81, 63, 54, 45};   // 48 kbit/s at A1..A4, B1..B4 (B: 96 kbit/s)
        for (int h = 0; h < 2; h++) {                             // 4 long-form entries per FIB
            Fib f;
            Fields fl = fig0_head(1);
            for (int k = 4 * h; k < 4 * h + 4; k++)
                fl.put(10 + k, 6).put(100 * k, 10).put(1, 1).put(k / 4, 3).put(k % 4, 2).put(sizes[k], 10);
            f.fig(0, fl.bytes());
            auto b = f.bits();
            q.process_FIB(b.data(), 0);
        }
        for (int k = 0; k < 8; k++) {
            Fib g;
            g.fig(0, fig0_head(2).put(0xB000 + k, 16).put(0, 1).put(0, 3).put(1, 4).put(0, 2).put(0, 6).put(10 + k, 6)
                         .put(0, 1).put(0, 1).bytes());
            char lab[17];
            std::snprintf(lab, sizeof lab, "SERVICE %-8d", k);
            g.fig(1, label(Fields().put(0, 4).put(0, 1).put(1, 3).put(0xB000 + k, 16), lab).bytes());
            auto gb = g.bits();
            q.process_FIB(gb.data(), 0);
            audiodata x;
            CHECK(q.dataforAudioService(lab, &x));
            CHECK(x.bitRate == (k < 4 ? 48 : 96) && x.protLevel == (k < 4 ? 0100 : 0200) + k % 4 + 1);
        }
    }

    // the synthetic transmitter's FIGs (dabsynth_cfg.figs): the FIBs it sends describe
    // its subchannels; parsed back they give the decoder configuration
    {
        dabsynth_subch sc[4] = {{0, 96, 128, 3, 1, 0}, {96, 48, 64, 0103, 0, 1}, {144, 54, 64, 0201, 0, 0},
                                {198, 35, 48, 3, 1, 0}};
        dabsynth_cfg cfg;
        std::memset(&cfg, 0, sizeof cfg);
        cfg.n_frames = 2;
        cfg.pre_offset = 1000;
        cfg.snr_db = 300.0f;
        cfg.amplitude = 1.0f;
        cfg.n_subch = 4;
        cfg.subch = sc;
        cfg.figs = 1;
        std::vector<float> iq(2 * dabsynth_stream_len(&cfg));
        std::vector<uint8_t> fic((size_t)cfg.n_frames * 4 * 768);
        CHECK(dabsynth_generate(&cfg, 7, iq.data(), fic.data(), nullptr, nullptr, nullptr) == 0);
        fib_processor q;
        for (size_t k = 0; k < fic.size() / 256; k++) q.process_FIB(&fic[256 * k], 0);
        CHECK(q.ensembleName() == "SYNTH ENSEMBLE  ");
        for (int i = 0; i < 4; i++) {
            char lab[17];
            std::snprintf(lab, sizeof lab, "SERVICE %02d      ", i);
            audiodata x;
            CHECK(q.kindofService(lab) == AUDIO_SERVICE);
            CHECK(q.dataforAudioService(lab, &x));
            CHECK(x.subchId == i && x.startAddr == sc[i].startAddr && x.length == sc[i].length);
            CHECK(x.bitRate == sc[i].bitRate && x.protLevel == sc[i].protLevel && x.uepFlag == (sc[i].uep ? 0 : 1));
            CHECK(x.ASCTy == (sc[i].dabplus ? 63 : 0));
        }
    }

    fp.clearEnsemble();
    CHECK(fp.kindofService("RADIO ONE       ") == UNKNOWN_SERVICE);
    CHECK(fp.serviceLabels().empty() && fp.ensembleName().empty());

    if (failures) {
        std::fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    std::printf("fib_processor: all checks passed\n");
    return 0;
}
