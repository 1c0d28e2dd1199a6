// TEST INFRASTRUCTURE: the drop-in classes driven the way sdr-j-dab's Qt GUI drives
// the reference's (gui.cpp), on the GPU.  The call sequence replayed:
//   setStart (gui.cpp:400-470)   ficHandler + mscHandler, then ofdmProcessor (thread)
//   nameofEnsemble / addtoEnsemble signals (fib-processor.cpp via ficHandler)
//   selectService (:795-840)     kindofService -> dataforAudioService -> set_audioChannel,
//                                getLanguage / getType;  dataforDataService ->
//                                (DSCTy, bitRate checked) -> set_dataChannel
//   set_mp2File (:898-926)       mscHandler::setFiles(mp2File, mp4File) / (NULL, ...)
//   TerminateProcess (:300-340)  setFiles(NULL, NULL), fclose, mscHandler::stop,
//                                ficHandler::stop, ofdmProcessor::stop
//   reset (:500-512)             ficHandler::clearEnsemble
// on a synthetic ensemble that announces itself in its FIC (FIG 0/1, 0/2, 0/3, 1/0,
// 1/1): an MPEG layer II service, a DAB+ service and a packet-mode data service.
//
// Part A replays the sequence with the services selected mid-stream and checks the
// outcome against the transmitter's truth (every MP2 frame dumped is a transmitted
// frame, every data group a transmitted one).  Part B decodes the whole stream with
// the MP2 and the packet service selected before the first frame and writes what the
// consumers produced to <outdir> (mp2.bin: the mp2 file; datagroups.bin: uint32 bit
// count + bits per group), which tests/test_gpu_dropin.py compares with the oracle's
// restatements (oracle_py.MP2 / Datagroups) run on the oracle's MSC bits of the
// same IQ.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "dabgpu_dropin.h"
#include "dabsynth.h"

static int failures = 0;
#define CHECK(c, ...)                                      \
    do {                                                   \
        if (!(c)) {                                        \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                      \
            std::printf("\n");                             \
            failures++;                                    \
        }                                                  \
    } while (0)

// gui.cpp's virtualInput: a recording handed over in pieces, as a device delivers them
struct MemInput : dabgpu::virtualInput {
    const float *iq;
    int64_t n, pos = 0;
    std::mutex m;
    int32_t getSamples(dabgpu::DSPCOMPLEX *v, int32_t k) override {
        std::lock_guard<std::mutex> g(m);
        k = (int32_t)std::min<int64_t>(k, n - pos);
        std::memcpy((void *)v, iq + 2 * pos, sizeof(float) * 2 * k);
        pos += k;
        return k;
    }
    int32_t Samples() override {
        std::lock_guard<std::mutex> g(m);
        return (int32_t)std::min<int64_t>(40000, n - pos);
    }
};

// the ensemble (tests/test_gpu_dropin.py builds the same one: keep in sync)
static const int NF = 28;
static dabsynth_subch SC[3] = {{0, 96, 128, 0103, 0, 0, DABSYNTH_MP2},
                               {96, 48, 64, 0103, 0, 1, 0},
                               {144, 24, 32, 0103, 0, 0, DABSYNTH_PACKET}};

static std::vector<uint8_t> pack(const uint8_t *bits, int n) {
    std::vector<uint8_t> b((size_t)n / 8, 0);
    for (int i = 0; i < n; i++) b[i / 8] |= (uint8_t)((bits[i] & 1) << (7 - (i & 7)));
    return b;
}

static bool wait_for(const std::function<bool()> &f, int seconds) {
    auto t0 = std::chrono::steady_clock::now();
    while (!f()) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(seconds)) return false;
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    return true;
}

int main(int argc, char **argv) {
    const std::string outdir = argc > 1 ? argv[1] : "/tmp";
    dabsynth_cfg cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.n_frames = NF;
    cfg.pre_offset = 50000;
    cfg.snr_db = 25.0f;
    cfg.cfo_hz = 50.0f;
    cfg.amplitude = 1.0f;
    cfg.n_subch = 3;
    cfg.subch = SC;
    cfg.figs = 1;
    const int64_t n = dabsynth_stream_len(&cfg);
    const int maxbits = 24 * 128, NC = 4 * NF;
    std::vector<float> iq(2 * n);
    std::vector<uint8_t> msc((size_t)NC * 3 * maxbits);
    int64_t f0 = 0;
    CHECK(dabsynth_generate(&cfg, 2024, iq.data(), nullptr, msc.data(), nullptr, &f0) == 0, "synth");
    // the transmitted MP2 frames and data groups (receiver CIFs 16.. carry them)
    std::set<std::vector<uint8_t>> tx_mp2, tx_dg;
    {
        dabgpu::packetAssembler pa(60, 0, [&](const std::vector<uint8_t> &g) { tx_dg.insert(g); });
        for (int c = 16; c < NC; c++) {
            tx_mp2.insert(pack(&msc[((size_t)c * 3 + 0) * maxbits], 24 * 128));
            std::vector<uint8_t> b(&msc[((size_t)c * 3 + 2) * maxbits], &msc[((size_t)c * 3 + 2) * maxbits] + 24 * 32);
            pa.add(b.data(), (int16_t)b.size());
        }
    }
    dabgpu::DabParams p;
    dabgpu::setModeParameters(&p, 1);

    // ---------------------------------------------------------------- part A
    {
        MemInput input;
        input.iq = iq.data();
        input.n = n;
        std::mutex mu;
        std::string ensembleName;
        std::vector<std::string> services;
        int crc_good = 0, crc_bad = 0;
        dabgpu::ficHandler::signals fs;
        fs.show_ficCRC = [&](bool ok) { std::lock_guard<std::mutex> g(mu); (ok ? crc_good : crc_bad)++; };
        fs.nameofEnsemble = [&](uint32_t, const std::string &name) { std::lock_guard<std::mutex> g(mu); ensembleName = name; };
        fs.addtoEnsemble = [&](const std::string &label) { std::lock_guard<std::mutex> g(mu); services.push_back(label); };
        dabgpu::ficHandler fic(fs, 2 * 1536);
        std::vector<std::vector<uint8_t>> groups;
        int aus = 0;
        dabgpu::mscHandler::outputs outs;
        outs.datagroup = [&](const std::vector<uint8_t> &g) { std::lock_guard<std::mutex> l(mu); groups.push_back(g); };
        outs.aac = [&](const uint8_t *, int16_t, bool ok, const dabgpu::mp4Processor::au_info &) { aus += ok; };
        dabgpu::mscHandler msch(&p, outs, 1);
        FILE *mp2File = std::tmpfile();
        dabgpu::ofdmProcessor::signals os;
        dabgpu::ofdmProcessor ofdm(&input, &p, os, &msch, &fic, 3, 1);
        // the services appear on the list as the FIC announces them
        CHECK(wait_for([&] { std::lock_guard<std::mutex> g(mu); return services.size() >= 3; }, 60),
              "addtoEnsemble: %zu services", services.size());
        {
            std::lock_guard<std::mutex> g(mu);
            CHECK(ensembleName == "SYNTH ENSEMBLE  ", "nameofEnsemble '%s'", ensembleName.c_str());
        }
        // selectService(SERVICE 00): MPEG layer II audio, its frames into the mp2 file
        std::string s0 = "SERVICE 00      ", s1 = "SERVICE 01      ", s2 = "SERVICE 02      ";
        CHECK(fic.kindofService(s0) == dabgpu::AUDIO_SERVICE, "kindofService audio");
        dabgpu::audiodata ad;
        std::memset(&ad, 0, sizeof ad);
        fic.dataforAudioService(s0, &ad);
        CHECK(ad.startAddr == 0 && ad.length == 96 && ad.bitRate == 128 && ad.protLevel == 0103 && ad.ASCTy == 0,
              "dataforAudioService %d %d %d %o %d", ad.startAddr, ad.length, ad.bitRate, ad.protLevel, ad.ASCTy);
        msch.setFiles(mp2File, nullptr);                    // set_mp2File
        msch.set_audioChannel(&ad);
        (void)msch.getLanguage();
        (void)msch.getType();
        CHECK(wait_for([&] { return ofdm.frames() >= 14; }, 60), "frames %lld", (long long)ofdm.frames());
        // SERVICE 01: DAB+ (ASCTy 077)
        CHECK(fic.kindofService(s1) == dabgpu::AUDIO_SERVICE, "kindofService DAB+");
        dabgpu::audiodata a1;
        fic.dataforAudioService(s1, &a1);
        CHECK(a1.ASCTy == 077 && a1.startAddr == 96 && a1.bitRate == 64, "DAB+ service %o %d", a1.ASCTy, a1.startAddr);
        // SERVICE 02: packet data (selectService checks DSCTy and bitRate first)
        CHECK(fic.kindofService(s2) == dabgpu::PACKET_SERVICE, "kindofService packet");
        dabgpu::packetdata pd;
        std::memset(&pd, 0, sizeof pd);
        fic.dataforDataService(s2, &pd);
        CHECK(pd.DSCTy == 60 && pd.bitRate == 32 && pd.startAddr == 144 && pd.length == 24 && pd.packetAddress == 0x102 &&
                  pd.DGflag == 0, "dataforDataService DSCTy %d bitRate %d start %d len %d addr %d", pd.DSCTy, pd.bitRate,
              pd.startAddr, pd.length, pd.packetAddress);
        msch.setFiles(nullptr, nullptr);                    // set_mp2File again: stop writing
        if (pd.DSCTy != 0 && pd.bitRate != 0) msch.set_dataChannel(&pd);
        CHECK(wait_for([&] { return ofdm.frames() >= NF; }, 60), "frames %lld", (long long)ofdm.frames());
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        // TerminateProcess
        msch.setFiles(nullptr, nullptr);
        msch.stop();
        fic.stop();
        ofdm.stop();
        // reset: the ensemble is forgotten
        fic.clearEnsemble();
        CHECK(fic.kindofService(s0) == dabgpu::UNKNOWN_SERVICE, "clearEnsemble");
        // the mp2 file: frames of lf bytes (mp2processor.cpp:581-582 writes the bit count
        // as a byte count), each a transmitted frame followed by zeros
        std::fflush(mp2File);
        const long sz = std::ftell(mp2File);
        std::rewind(mp2File);
        std::vector<uint8_t> file((size_t)std::max(sz, 0L));
        CHECK(std::fread(file.data(), 1, file.size(), mp2File) == file.size(), "read back");
        std::fclose(mp2File);
        const size_t lf = 24 * 128, fb = lf / 8;
        int mp2_frames = 0, mp2_bad = 0;
        for (size_t o = 0; o + lf <= file.size(); o += lf) {
            std::vector<uint8_t> fr(file.begin() + o, file.begin() + o + fb);
            mp2_frames++;
            mp2_bad += !tx_mp2.count(fr) || std::any_of(file.begin() + o + fb, file.begin() + o + lf, [](uint8_t b) { return b; });
        }
        CHECK(file.size() % lf == 0 && mp2_frames >= 8 && mp2_bad == 0, "mp2 file %zu bytes, %d frames, %d bad",
              file.size(), mp2_frames, mp2_bad);
        int dg_bad = 0;
        for (auto &g : groups) dg_bad += !tx_dg.count(g);
        CHECK(groups.size() >= 3 && dg_bad == 0, "data groups %zu, %d not transmitted", groups.size(), dg_bad);
        CHECK(crc_good > 0 && fic.get_ficRatio() > 50, "show_ficCRC %d good %d bad, ratio %d", crc_good, crc_bad,
              fic.get_ficRatio());
        std::printf("gui sequence: ok (%zu services, %d MP2 frames dumped, %zu data groups, FIC ratio %d%%)\n",
                    services.size(), mp2_frames, groups.size(), fic.get_ficRatio());
    }

    // ---------------------------------------------------------------- part B
    for (int kind = 0; kind < 2; kind++) {
        MemInput input;
        input.iq = iq.data();
        input.n = n;
        std::mutex mu;
        dabgpu::ficHandler fic(dabgpu::ficHandler::signals{}, 2 * 1536);
        std::vector<std::vector<uint8_t>> groups;
        dabgpu::mscHandler::outputs outs;
        outs.datagroup = [&](const std::vector<uint8_t> &g) { std::lock_guard<std::mutex> l(mu); groups.push_back(g); };
        dabgpu::mscHandler msch(&p, outs, 1);
        const std::string path = outdir + (kind == 0 ? "/mp2.bin" : "/datagroups.bin");
        FILE *f = std::fopen(path.c_str(), "wb");
        CHECK(f != nullptr, "open %s", path.c_str());
        if (!f) break;
        if (kind == 0) {
            dabgpu::audiodata ad{0, 0, 1, 0103, 96, 128, 0, 0, 0};
            msch.setFiles(f, nullptr);
            msch.set_audioChannel(&ad);
        } else {
            dabgpu::packetdata pd{2, 144, 1, 0103, 60, 24, 32, 0, 0, 0x102};
            msch.set_dataChannel(&pd);
        }
        int64_t frames = 0;
        // the GUI's display rings (gui.cpp:109,123) and their readers: showIQ takes `amount`
        // values (gui.cpp:1223-1229), showSpectrum the spectrum handler's block and flushes
        // (spectrum-handler.cpp:113-125; here the whole 32768 samples)
        dabgpu::RingBuffer<dabgpu::DSPCOMPLEX> iqBuffer(2 * 1536), spectrumBuffer(2 * 32768);
        std::vector<dabgpu::DSPCOMPLEX> iqv, specv;
        int n_iq = 0, n_spec = 0, iq_short = 0;
        dabgpu::ofdmProcessor::signals os;
        os.showIQ = [&](int amount) {
            std::vector<dabgpu::DSPCOMPLEX> Values(amount);
            const int t = iqBuffer.getDataFromBuffer(Values.data(), amount);
            iq_short += t != amount;
            iqv.insert(iqv.end(), Values.begin(), Values.begin() + t);
            n_iq++;
        };
        os.showSpectrum = [&](int amount) {
            if (spectrumBuffer.GetRingBufferReadAvailable() < amount) return;
            std::vector<dabgpu::DSPCOMPLEX> sp(amount);
            spectrumBuffer.getDataFromBuffer(sp.data(), amount);
            spectrumBuffer.FlushRingBuffer();
            specv.insert(specv.end(), sp.begin(), sp.end());
            n_spec++;
        };
        dabgpu::ofdmDecoder::iq_count = 0;          // a fresh GUI process: processToken's static cnt is 0
        // the packet pass also feeds an IQ ring and sets an out-of-range display token (ADVICE r5:
        // a token outside 1..75 turns the display feed off -- as in the reference, where it never
        // matches blkno -- and the decode goes on)
        dabgpu::RingBuffer<dabgpu::DSPCOMPLEX> iq2(2 * 1536);
        {
            dabgpu::ofdmProcessor ofdm(&input, &p, kind == 0 ? os : dabgpu::ofdmProcessor::signals{}, &msch, &fic, 3,
                                       kind == 0 ? &spectrumBuffer : nullptr, kind == 0 ? &iqBuffer : &iq2, 1);
            if (kind == 1) ofdm.set_displayToken(99);
            CHECK(wait_for([&] { return ofdm.frames() >= NF; }, 60), "part B frames %lld", (long long)ofdm.frames());
            std::this_thread::sleep_for(std::chrono::milliseconds(100));
            frames = ofdm.frames();
        }
        msch.setFiles(nullptr, nullptr);
        std::lock_guard<std::mutex> g(mu);
        for (auto &grp : groups) {
            const uint32_t nb = (uint32_t)grp.size();
            std::fwrite(&nb, 4, 1, f);
            std::fwrite(grp.data(), 1, grp.size(), f);
        }
        std::fclose(f);
        std::printf("part B %s: %lld frames, %zu data groups\n", kind == 0 ? "mp2" : "packet", (long long)frames,
                    groups.size());
        if (kind == 0) {
            // the display feeds, compared with the oracle's by tests/test_gpu_dropin.py
            CHECK(n_iq >= 2 && iq_short == 0, "showIQ %d times (%d short reads)", n_iq, iq_short);
            CHECK(n_spec >= 10, "showSpectrum %d times", n_spec);
            for (auto [name, v] : {std::make_pair("/iq_display.bin", &iqv), std::make_pair("/spectrum.bin", &specv)}) {
                FILE *o = std::fopen((outdir + name).c_str(), "wb");
                CHECK(o != nullptr, "open %s", name);
                if (o) {
                    std::fwrite(v->data(), sizeof(dabgpu::DSPCOMPLEX), v->size(), o);
                    std::fclose(o);
                }
            }
            std::printf("display feeds: showIQ %d x 1536 carriers, showSpectrum %d x 32768 samples\n", n_iq, n_spec);
        }
    }
    if (failures) {
        std::printf("GUI FAILED (%d)\n", failures);
        return 1;
    }
    std::printf("GUI OK\n");
    return 0;
}
