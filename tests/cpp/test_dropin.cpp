// TEST INFRASTRUCTURE: the C++ drop-in classes (sdr-j-dab_amd/host) on the GPU
// against the CPU oracle (oracle/liboracle.so) and the synthetic transmitter.
// Prints one line per check and "DROPIN OK" at the end; exit code 0 on success.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "dab_oracle.h"
#include "dabgpu_dropin.h"
#include "fib_processor.h"
#include "dabsynth.h"

static int failures = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                      \
            std::printf("\n");                             \
            failures++;                                    \
        }                                                  \
    } while (0)

static std::vector<int16_t> noisy_mother(std::mt19937 &rng, const std::vector<uint8_t> &bits, double sigma) {
    std::vector<uint8_t> coded(4 * (bits.size() + 6));
    dabsynth_conv_encode(bits.data(), (int)bits.size(), coded.data());
    std::normal_distribution<double> n(0.0, sigma);
    std::vector<int16_t> soft(coded.size());
    for (size_t i = 0; i < coded.size(); i++) {
        double v = (2.0 * coded[i] - 1.0) * 127.0 + n(rng);
        soft[i] = (int16_t)std::max(-127.0, std::min(127.0, v));
    }
    return soft;
}

int main() {
    std::mt19937 rng(7);
    // viterbi (viterbi.cpp:225-242)
    {
        const int nb = 768;
        dabgpu::viterbi v(nb);
        for (double sigma : {0.0, 90.0, 160.0}) {
            std::vector<uint8_t> bits(nb);
            for (auto &b : bits) b = rng() & 1;
            auto soft = noisy_mother(rng, bits, sigma);
            std::vector<uint8_t> g(nb), o(nb);
            v.deconvolve(soft.data(), g.data());
            orc_viterbi(soft.data(), nb, o.data());
            CHECK(g == o, "viterbi sigma %.0f", sigma);
        }
        std::printf("viterbi: ok\n");
    }
    // uep / eep deconvolve (deconvolve.cpp:142-366), no energy dispersal
    {
        struct Case { int uep, br, pl, cus; } cases[] = {{1, 128, 3, 96}, {1, 64, 2, 58}, {0, 64, 0103, 48},
                                                         {0, 96, 0204, 54}};
        for (auto &cs : cases) {
            const int frag = cs.cus * 64;
            std::vector<int16_t> in(frag);
            std::uniform_int_distribution<int> u(-127, 127);
            for (auto &x : in) x = (int16_t)u(rng);
            std::vector<uint8_t> g(24 * cs.br), o(24 * cs.br);
            bool ok;
            if (cs.uep) {
                dabgpu::uep_deconvolve d(cs.br, cs.pl);
                ok = d.deconvolve(in.data(), frag, g.data());
            } else {
                dabgpu::eep_deconvolve d(cs.br, cs.pl);
                ok = d.deconvolve(in.data(), frag, g.data());
            }
            std::vector<int16_t> vb(4 * 24 * cs.br + 24 + 64);
            int r = orc_msc_depuncture(cs.uep, cs.br, cs.pl, in.data(), vb.data());
            orc_viterbi(vb.data(), 24 * cs.br, o.data());
            CHECK(ok && r >= 0 && g == o, "%s %d kbps level 0%o", cs.uep ? "uep" : "eep", cs.br, cs.pl);
        }
        std::printf("uep/eep_deconvolve: ok\n");
    }
    // reedSolomon::dec (reed-solomon.cpp:129-141)
    {
        dabgpu::reedSolomon rs(8, 0435, 0, 1, 10);
        for (int t = 0; t < 60; t++) {
            uint8_t data[110], cw[120], og[110], oo[110];
            for (auto &b : data) b = (uint8_t)rng();
            orc_rs_enc(data, cw);
            const int ne = t % 8;
            for (int e = 0; e < ne; e++) cw[rng() % 120] ^= (uint8_t)(1 + rng() % 255);
            const int16_t rg = rs.dec(cw, og, 135), ro = orc_rs_dec(cw, oo);
            CHECK(rg == ro && !std::memcmp(og, oo, 110), "rs t=%d (%d vs %d)", t, rg, ro);
        }
        std::printf("reedSolomon: ok\n");
    }
    // phaseReference::findIndex, ficHandler on a synthetic stream
    {
        dabsynth_subch sc = {0, 96, 128, 3, 1, 0};
        dabsynth_cfg cfg;
        std::memset(&cfg, 0, sizeof cfg);
        cfg.n_frames = 3;
        cfg.pre_offset = 50000;
        cfg.snr_db = 300.0f;
        cfg.amplitude = 1.0f;
        cfg.n_subch = 1;
        cfg.subch = &sc;
        const int64_t n = dabsynth_stream_len(&cfg);
        std::vector<float> iq(2 * n);
        std::vector<uint8_t> fic_truth((size_t)3 * 4 * 768), msc_truth((size_t)12 * 1 * 24 * 128);
        int64_t f0 = 0;
        CHECK(dabsynth_generate(&cfg, 11, iq.data(), fic_truth.data(), msc_truth.data(), nullptr, &f0) == 0, "synth");
        std::vector<orc_frame_info> info(3);
        std::vector<int16_t> soft((size_t)3 * 75 * 3072);
        const int nf = orc_ofdm_run(iq.data(), n, 3, 1, 3, info.data(), soft.data());
        CHECK(nf == 3, "oracle frames %d", nf);
        dabgpu::phaseReference pr(3);
        for (int f = 0; f < nf; f++) {
            const float *w = iq.data() + 2 * info[f].window_start;
            const int32_t g = pr.findIndex((dabgpu::DSPCOMPLEX *)w);
            const int32_t o = orc_find_index(w, 3, nullptr, nullptr);
            CHECK(g == o && g == info[f].start_index, "findIndex frame %d: %d %d %d", f, g, o, info[f].start_index);
        }
        std::printf("phaseReference: ok\n");
        int good = 0, total = 0, mismatch = 0;
        std::vector<uint8_t> ref_bits(768), ref_ok(3);
        int cur_frame = 0;
        dabgpu::ficHandler fh([&](const uint8_t *fib, bool ok, int16_t ficno) {
            total++;
            good += ok ? 1 : 0;
            (void)fib;
            (void)ficno;
        });
        for (int f = 0; f < nf; f++) {
            cur_frame = f;
            for (int l = 1; l <= 3; l++) fh.process_ficBlock(soft.data() + ((size_t)f * 75 + (l - 1)) * 3072, (int16_t)l);
            for (int b = 0; b < 4; b++) {
                orc_fic_process(soft.data() + (size_t)f * 75 * 3072 + 2304 * b, ref_bits.data(), ref_ok.data());
                mismatch += !(ref_ok[0] && ref_ok[1] && ref_ok[2]);
            }
        }
        (void)cur_frame;
        CHECK(total == 12 * nf && good == total && mismatch == 0, "ficHandler %d/%d", good, total);
        std::printf("ficHandler: ok (%d FIBs, ratio %d%%)\n", total, fh.get_ficRatio());
    }
    // ensembleDecoder: 2 streams, UEP + EEP + DAB+ subchannels vs transmitter truth
    {
        dabsynth_subch sc[3] = {{0, 96, 128, 3, 1, 0}, {96, 48, 64, 0103, 0, 1}, {144, 72, 96, 0103, 0, 3}};
        dabsynth_cfg cfg;
        std::memset(&cfg, 0, sizeof cfg);
        const int F = 3, runs = 3;
        cfg.n_frames = F * runs;
        cfg.pre_offset = 50000;
        cfg.snr_db = 300.0f;
        cfg.amplitude = 1.0f;
        cfg.n_subch = 3;
        cfg.subch = sc;
        const int64_t n = dabsynth_stream_len(&cfg);
        const int NC = 4 * F * runs, maxbits = 24 * 128;
        std::vector<std::vector<float>> iq(2, std::vector<float>(2 * n));
        std::vector<std::vector<uint8_t>> fic(2, std::vector<uint8_t>((size_t)F * runs * 4 * 768)),
            msc(2, std::vector<uint8_t>((size_t)NC * 3 * maxbits));
        for (int s = 0; s < 2; s++) {
            int64_t f0;
            dabsynth_generate(&cfg, 100 + s, iq[s].data(), fic[s].data(), msc[s].data(), nullptr, &f0);
        }
        dabgpu::ensembleDecoder::config ec;
        ec.n_streams = 2;
        ec.n_frames = F;
        ec.subch = {{0, 96, 128, 3, 0, 0}, {96, 48, 64, 0103, 1, DABGPU_SUBCH_DABPLUS},
                    {144, 72, 96, 0103, 1, DABGPU_SUBCH_DABPLUS}};
        dabgpu::ensembleDecoder dec(ec);
        int fib_bad = 0, fib_n = 0, msc_bad = 0, msc_n = 0, sf_ok = 0, sf_bad = 0;
        dec.on_fib([&](int s, int64_t frame, int ficno, const uint8_t *bits, bool ok) {
            fib_n++;
            fib_bad += !ok;
            (void)s; (void)frame; (void)ficno; (void)bits;
        });
        dec.on_msc([&](int s, int64_t cif, int k, const uint8_t *bits, int nbits) {
            msc_n++;
            if (std::memcmp(bits, msc[s].data() + ((size_t)cif * 3 + k) * maxbits, nbits)) msc_bad++;
        });
        dec.on_superframe([&](int s, int64_t cif, int k, const dabgpu_superframe &info, const uint8_t *b, int nb) {
            (void)s; (void)cif; (void)k; (void)b;
            if (info.status == 3) {
                sf_ok += (nb > 0 && (info.au_crc_ok & 0xF) == 0xF);
            } else if (info.status == 2) {
                sf_bad++;
            }
        });
        dec.load({(const dabgpu::DSPCOMPLEX *)iq[0].data(), (const dabgpu::DSPCOMPLEX *)iq[1].data()}, {n, n});
        dec.acquire();
        for (int r = 0; r < runs; r++) CHECK(dec.step(), "ensembleDecoder step %d", r);
        CHECK(fib_n == 2 * F * runs * 12 && fib_bad == 0, "FIBs %d bad %d", fib_n, fib_bad);
        CHECK(msc_n == 2 * (NC - 16) * 3 && msc_bad == 0, "MSC %d bad %d", msc_n, msc_bad);
        CHECK(sf_ok >= 2 * 2 * 3 && sf_bad == 0, "superframes ok %d bad %d", sf_ok, sf_bad);
        std::printf("ensembleDecoder: ok (%d FIBs, %d MSC CIF-subchannels, %d superframes)\n", fib_n, msc_n, sf_ok);
    }
    // a functional ficHandler: the GPU-decoded FIBs of an ensemble that describes
    // itself (FIG 0/1, 0/2, 1/0, 1/1) configure the MSC decoder through
    // fib_processor::dataforAudioService, and that decoder reproduces the MSC bits
    {
        dabsynth_subch sc[3] = {{0, 96, 128, 3, 1, 0}, {96, 48, 64, 0103, 0, 1}, {144, 54, 64, 0201, 0, 0}};
        dabsynth_cfg cfg;
        std::memset(&cfg, 0, sizeof cfg);
        const int F = 3, runs = 2;
        cfg.n_frames = F * runs;
        cfg.pre_offset = 50000;
        cfg.snr_db = 30.0f;
        cfg.amplitude = 1.0f;
        cfg.n_subch = 3;
        cfg.subch = sc;
        cfg.figs = 1;
        const int64_t n = dabsynth_stream_len(&cfg);
        const int NC = 4 * F * runs, maxbits = 24 * 128;
        std::vector<float> iq(2 * n);
        std::vector<uint8_t> msc((size_t)NC * 3 * maxbits);
        int64_t f0;
        dabsynth_generate(&cfg, 555, iq.data(), nullptr, msc.data(), nullptr, &f0);
        dabgpu::fib_processor fibs;
        {   // pass 1: FIC only
            dabgpu::ensembleDecoder::config ec;
            ec.n_streams = 1;
            ec.n_frames = F;
            dabgpu::ensembleDecoder dec(ec);
            int good = 0;
            dec.on_fib([&](int, int64_t, int ficno, const uint8_t *bits, bool ok) {
                if (ok) fibs.process_FIB(bits, (uint16_t)ficno), good++;
            });
            dec.load({(const dabgpu::DSPCOMPLEX *)iq.data()}, {n});
            dec.acquire();
            for (int r = 0; r < runs; r++) CHECK(dec.step(), "FIC pass step %d", r);
            CHECK(good == 12 * F * runs, "FIC pass: %d good FIBs", good);
        }
        CHECK(fibs.ensembleName() == "SYNTH ENSEMBLE  ", "ensemble '%s'", fibs.ensembleName().c_str());
        dabgpu::ensembleDecoder::config ec;
        ec.n_streams = 1;
        ec.n_frames = F;
        for (int i = 0; i < 3; i++) {
            char lab[17];
            std::snprintf(lab, sizeof lab, "SERVICE %02d      ", i);
            dabgpu::audiodata a;
            const bool ok = fibs.kindofService(lab) == dabgpu::AUDIO_SERVICE && fibs.dataforAudioService(lab, &a);
            CHECK(ok, "service %d from the FIC", i);
            if (!ok) break;
            CHECK(a.startAddr == sc[i].startAddr && a.length == sc[i].length && a.bitRate == sc[i].bitRate &&
                      a.protLevel == sc[i].protLevel, "service %d subchannel", i);
            ec.subch.push_back({a.startAddr, a.length, a.bitRate, a.protLevel, (int16_t)a.uepFlag,
                                (int16_t)(a.ASCTy == 63 ? DABGPU_SUBCH_DABPLUS : 0)});
        }
        if (ec.subch.size() == 3) {   // pass 2: the services the FIC announced
            dabgpu::ensembleDecoder dec(ec);
            int msc_n = 0, msc_bad = 0, sf_ok = 0;
            dec.on_msc([&](int, int64_t cif, int k, const uint8_t *bits, int nbits) {
                msc_n++;
                if (std::memcmp(bits, msc.data() + ((size_t)cif * 3 + k) * maxbits, nbits)) msc_bad++;
            });
            dec.on_superframe([&](int, int64_t, int, const dabgpu_superframe &info, const uint8_t *, int) {
                sf_ok += info.status == 3;
            });
            dec.load({(const dabgpu::DSPCOMPLEX *)iq.data()}, {n});
            dec.acquire();
            for (int r = 0; r < runs; r++) CHECK(dec.step(), "MSC pass step %d", r);
            CHECK(msc_n == (NC - 16) * 3 && msc_bad == 0, "self-configured MSC %d bad %d", msc_n, msc_bad);
            CHECK(sf_ok >= 1, "self-configured DAB+ superframes %d", sf_ok);
            std::printf("fib_processor + ensembleDecoder: ok (%d MSC CIF-subchannels, %d superframes)\n", msc_n, sf_ok);
        }
    }
    if (failures) {
        std::printf("DROPIN FAILED (%d)\n", failures);
        return 1;
    }
    std::printf("DROPIN OK\n");
    return 0;
}
