// TEST INFRASTRUCTURE: host-side pieces of the OFDM drop-in boundary, no GPU needed:
//  - dabgpu::RingBuffer<T> against the reference ring's contract (ringbuffer.h:127-319):
//    power-of-two capacity (else 32768), partial put/get, wrap-around, skip, flush, and a
//    producer/consumer thread pair moving 2^22 values in odd-sized pieces in order
//    (built with -fsanitize=thread: the pair must be race-free);
//  - the libsndfile stand-in behind ofdmProcessor::startDumping(SNDFILE *): writes
//    <out>.sdr, which tests/test_formats_cpu.py reads back with Python's wave module.
#include <complex>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "dabgpu_dropin.h"

static int failures = 0;
#define CHECK(c, ...)                                        \
    do {                                                     \
        if (!(c)) {                                          \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                        \
            std::printf("\n");                               \
            failures++;                                      \
        }                                                    \
    } while (0)

int main(int argc, char **argv) {
    using dabgpu::RingBuffer;
    {
        RingBuffer<int> r(1000);                         // not a power of two: 32768
        CHECK(r.GetRingBufferWriteAvailable() == 32768, "fallback capacity %d", r.GetRingBufferWriteAvailable());
    }
    {
        RingBuffer<int> r(8);
        int a[12], b[12];
        for (int i = 0; i < 12; i++) a[i] = i + 1;
        CHECK(r.putDataIntoBuffer(a, 12) == 8, "put past capacity");
        CHECK(r.GetRingBufferReadAvailable() == 8 && r.GetRingBufferWriteAvailable() == 0, "full");
        CHECK(r.getDataFromBuffer(b, 5) == 5 && b[0] == 1 && b[4] == 5, "get 5");
        CHECK(r.putDataIntoBuffer(a + 8, 4) == 4, "wrap put");
        CHECK(r.ReadSpace() == 7 && r.WriteSpace() == 1, "spaces %d %d", r.ReadSpace(), r.WriteSpace());
        CHECK(r.skipDataInBuffer(2) == 2, "skip");
        std::memset(b, 0, sizeof b);
        CHECK(r.getDataFromBuffer(b, 12) == 5, "get rest");
        CHECK(b[0] == 8 && b[1] == 9 && b[2] == 10 && b[3] == 11 && b[4] == 12, "order across the wrap %d %d", b[0], b[4]);
        CHECK(r.getDataFromBuffer(b, 1) == 0, "empty");
        r.putDataIntoBuffer(a, 3);
        r.FlushRingBuffer();
        CHECK(r.GetRingBufferReadAvailable() == 0 && r.GetRingBufferWriteAvailable() == 8, "flush");
    }
    {
        RingBuffer<std::complex<float>> r(2 * 1536);     // gui.cpp:109's iqBuffer
        const int N = 1 << 22;
        long bad = 0;
        std::thread prod([&] {
            std::vector<std::complex<float>> v(777);
            int k = 0;
            while (k < N) {
                const int n = std::min((int)v.size(), N - k);
                for (int i = 0; i < n; i++) v[i] = std::complex<float>((float)(k + i), -(float)(k + i));
                int done = 0;
                while (done < n) done += r.putDataIntoBuffer(v.data() + done, n - done);
                k += n;
            }
        });
        std::vector<std::complex<float>> w(1001);
        int k = 0;
        while (k < N) {
            const int got = r.getDataFromBuffer(w.data(), (int)w.size());
            for (int i = 0; i < got; i++) bad += w[i] != std::complex<float>((float)(k + i), -(float)(k + i));
            k += got;
        }
        prod.join();
        CHECK(bad == 0, "%ld values out of order", bad);
    }
    if (argc > 1) {                                      // gui.cpp:861-893 + ofdm-processor.cpp:150-157
        dabgpu::SF_INFO info;
        std::memset(&info, 0, sizeof info);
        info.samplerate = 2048000;
        info.channels = 2;
        info.format = dabgpu::SF_FORMAT_WAV | dabgpu::SF_FORMAT_PCM_16;
        dabgpu::SNDFILE *f = dabgpu::sf_open(argv[1], dabgpu::SFM_WRITE, &info);
        CHECK(f != nullptr, "sf_open %s", argv[1]);
        std::vector<int16_t> buf(2 * 4096);
        for (int blk = 0; blk < 3 && f; blk++) {
            for (int i = 0; i < 4096; i++) {
                buf[2 * i] = (int16_t)(blk * 4096 + i - 6000);
                buf[2 * i + 1] = (int16_t)(-(blk * 4096 + i));
            }
            CHECK(dabgpu::sf_writef_short(f, buf.data(), 4096) == 4096, "sf_writef_short");
        }
        CHECK(dabgpu::sf_close(f) == 0, "sf_close");
        info.format = dabgpu::SF_FORMAT_WAV;             // only PCM16 is supported
        CHECK(dabgpu::sf_open(argv[1], dabgpu::SFM_WRITE, &info) == nullptr, "non-PCM16 refused");
    }
    if (failures) {
        std::printf("RINGBUFFER FAILED (%d)\n", failures);
        return 1;
    }
    std::printf("RINGBUFFER OK\n");
    return 0;
}
