// TEST INFRASTRUCTURE: a C surface over the host MSC consumers (msc_consumers.h) so the
// CPU tests can drive mp2Processor and packetAssembler from Python (ctypes) and
// compare them with the restatements in tests/oracle_py.py.
#include <cstring>
#include <vector>

#include "msc_consumers.h"

struct Capture {
    std::vector<std::vector<uint8_t>> items;
    std::vector<int> rates;
};

extern "C" {

void *cw_mp2_new(int bitRate) {
    auto *c = new Capture();
    auto *p = new dabgpu::mp2Processor((int16_t)bitRate, [c](const uint8_t *f, int32_t nbits, int32_t rate) {
        c->items.emplace_back(f, f + nbits / 8);
        c->rates.push_back(rate);
    });
    return new std::pair<dabgpu::mp2Processor *, Capture *>(p, c);
}
void cw_mp2_add(void *h, uint8_t *bits, int n) {
    static_cast<std::pair<dabgpu::mp2Processor *, Capture *> *>(h)->first->addtoFrame(bits, (int16_t)n);
}
void *cw_pa_new(int DSCTy, int DGflag) {
    auto *c = new Capture();
    auto *p = new dabgpu::packetAssembler((uint8_t)DSCTy, (uint8_t)DGflag,
                                          [c](const std::vector<uint8_t> &bits) { c->items.push_back(bits); });
    return new std::pair<dabgpu::packetAssembler *, Capture *>(p, c);
}
void cw_pa_add(void *h, uint8_t *bits, int n) {
    static_cast<std::pair<dabgpu::packetAssembler *, Capture *> *>(h)->first->add(bits, (int16_t)n);
}
int cw_pa_crc_errors(void *h) {
    return static_cast<std::pair<dabgpu::packetAssembler *, Capture *> *>(h)->first->crcErrors();
}
// captured item i (bytes / bits) into out (size maxn); returns its length, -1 past the end
int cw_item(void *h, int i, uint8_t *out, int maxn, int *rate) {
    Capture *c = static_cast<std::pair<void *, Capture *> *>(h)->second;
    if (i < 0 || i >= (int)c->items.size()) return -1;
    const auto &v = c->items[i];
    std::memcpy(out, v.data(), std::min<size_t>(v.size(), (size_t)maxn));
    if (rate) *rate = i < (int)c->rates.size() ? c->rates[i] : 0;
    return (int)v.size();
}

}
