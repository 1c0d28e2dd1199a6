// TEST INFRASTRUCTURE: drives dabgpu::fib_processor (sdr-j-dab_amd/host/fib_processor.*)
// from a script on stdin and prints what its public interface answers, one JSON line
// per query, for tests/test_fib_cpu.py to compare with the restatement of the
// reference's fib-processor.cpp in tests/oracle_py.py (FibProcessor).
//   F <64 hex digits>   process_FIB of one FIB (32 bytes, bits MSB first)
//   C                   clearEnsemble
//   N                   setupforNewFrame
//   Q <hex>             kindofService / dataforAudioService / dataforDataService of the
//                       label with these UTF-8 bytes
//   D                   service labels (slot order) and the callbacks since the last D
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "fib_processor.h"

using namespace dabgpu;

static std::string hex(const std::string &s) {
    static const char *h = "0123456789abcdef";
    std::string o;
    for (unsigned char c : s) {
        o += h[c >> 4];
        o += h[c & 15];
    }
    return o;
}
static std::string unhex(const std::string &s) {
    std::string o;
    for (size_t i = 0; i + 1 < s.size(); i += 2) o += (char)std::stoi(s.substr(i, 2), nullptr, 16);
    return o;
}

int main() {
    fib_processor fp;
    std::vector<std::string> events;
    fp.on_ensemble([&](uint32_t eid, const std::string &name) {
        events.push_back("[\"E\", " + std::to_string(eid) + ", \"" + hex(name) + "\"]");
    });
    fp.on_service([&](const std::string &label) { events.push_back("[\"S\", \"" + hex(label) + "\"]"); });
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line.empty()) continue;
        const char op = line[0];
        const std::string arg = line.size() > 2 ? line.substr(2) : std::string();
        if (op == 'F') {
            const std::string bytes = unhex(arg);
            uint8_t bits[256];
            for (int i = 0; i < 256; i++) bits[i] = ((uint8_t)bytes[i >> 3] >> (7 - (i & 7))) & 1;
            fp.process_FIB(bits, 0);
        } else if (op == 'C') {
            fp.clearEnsemble();
        } else if (op == 'N') {
            fp.setupforNewFrame();
        } else if (op == 'Q') {
            const std::string label = unhex(arg);
            const int kind = fp.kindofService(label);
            audiodata a;
            packetdata p;
            std::memset(&a, 0, sizeof a);
            std::memset(&p, 0, sizeof p);
            const bool ha = fp.dataforAudioService(label, &a);
            const bool hp = fp.dataforDataService(label, &p);
            std::printf("{\"q\": \"%s\", \"kind\": %d, \"audio\": ", arg.c_str(), kind);
            if (ha)
                std::printf("[%d, %d, %d, %d, %d, %d, %d, %d, %d]", a.subchId, a.startAddr, a.uepFlag, a.protLevel,
                            a.length, a.bitRate, a.ASCTy, a.language, a.programType);
            else
                std::printf("null");
            std::printf(", \"data\": ");
            if (hp)
                std::printf("[%d, %d, %d, %d, %d, %d, %d, %d, %d, %d]", p.subchId, p.startAddr, p.uepFlag, p.protLevel,
                            p.DSCTy, p.length, p.bitRate, p.FEC_scheme, p.DGflag, p.packetAddress);
            else
                std::printf("null");
            std::printf("}\n");
        } else if (op == 'D') {
            std::printf("{\"labels\": [");
            const std::vector<std::string> ls = fp.serviceLabels();
            for (size_t i = 0; i < ls.size(); i++) std::printf("%s\"%s\"", i ? ", " : "", hex(ls[i]).c_str());
            std::printf("], \"events\": [");
            for (size_t i = 0; i < events.size(); i++) std::printf("%s%s", i ? ", " : "", events[i].c_str());
            std::printf("]}\n");
            events.clear();
        }
    }
    return 0;
}
