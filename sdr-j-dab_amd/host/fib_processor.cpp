// fib_processor.cpp -- see fib_processor.h.  Bit positions and control flow follow
// src/backend/fib-processor.cpp of the reference (line numbers cited per function).
#include "fib_processor.h"

#include <cstdio>

namespace dabgpu {
namespace {

// MSB-first bit fields of a bit array, one bit per byte (dab-constants.h:182-308)
uint32_t bits(const uint8_t *d, int off, int n) {
    uint32_t r = 0;
    for (int i = 0; i < n; i++) r = (r << 1) | (d[off + i] & 1u);
    return r;
}

// Short-form sub-channel table (ETSI EN 300 401 table 8, fib-processor.cpp:30-94):
// for table index 0..63 the sub-channel size in CUs, protection level and bit
// rate, listed per bit rate as (size, level) pairs from the weakest level up.
struct UepRow { int16_t cus, level, kbps; };
const std::vector<UepRow> &uep_table() {
    static const std::vector<UepRow> t = [] {
        struct Group { int kbps; std::vector<std::pair<int, int>> rows; };
        const Group g[] = {
            {32, {{16, 5}, {21, 4}, {24, 3}, {29, 2}, {35, 1}}},
            {48, {{24, 5}, {29, 4}, {35, 3}, {42, 2}, {52, 1}}},
            {56, {{29, 5}, {35, 4}, {42, 3}, {52, 2}}},
            {64, {{32, 5}, {42, 4}, {48, 3}, {58, 2}, {70, 1}}},
            {80, {{40, 5}, {52, 4}, {58, 3}, {70, 2}, {84, 1}}},
            {96, {{48, 5}, {58, 4}, {70, 3}, {84, 2}, {104, 1}}},
            {112, {{58, 5}, {70, 4}, {84, 3}, {104, 2}}},
            {128, {{64, 5}, {84, 4}, {96, 3}, {116, 2}, {140, 1}}},
            {160, {{80, 5}, {104, 4}, {116, 3}, {140, 2}, {168, 1}}},
            {192, {{96, 5}, {116, 4}, {140, 3}, {168, 2}, {208, 1}}},
            {224, {{116, 5}, {140, 4}, {168, 3}, {208, 2}, {232, 1}}},
            {256, {{128, 5}, {168, 4}, {192, 3}, {232, 2}, {280, 1}}},
            {320, {{160, 5}, {208, 4}, {280, 2}}},
            {384, {{192, 5}, {280, 3}, {416, 1}}},
        };
        std::vector<UepRow> v;
        for (const Group &x : g)
            for (auto [cus, lvl] : x.rows) v.push_back({(int16_t)cus, (int16_t)lvl, (int16_t)x.kbps});
        return v;
    }();
    return t;
}

// EBU Latin based repertoire (ETSI TS 101 756 annex C; charsets.cpp:32-67): equal to
// the code point except these
uint32_t ebu_latin(uint8_t c) {
    static const uint16_t hi[128] = {
        0xe1, 0xe0, 0xe9, 0xe8, 0xed, 0xec, 0xf3, 0xf2, 0xfa, 0xf9, 0xd1, 0xc7, 0x15e, 0xdf, 0xa1, 0x132,
        0xe2, 0xe4, 0xea, 0xeb, 0xee, 0xef, 0xf4, 0xf6, 0xfb, 0xfc, 0xf1, 0xe7, 0x15f, 0x11f, 0x131, 0x133,
        0xaa, 0x3b1, 0xa9, 0x2030, 0x11e, 0x11b, 0x148, 0x151, 0x3c0, 0x20ac, 0xa3, 0x24, 0x2190, 0x2191, 0x2192, 0x2193,
        0xba, 0xb9, 0xb2, 0xb3, 0xb1, 0x130, 0x144, 0x171, 0xb5, 0xbf, 0xf7, 0xb0, 0xbc, 0xbd, 0xbe, 0xa7,
        0xc1, 0xc0, 0xc9, 0xc8, 0xcd, 0xcc, 0xd3, 0xd2, 0xda, 0xd9, 0x158, 0x10c, 0x160, 0x17d, 0xd0, 0x13f,
        0xc2, 0xc4, 0xca, 0xcb, 0xce, 0xcf, 0xd4, 0xd6, 0xdb, 0xdc, 0x159, 0x10d, 0x161, 0x17e, 0x111, 0x140,
        0xc3, 0xc5, 0xc6, 0x152, 0x177, 0xdd, 0xd5, 0xd8, 0xde, 0x14a, 0x154, 0x106, 0x15a, 0x179, 0x166, 0xf0,
        0xe3, 0xe5, 0xe6, 0x153, 0x175, 0xfd, 0xf5, 0xf8, 0xfe, 0x14b, 0x155, 0x107, 0x15b, 0x17a, 0x167, 0xff};
    if (c >= 0x80) return hi[c - 0x80];
    switch (c) {
    case 0x1f: return 0x2d;
    case 0x24: return 0xa4;
    case 0x5e: return 0x2015;
    case 0x60: return 0x2551;
    case 0x7e: return 0xaf;
    default: return c;
    }
}

void put_utf8(std::string &s, uint32_t u) {
    if (u < 0x80) {
        s += (char)u;
    } else if (u < 0x800) {
        s += (char)(0xC0 | (u >> 6));
        s += (char)(0x80 | (u & 0x3F));
    } else {
        s += (char)(0xE0 | (u >> 12));
        s += (char)(0x80 | ((u >> 6) & 0x3F));
        s += (char)(0x80 | (u & 0x3F));
    }
}

// toQStringUsingCharset (charsets.cpp:69-95) for the 16 label bytes
std::string label_text(const uint8_t *b, int n, int charset) {
    std::string s;
    if (charset == 0x0F) {                          // UnicodeUtf8
        for (int i = 0; i < n && b[i]; i++) s += (char)b[i];
        return s;
    }
    if (charset == 0x06) {                          // UnicodeUcs2 (QString::fromUtf16, little-endian host)
        for (int i = 0; i + 1 < n; i += 2) {
            const uint32_t u = b[i] | ((uint32_t)b[i + 1] << 8);
            if (!u) break;
            put_utf8(s, u);
        }
        return s;
    }
    // EbuLatin and (as the reference's default branch) everything else; the
    // reference's strlen() stops at the first NUL
    for (int i = 0; i < n && b[i]; i++) put_utf8(s, ebu_latin(b[i]));
    return s;
}

}  // namespace

fib_processor::fib_processor() { clearEnsemble(); }

// fib-processor.cpp:123-160
void fib_processor::process_FIB(const uint8_t *p, uint16_t) {
    int processed = 0;
    const uint8_t *d = p;
    while (processed < 30) {
        const int type = (int)bits(d, 0, 3);
        if (type == 7) return;
        if (type == 0) fig0(d);
        else if (type == 1) fig1(d);
        else if (type == 2) fig2(d);
        processed += (int)bits(d, 3, 5) + 1;
        d = p + processed * 8;
    }
}

// fib-processor.cpp:162-239
void fib_processor::fig0(const uint8_t *d) {
    const int len = (int)bits(d, 3, 5);
    const int pd = (int)bits(d, 8 + 2, 1);
    switch (bits(d, 8 + 3, 5)) {
    case 1:                                        // :278-286
        for (int used = 2; used < len - 1;) used = fig0_1(d, used);
        break;
    case 2:                                        // :356-367
        for (int used = 2; used < len;) used = fig0_2(d, used, pd);
        break;
    case 3:                                        // :424-431
        for (int used = 2; used < len;) used = fig0_3(d, used);
        break;
    case 14:
        fig0_14(d);
        break;
    case 16:
        fig0_16(d);
        break;
    case 17:
        fig0_17(d);
        break;
    default:
        break;
    }
}

// fib-processor.cpp:288-354
int fib_processor::fig0_1(const uint8_t *d, int used) {
    int o = used * 8;
    const int id = (int)bits(d, o, 6);
    subchannel &s = sub_[id];
    s.StartAddr = (int32_t)bits(d, o + 6, 10);
    if (bits(d, o + 16, 1) == 0) {                 // short form: UEP table index
        const UepRow &r = uep_table()[bits(d, o + 18, 6)];
        s.Length = r.cus;
        s.uepFlag = 0;
        s.protLevel = r.level;
        s.BitRate = r.kbps;
        o += 24;
    } else {                                       // long form: EEP
        s.uepFlag = 1;
        const int option = (int)bits(d, o + 17, 3);
        const int level = (int)bits(d, o + 20, 2) + 1;
        const int size = (int)bits(d, o + 22, 10);
        static const int divA[4] = {12, 8, 6, 4}, divB[4] = {27, 21, 18, 15};
        if (option == 0) {                         // EEP-A: level + 0100
            s.protLevel = level + 0100;
            s.Length = size;
            s.BitRate = size / divA[level - 1] * 8;
        } else if (option == 1) {                  // EEP-B: level + 0200
            s.protLevel = level + 0200;
            s.Length = size;
            s.BitRate = size / divB[level - 1] * 32;
        }
        o += 32;
    }
    return o / 8;
}

// fib-processor.cpp:377-422
int fib_processor::fig0_2(const uint8_t *d, int used, int pd) {
    int o = used * 8;
    int32_t sid;
    if (pd == 1) {
        sid = (int32_t)bits(d, o, 32);
        o += 32;
    } else {
        sid = (int32_t)bits(d, o, 16);
        o += 16;
    }
    const int ncomp = (int)bits(d, o + 4, 4);
    o += 8;
    for (int i = 0; i < ncomp; i++) {
        const int8_t tmid = (int8_t)bits(d, o, 2);
        // a new binding writes only these fields: the slot keeps whatever else its
        // previous component left (sub-channel, DSCTy, ... until a FIG 0/3)
        if (tmid == 0) {                           // audio
            const int k = bind(tmid, sid, (int16_t)i);
            if (k >= 0) {
                components_[k].ASCTy = (int16_t)bits(d, o + 2, 6);
                components_[k].subchannelId = (int16_t)bits(d, o + 8, 6);
                components_[k].PS_flag = (int16_t)bits(d, o + 14, 1);
            }
        } else if (tmid == 3) {                    // packet data
            const int k = bind(tmid, sid, (int16_t)i);
            if (k >= 0) {
                components_[k].SCId = (uint16_t)bits(d, o + 2, 12);
                components_[k].PS_flag = (int16_t)bits(d, o + 14, 1);
                components_[k].CAflag = (uint8_t)bits(d, o + 15, 1);
            }
        }
        o += 16;
    }
    return o / 8;
}

// fib-processor.cpp:433-453
int fib_processor::fig0_3(const uint8_t *d, int used) {
    const int o = used * 8;
    const int16_t scid = (int16_t)bits(d, o, 12);
    const int k = find_packet_component(scid);
    if (k >= 0) {
        component &c = components_[k];
        c.DGflag = (int8_t)bits(d, o + 16, 1);
        c.DSCTy = (int16_t)bits(d, o + 18, 6);
        c.subchannelId = (int16_t)bits(d, o + 24, 6);
        c.packetAddress = (int16_t)bits(d, o + 30, 10);
    }
    return used + 7;
}

// fib-processor.cpp:688-705 (FEC of the entries whose SubChId field matches)
void fib_processor::fig0_14(const uint8_t *d) {
    const int len = (int)bits(d, 3, 5);
    for (int used = 2; used < len; used++) {
        const int id = (int)bits(d, used * 8, 6);
        const int16_t fec = (int16_t)bits(d, used * 8 + 6, 2);
        for (subchannel &s : sub_)
            if (s.SubChId == id) s.FEC_scheme = fec;
    }
}

// fib-processor.cpp:707-724: the programme number is stored nowhere the lookups read,
// but every SId gets a service entry
void fib_processor::fig0_16(const uint8_t *d) {
    const int len = (int)bits(d, 3, 5);
    for (int o = 16; o < len * 8; o += 72) find_service((int32_t)bits(d, o, 16));
}

// fib-processor.cpp:726-752
void fib_processor::fig0_17(const uint8_t *d) {
    const int len = (int)bits(d, 3, 5);
    for (int o = 16; o < len * 8;) {
        const int32_t sid = (int32_t)bits(d, o, 16);
        const bool lflag = bits(d, o + 18, 1), ccflag = bits(d, o + 19, 1);
        service &s = services_[find_service(sid)];
        if (lflag) {
            s.language = (int16_t)bits(d, o + 24, 8);
            s.hasLanguage = true;
            o += 8;
        }
        s.programType = (int16_t)bits(d, o + 27, 5);
        o += ccflag ? 40 : 32;
    }
}

// fib-processor.cpp:850-997 (extensions 0, 1 and 5; 3 and 4 are parsed there but
// stored nowhere)
void fib_processor::fig1(const uint8_t *d) {
    const int charset = (int)bits(d, 8, 4);
    const bool oe = bits(d, 12, 1);
    const int ext = (int)bits(d, 13, 3);
    uint8_t raw[16];
    auto read_label = [&](int off) {
        for (int i = 0; i < 16; i++) raw[i] = (uint8_t)bits(d, off + 8 * i, 8);
    };
    if (ext == 0) {                                // ensemble label
        const uint32_t eid = bits(d, 16, 16);
        if (charset <= 16) {
            read_label(32);
            if (!oe) {
                const std::string name = label_text(raw, 16, charset);
                if (firstTime_) {
                    ensemble_ = name;
                    if (ens_cb_) ens_cb_(eid, name);
                }
                firstTime_ = false;
            }
        }
    } else if (ext == 1 || ext == 5) {             // service label (16-bit SId) / data service label (32-bit SId)
        const int32_t sid = (int32_t)(ext == 1 ? bits(d, 16, 16) : bits(d, 16, 32));
        service &s = services_[find_service(sid)];
        if (!s.hasName && charset <= 16) {
            read_label(ext == 1 ? 32 : 48);
            s.label += label_text(raw, 16, charset);
            if (ext == 5) {                          // addtoEnsemble only without MSC_DATA__ for 1/5
                static const uint8_t suffix[8] = {' ', '(', 'd', 'a', 't', 'a', ')', 0};
                s.label += label_text(suffix, 8, charset);
            } else if (svc_cb_) {
                svc_cb_(s.label);
            }
            s.hasName = true;
        }
    }
}

// fib-processor.cpp:998-1037: FIG 2 extension 5, a data service label (32-bit SId)
void fib_processor::fig2(const uint8_t *d) {
    const int charset = (int)bits(d, 8, 4);
    if (bits(d, 13, 3) != 5) return;
    service &s = services_[find_service((int32_t)bits(d, 16, 32))];
    if (!s.hasName && charset <= 16) {
        uint8_t raw[16];
        for (int i = 0; i < 16; i++) raw[i] = (uint8_t)bits(d, 48 + 8 * i, 8);
        s.label += label_text(raw, 16, charset);
        s.hasName = true;
    }
}

// fib-processor.cpp:1041-1058: the in-use entry with this SId, else a new one in the
// first free slot, else entry 0
int fib_processor::find_service(int32_t sid) {
    for (int i = 0; i < 64; i++)
        if (services_[i].inUse && services_[i].serviceId == sid) return i;
    for (int i = 0; i < 64; i++)
        if (!services_[i].inUse) {
            services_[i].inUse = true;
            services_[i].hasName = false;
            services_[i].serviceId = sid;
            return i;
        }
    return 0;
}

// fib-processor.cpp:1060-1075
int fib_processor::find_packet_component(int16_t scid) const {
    for (int i = 0; i < 64; i++)
        if (components_[i].inUse && components_[i].TMid == 3 && components_[i].SCId == (uint16_t)scid) return i;
    return -1;
}

// bind_audioService / bind_packetService (fib-processor.cpp:1077-1140): once per
// (service, component number), in the first free slot; returns the slot (-1: bound
// already, or the table is full, where the reference writes slot -1)
int fib_processor::bind(int8_t tmid, int32_t sid, int16_t compnr) {
    const int s = find_service(sid);
    int first_free = -1;
    for (int i = 0; i < 64; i++) {
        if (!components_[i].inUse) {
            if (first_free < 0) first_free = i;
            continue;
        }
        if (components_[i].service == s && components_[i].componentNr == compnr) return -1;
    }
    if (first_free < 0) return -1;
    component &k = components_[first_free];
    k.inUse = true;
    k.TMid = tmid;
    k.service = s;
    k.componentNr = compnr;
    return first_free;
}

// fib-processor.cpp:1142-1163
void fib_processor::setupforNewFrame() {
    for (component &c : components_) c.inUse = false;
}
void fib_processor::clearEnsemble() {
    for (component &c : components_) c = component();
    for (subchannel &s : sub_) s = subchannel();
    for (service &s : services_) {                 // language / programType / hasLanguage stay
        s.inUse = false;
        s.serviceId = -1;
        s.label.clear();
    }
    ensemble_.clear();
    firstTime_ = true;
}

// fib-processor.cpp:1197-1229
uint8_t fib_processor::kindofService(const std::string &label) {
    for (int i = 0; i < 64; i++) {
        const service &s = services_[i];
        if (!s.inUse || !s.hasName || s.label != label) continue;
        for (const component &c : components_) {
            if (!c.inUse || services_[c.service].serviceId != s.serviceId) continue;
            if (c.TMid == 3) return PACKET_SERVICE;
            if (c.TMid == 0) return AUDIO_SERVICE;
        }
    }
    return UNKNOWN_SERVICE;
}

// fib-processor.cpp:1275-1316
bool fib_processor::dataforAudioService(const std::string &label, audiodata *d) {
    for (int i = 0; i < 64; i++) {
        const service &s = services_[i];
        if (!s.inUse || !s.hasName || s.label != label) continue;
        for (const component &c : components_) {
            if (!c.inUse || services_[c.service].serviceId != s.serviceId) continue;
            if (c.TMid != 0) {
                fprintf(stderr, "fatal error, expected audio service\n");
                return false;
            }
            const subchannel &x = sub_[c.subchannelId];
            d->subchId = c.subchannelId;
            d->startAddr = (int16_t)x.StartAddr;
            d->uepFlag = (uint8_t)x.uepFlag;
            d->protLevel = (int16_t)x.protLevel;
            d->length = (int16_t)x.Length;
            d->bitRate = (int16_t)x.BitRate;
            d->ASCTy = c.ASCTy;
            d->language = s.language;
            d->programType = s.programType;
            return true;
        }
    }
    fprintf(stderr, "service %s insuffiently defined\n", label.c_str());
    return false;
}

// fib-processor.cpp:1231-1273
bool fib_processor::dataforDataService(const std::string &label, packetdata *d) {
    for (int i = 0; i < 64; i++) {
        const service &s = services_[i];
        if (!s.inUse || !s.hasName || s.label != label) continue;
        for (const component &c : components_) {
            if (!c.inUse || services_[c.service].serviceId != s.serviceId) continue;
            if (c.TMid != 3) {
                fprintf(stderr, "fatal error, expected data service\n");
                return false;
            }
            const subchannel &x = sub_[c.subchannelId];
            d->subchId = c.subchannelId;
            d->startAddr = (int16_t)x.StartAddr;
            d->uepFlag = (uint8_t)x.uepFlag;
            d->protLevel = (int16_t)x.protLevel;
            d->DSCTy = c.DSCTy;
            d->length = (int16_t)x.Length;
            d->bitRate = (int16_t)x.BitRate;
            d->FEC_scheme = x.FEC_scheme;
            d->DGflag = c.DGflag;
            d->packetAddress = c.packetAddress;
            return true;
        }
    }
    fprintf(stderr, "service %s insuffiently defined\n", label.c_str());
    return false;
}

std::vector<std::string> fib_processor::serviceLabels() const {
    std::vector<std::string> v;
    for (const service &s : services_)
        if (s.inUse && s.hasName) v.push_back(s.label);
    return v;
}

}  // namespace dabgpu
