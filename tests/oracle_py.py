"""TEST INFRASTRUCTURE: ctypes access to the CPU oracle (oracle/liboracle.so, our
C restatement) and, when present, the reference's own compiled sources
(oracle/_ref/libdabref.so).  Used only by tests/, smoke() and bench's CPU baseline."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "liboracle.so")
REF = os.path.join(ROOT, "oracle", "_ref", "libdabref.so")


class FrameInfo(C.Structure):
    _fields_ = [("window_start", C.c_int64), ("start_index", C.c_int32), ("coarse", C.c_int32),
                ("fine", C.c_int16), ("correction", C.c_int16), ("lp_window", C.c_int32)]


def P(a):
    return C.c_void_p(a.ctypes.data)


_o = None
_r = None


def oracle():
    global _o
    if _o is None:
        _o = C.CDLL(ORACLE)
        _o.orc_get_phi.restype = C.c_float
        _o.orc_find_index.restype = C.c_int32
        _o.orc_process_block0.restype = C.c_int16
        _o.orc_rs_dec.restype = C.c_int16
        _o.orc_ofdm_run.argtypes = [C.c_void_p, C.c_int64, C.c_int16, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        _o.orc_ofdm_run_fft.argtypes = [C.c_void_p, C.c_int64, C.c_int16, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_int]
        _o.orc_process_block0_fft.restype = C.c_int16
        _o.orc_null_scan.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        _o.orc_get_snr.restype = C.c_int16
        _o.orc_init()           # tables built once: the functions are then safe from threads
    return _o


def ref():
    """reference sources compiled by oracle/Makefile (None when not built)."""
    global _r
    if _r is None and os.path.exists(REF):
        _r = C.CDLL(REF)
        _r.ref_get_phi.restype = C.c_float
    return _r


def viterbi(soft, nbits):
    out = np.zeros(nbits, np.uint8)
    oracle().orc_viterbi(P(np.ascontiguousarray(soft, np.int16)), nbits, P(out))
    return out


def fic_process(block):
    bits = np.zeros(768, np.uint8)
    ok = np.zeros(3, np.uint8)
    oracle().orc_fic_process(P(np.ascontiguousarray(block, np.int16)), P(bits), P(ok))
    return bits, ok


def prbs(n):
    out = np.zeros(n, np.uint8)
    oracle().orc_prbs(n, P(out))
    return out


def msc_deconvolve(uep, bitrate, plevel, frag):
    nb = 24 * bitrate
    vb = np.zeros(4 * nb + 24, np.int16)
    used = oracle().orc_msc_depuncture(uep, bitrate, plevel, P(np.ascontiguousarray(frag, np.int16)), P(vb))
    assert used >= 0
    out = viterbi(vb, nb)
    return out ^ prbs(nb)


def ofdm_run(iq, max_frames, threshold=3, method=1, fft_kind=0):
    """ofdmProcessor::run over a cf32 stream; fft_kind 1 runs it with the fp32 radix-4 FFT
    (orc_fft2048_f32, FFTW3f's precision class: the CPU baseline) instead of the double one"""
    info = (FrameInfo * max_frames)()
    soft = np.zeros((max_frames, 75, 3072), np.int16)
    if fft_kind:
        n = oracle().orc_ofdm_run_fft(P(iq), C.c_int64(len(iq) // 2), threshold, method, max_frames, info, P(soft),
                                      fft_kind)
    else:
        n = oracle().orc_ofdm_run(P(iq), C.c_int64(len(iq) // 2), threshold, method, max_frames, info, P(soft))
    return n, list(info)[:n], soft[:n]


class Display(C.Structure):
    _fields_ = [("iq_disp", C.c_void_p), ("disp_frame", C.c_void_p), ("max_disp", C.c_int32), ("n_disp", C.c_int32),
                ("spec_start", C.c_void_p), ("max_spec", C.c_int32), ("n_spec", C.c_int32), ("token", C.c_int32)]


def ofdm_run_display(iq, max_frames, threshold=3, method=1, max_disp=64, max_spec=64, token=2):
    """ofdm_run plus the reference's display feeds: (n, info, soft, iq_disp [k][1536] complex64,
    disp_frame [k], spec_start [k]) -- iqBuffer (ofdm-decoder.cpp:192-206) and
    spectrumBuffer (ofdm-processor.cpp:161-180,220-238) emissions in order"""
    info = (FrameInfo * max_frames)()
    soft = np.zeros((max_frames, 75, 3072), np.int16)
    disp = np.zeros((max_disp, 1536, 2), np.float32)
    dfr = np.zeros(max_disp, np.int32)
    spec = np.zeros(max_spec, np.int64)
    d = Display(disp.ctypes.data, dfr.ctypes.data, max_disp, 0, spec.ctypes.data, max_spec, 0, token)
    n = oracle().orc_ofdm_run_display(P(iq), C.c_int64(len(iq) // 2), C.c_int16(threshold), method, max_frames, info,
                                      P(soft), C.byref(d))
    nd, ns = min(d.n_disp, max_disp), min(d.n_spec, max_spec)
    return (n, list(info)[:n], soft[:n], disp[:nd, :, 0] + 1j * disp[:nd, :, 1], dfr[:nd], spec[:ns])


def null_scan(iq, n, scan=True):
    """ofdmProcessor::run's null search over iq[0, n) with scanMode (ofdm-processor.cpp:259-338):
    (found, attempts, no_signal, pos) where the samples run out or a null's end is found"""
    a, ns, pos = C.c_int32(), C.c_int32(), C.c_int64()
    found = oracle().orc_null_scan(P(iq), C.c_int64(n), int(scan), C.byref(a), C.byref(ns), C.byref(pos))
    return found, a.value, ns.value, pos.value


def process_token(sym_ts, phase_ref, fft_kind=0):
    """returns ibits, softf; updates phase_ref (cf32 float array [4096]) in place.  fft_kind 1:
    the fp32 radix-4 FFT (the soft values' fp32 floor) instead of the double one"""
    ib = np.zeros(3072, np.int16)
    sf = np.zeros(3072, np.float32)
    if fft_kind:
        oracle().orc_process_token_fft(P(np.ascontiguousarray(sym_ts, np.float32)), P(phase_ref), P(ib), P(sf),
                                       fft_kind)
    else:
        oracle().orc_process_token(P(np.ascontiguousarray(sym_ts, np.float32)), P(phase_ref), P(ib), P(sf))
    return ib, sf


def process_block0(blk, flag=1, method=1, fft_kind=0):
    pr = np.zeros(4096, np.float32)
    if fft_kind:
        c = oracle().orc_process_block0_fft(P(np.ascontiguousarray(blk, np.float32)), P(pr), flag, method, fft_kind)
    else:
        c = oracle().orc_process_block0(P(np.ascontiguousarray(blk, np.float32)), P(pr), flag, method)
    return c, pr


def find_index(win, level=3):
    mx, sm = C.c_float(), C.c_float()
    r = oracle().orc_find_index(P(np.ascontiguousarray(win, np.float32)), level, C.byref(mx), C.byref(sm))
    return r, mx.value, sm.value


def rs_dec(cw):
    """reedSolomon::dec(rsIn, rsOut, 135) (reed-solomon.cpp:129-141): (out[110], ret)."""
    out = np.zeros(110, np.uint8)
    r = oracle().orc_rs_dec(P(np.ascontiguousarray(cw, np.uint8)), P(out))
    return out, int(r)


class MP4:
    """mp4Processor::addtoFrame state machine (mp4processor.cpp:107-292) over
    successive CIF payloads of one DAB+ subchannel."""

    class _St(C.Structure):
        _fields_ = [("bitRate", C.c_int), ("fill", C.c_int), ("blocks", C.c_int), ("ring", C.c_uint8 * (120 * 48))]

    def __init__(self, bitrate):
        self.st = MP4._St()
        self.br = bitrate
        oracle().orc_mp4_init(C.byref(self.st), bitrate)

    def add(self, bits):
        """-> dict(status, out[110*RSDims], n_corrected, num_aus, au_start, au_crc)"""
        rs = self.br // 8
        out = np.zeros(110 * rs, np.uint8)
        nc = C.c_int16(0)
        na = C.c_int(0)
        aus = np.zeros(8, np.int16)
        crc = np.zeros(8, np.uint8)
        st = oracle().orc_mp4_add(C.byref(self.st), P(np.ascontiguousarray(bits, np.uint8)), P(out),
                                  C.byref(nc), C.byref(na), P(aus), P(crc))
        return dict(status=int(st), out=out, n_corrected=int(nc.value), num_aus=int(na.value),
                    au_start=aus, au_crc=crc)


def get_snr(spectrum):
    """get_snr (ofdm-decoder.cpp:212-230) of a cf32[2048] spectrum (float array [4096])"""
    return int(oracle().orc_get_snr(P(np.ascontiguousarray(spectrum, np.float32))))


def fft(x, inverse=False, fft_kind=0):
    """the oracle's 2048-point FFT of cf32 [4096]: double precision rounded to float
    (fft_kind 0), the fp32 radix-4 Stockham transform (1), fp32 radix-2 DIT (2) / DIF (3)"""
    out = np.zeros(4096, np.float32)
    oracle().orc_fft2048_kind(P(np.ascontiguousarray(x, np.float32)), P(out), int(inverse), int(fft_kind))
    return out


def decode_stream(iq, max_frames, subch, method=1, threshold=3):
    """The reference CPU path restated, over one stream: ofdmProcessor::run (frames,
    soft bits), ficHandler::process_ficInput per FIC block, dabConcurrent per
    subchannel (16-CIF de-interleave, UEP/EEP depuncture, Viterbi, energy dispersal).
    subch: tuples (startAddr, CUs, bitRate, protLevel, uep, ...) with uep = 1 for UEP.
    Returns dict(n, info, soft [n,75,3072], fic [n,4,768], crc [n,12], msc [4n][nsub][24*maxbr])."""
    n, info, soft = ofdm_run(iq, max_frames, threshold=threshold, method=method)
    fic = np.zeros((n, 4, 768), np.uint8)
    crc = np.zeros((n, 12), np.uint8)
    for f in range(n):
        blk = soft[f, 0:3].reshape(-1)
        for b in range(4):
            fic[f, b], crc[f, 3 * b:3 * b + 3] = fic_process(blk[2304 * b:2304 * (b + 1)])
    maxb = 24 * max([sc[2] for sc in subch] + [8])
    msc = np.zeros((4 * n, len(subch), maxb), np.uint8)
    cifs = soft[:, 3:75].reshape(4 * n, -1)
    for k, sc in enumerate(subch):
        sa, ln, br, pl, uep = sc[:5]
        frag = np.ascontiguousarray(cifs[:, sa * 64:(sa + ln) * 64])
        out = np.zeros((4 * n, 24 * br), np.uint8)
        assert oracle().orc_msc_stream(uep, br, pl, ln * 64, 4 * n, P(frag), P(out)) == 0
        msc[:, k, :24 * br] = out
    return dict(n=n, info=info, soft=soft, fic=fic, crc=crc, msc=msc)


def decode_streams(iqs, max_frames, subch, method=1, threads=16):
    """decode_stream over several streams on a thread pool (the oracle is reentrant
    and ctypes drops the GIL during the calls)"""
    from concurrent.futures import ThreadPoolExecutor
    oracle()
    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        return list(ex.map(lambda x: decode_stream(x, max_frames, subch, method), iqs))


# ---- MSC consumers (host code in the product; restated here as the checker) --------
def check_crc_bits(bits):
    """check_CRC_bits (dab-constants.h:310-340) on a bit list; inverts the last 16 in place"""
    n = len(bits)
    for i in range(n - 16, n):
        bits[i] ^= 1
    b = [1] * 16
    poly = [0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0]
    for i in range(n):
        if (b[0] ^ bits[i]) == 1:
            for f in range(15):
                b[f] = poly[f] ^ b[f + 1]
            b[15] = 1
        else:
            b[:15] = b[1:16]
            b[15] = 0
    return sum(b) == 0


class MP2:
    """mp2Processor::addtoFrame (mp2processor.cpp:572-629): 12-one sync, 24-bit header
    (sample rate via mp2sampleRate :276-285, setSamplerate :262-269), frame of 24*bitRate
    bits (twice that at 24 kHz).  frames: list of (bytes, sampleRate)."""
    RATES = [44100, 48000, 32000, 0, 22050, 24000, 16000, 0]

    def __init__(self, bitrate):
        self.size = 24 * bitrate
        self.frame = bytearray(2 * self.size)
        self.ok = self.hc = self.bc = 0
        self.baud = 48000
        self.frames = []

    def _bit(self, b, nm):
        if b:
            self.frame[nm // 8] |= 1 << (7 - (nm & 7))
        else:
            self.frame[nm // 8] &= ~(1 << (7 - (nm & 7))) & 0xFF

    def add(self, bits):
        lf = self.size if self.baud == 48000 else 2 * self.size
        for v in bits:
            if self.ok == 2:
                self._bit(v, self.bc)
                self.bc += 1
                if self.bc >= lf:
                    self.frames.append((bytes(self.frame[:lf // 8]), self.baud))
                    self.ok = self.hc = self.bc = 0
            elif self.ok == 0:
                if v == 1:
                    self.hc += 1
                    if self.hc == 12:
                        self.bc = 0
                        for _ in range(12):
                            self._bit(1, self.bc)
                            self.bc += 1
                        self.ok = 1
                else:
                    self.hc = 0
            else:
                self._bit(v, self.bc)
                self.bc += 1
                if self.bc == 24:
                    f = self.frame
                    rate = 0
                    if f[0] == 0xFF and (f[1] & 0xF6) == 0xF4 and f[2] - 0x10 < 0xE0:
                        rate = MP2.RATES[(((f[1] & 0x08) >> 1) ^ 4) + ((f[2] >> 2) & 3)]
                    if rate in (48000, 24000):
                        self.baud = rate
                    self.ok = 2
            lf = self.size if self.baud == 48000 else 2 * self.size


class Datagroups:
    """mscDatagroup::handlePackets / handlePacket / handleTDCAsyncstream
    (msc-datagroup.cpp:221-339): groups = list of data-group bit lists."""

    def __init__(self, dscty, dgflag):
        self.dscty, self.dgflag = dscty, dgflag
        self.state, self.addr, self.series = 0, -1, []
        self.groups, self.crc_errors = [], 0

    @staticmethod
    def _get(d, off, n):
        r = 0
        for i in range(n):
            r = (r << 1) | d[off + i]
        return r

    def add(self, bits):
        data = [int(x) for x in bits]
        if self.dscty == 5 and self.dgflag:
            pl = (self._get(data, 0, 2) + 1) * 24
            seg = data[:pl * 8]
            check_crc_bits(seg)
            return
        pos, length = 0, len(data)
        while True:
            plen = (self._get(data, pos, 2) + 1) * 24 * 8
            if length < plen:
                return
            self._packet(data, pos)
            length -= plen
            if length < 2:
                return
            pos += plen

    def _packet(self, data, pos):
        g = lambda o, n: self._get(data, pos + o, n)
        plen = (g(0, 2) + 1) * 24
        fl, address, useful = g(4, 2), g(6, 10), g(17, 7)
        seg = data[pos:pos + plen * 8]
        ok = check_crc_bits(seg)
        data[pos:pos + plen * 8] = seg
        if not ok:
            self.crc_errors += 1
            return
        if address == 0:
            return
        if self.addr == -1:
            self.addr = address
        if self.addr != address:
            return
        take = data[pos + 24:pos + 24 + 8 * useful]
        if self.state == 0:
            if fl == 2:
                self.state, self.series = 1, list(take)
            elif fl == 3:
                self.series = list(take)
                self.groups.append(list(self.series))
            else:
                self.series = []
        else:
            if fl == 0:
                self.series += take
            elif fl == 1:
                self.series += take
                self.groups.append(list(self.series))
                self.state = 0
            elif fl == 2:
                self.state, self.series = 1, list(take)
            else:
                self.state, self.series = 0, []


# ---- FIG parser: fib-processor.cpp restated (TEST INFRASTRUCTURE) ----------------
# ETSI EN 300 401 table 8 (fib-processor.cpp:32-95): (CUs, protection level, kbit/s)
UEP_TABLE = [
    (16, 5, 32), (21, 4, 32), (24, 3, 32), (29, 2, 32), (35, 1, 32),
    (24, 5, 48), (29, 4, 48), (35, 3, 48), (42, 2, 48), (52, 1, 48),
    (29, 5, 56), (35, 4, 56), (42, 3, 56), (52, 2, 56),
    (32, 5, 64), (42, 4, 64), (48, 3, 64), (58, 2, 64), (70, 1, 64),
    (40, 5, 80), (52, 4, 80), (58, 3, 80), (70, 2, 80), (84, 1, 80),
    (48, 5, 96), (58, 4, 96), (70, 3, 96), (84, 2, 96), (104, 1, 96),
    (58, 5, 112), (70, 4, 112), (84, 3, 112), (104, 2, 112),
    (64, 5, 128), (84, 4, 128), (96, 3, 128), (116, 2, 128), (140, 1, 128),
    (80, 5, 160), (104, 4, 160), (116, 3, 160), (140, 2, 160), (168, 1, 160),
    (96, 5, 192), (116, 4, 192), (140, 3, 192), (168, 2, 192), (208, 1, 192),
    (116, 5, 224), (140, 4, 224), (168, 3, 224), (208, 2, 224), (232, 1, 224),
    (128, 5, 256), (168, 4, 256), (192, 3, 256), (232, 2, 256), (280, 1, 256),
    (160, 5, 320), (208, 4, 320), (280, 2, 320),
    (192, 5, 384), (280, 3, 384), (416, 1, 384)]

# EBU Latin based repertoire -> UCS-2 (ETSI TS 101 756 annex C; charsets.cpp:32-67):
# identity except these code points
_EBU_DIFF = {0x1f: 0x2d, 0x24: 0xa4, 0x5e: 0x2015, 0x60: 0x2551, 0x7e: 0xaf}
_EBU_HI = [
    0xe1, 0xe0, 0xe9, 0xe8, 0xed, 0xec, 0xf3, 0xf2, 0xfa, 0xf9, 0xd1, 0xc7, 0x15e, 0xdf, 0xa1, 0x132,
    0xe2, 0xe4, 0xea, 0xeb, 0xee, 0xef, 0xf4, 0xf6, 0xfb, 0xfc, 0xf1, 0xe7, 0x15f, 0x11f, 0x131, 0x133,
    0xaa, 0x3b1, 0xa9, 0x2030, 0x11e, 0x11b, 0x148, 0x151, 0x3c0, 0x20ac, 0xa3, 0x24, 0x2190, 0x2191, 0x2192, 0x2193,
    0xba, 0xb9, 0xb2, 0xb3, 0xb1, 0x130, 0x144, 0x171, 0xb5, 0xbf, 0xf7, 0xb0, 0xbc, 0xbd, 0xbe, 0xa7,
    0xc1, 0xc0, 0xc9, 0xc8, 0xcd, 0xcc, 0xd3, 0xd2, 0xda, 0xd9, 0x158, 0x10c, 0x160, 0x17d, 0xd0, 0x13f,
    0xc2, 0xc4, 0xca, 0xcb, 0xce, 0xcf, 0xd4, 0xd6, 0xdb, 0xdc, 0x159, 0x10d, 0x161, 0x17e, 0x111, 0x140,
    0xc3, 0xc5, 0xc6, 0x152, 0x177, 0xdd, 0xd5, 0xd8, 0xde, 0x14a, 0x154, 0x106, 0x15a, 0x179, 0x166, 0xf0,
    0xe3, 0xe5, 0xe6, 0x153, 0x175, 0xfd, 0xf5, 0xf8, 0xfe, 0x14b, 0x155, 0x107, 0x15b, 0x17a, 0x167, 0xff]


def charset_text(raw, charset):
    """toQStringUsingCharset (charsets.cpp:69-95) of a NUL-terminated byte string:
    UTF-8 (0x0F) decoded, EBU Latin (0x00 and every other value) mapped per byte
    up to the first NUL.  (UCS-2, 0x06, reads past the reference's buffer when the
    label has no zero pair: not restated.)"""
    raw = bytes(raw)
    if 0 in raw:
        raw = raw[:raw.index(0)]
    if charset == 0x0F:
        return raw.decode("utf-8", "replace")
    return "".join(chr(_EBU_HI[b - 0x80] if b >= 0x80 else _EBU_DIFF.get(b, b)) for b in raw)


class FibProcessor:
    """fib_processor (fib-processor.cpp) restated over the FIGs that reach the service
    lookups: FIG 0/1, 0/2, 0/3, 0/14, 0/16, 0/17, 1/0, 1/1, 1/5, 2/5; the lookups
    kindofService / dataforAudioService / dataforDataService; clearEnsemble /
    setupforNewFrame.  Signals are recorded in `events` (("E", EId, name) for
    nameofEnsemble, ("S", label) for addtoEnsemble)."""

    UNKNOWN, AUDIO, PACKET = 0o100, 0o101, 0o102

    def __init__(self):
        self.services = [dict(inUse=False, serviceId=-1, hasName=False, label="", language=0,
                              programType=0, hasLanguage=False) for _ in range(64)]
        self.events = []
        self.clearEnsemble()                                       # :98-114

    @staticmethod
    def _bits(d, off, n):                                          # getBits / getLBits (dab-constants.h:182-308)
        v = 0
        for i in range(n):
            v = (v << 1) | (int(d[off + i]) & 1)
        return v

    def process_FIB(self, d):                                      # :123-158
        done = 0
        p = 0
        while done < 30:
            t = self._bits(d[p:], 0, 3)
            if t == 7:
                return
            if t == 0:
                self._fig0(d[p:])
            elif t == 1:
                self._fig1(d[p:])
            elif t == 2:
                self._fig2(d[p:])
            done += self._bits(d[p:], 3, 5) + 1
            p = done * 8

    def _fig0(self, d):                                            # :162-239
        ext = self._bits(d, 8 + 3, 5)
        L = self._bits(d, 3, 5)
        pd = self._bits(d, 8 + 2, 1)
        if ext == 1:                                               # :278-286
            used = 2
            while used < L - 1:
                used = self._fig0_1(d, used)
        elif ext == 2:                                             # :356-367
            used = 2
            while used < L:
                used = self._fig0_2(d, used, pd)
        elif ext == 3:                                             # :424-431
            used = 2
            while used < L:
                used = self._fig0_3(d, used)
        elif ext == 14:                                            # :688-705
            used = 2
            while used < L:
                sid = self._bits(d, used * 8, 6)
                fec = self._bits(d, used * 8 + 6, 2)
                used += 1
                for f in self.ficList:
                    if f["SubChId"] == sid:
                        f["FEC_scheme"] = fec
        elif ext == 16:                                            # :707-724
            off = 16
            while off < L * 8:
                s = self._find_service(self._bits(d, off, 16))
                if not s.get("hasPNum"):
                    s["hasPNum"] = True
                off += 72
        elif ext == 17:                                            # :726-752
            off = 16
            while off < L * 8:
                sid = self._bits(d, off, 16)
                lflag = self._bits(d, off + 18, 1)
                ccflag = self._bits(d, off + 19, 1)
                s = self._find_service(sid)
                if lflag:
                    s["language"] = self._bits(d, off + 24, 8)
                    s["hasLanguage"] = True
                    off += 8
                s["programType"] = self._bits(d, off + 27, 5)
                off += 40 if ccflag else 32

    def _fig0_1(self, d, used):                                    # :288-347
        o = used * 8
        sid = self._bits(d, o, 6)
        f = self.ficList[sid]
        f["StartAddr"] = self._bits(d, o + 6, 10)
        if self._bits(d, o + 16, 1) == 0:
            cus, lvl, rate = UEP_TABLE[self._bits(d, o + 18, 6)]
            f.update(Length=cus, uepFlag=0, protLevel=lvl, BitRate=rate)
            o += 24
        else:
            f["uepFlag"] = 1
            option = self._bits(d, o + 17, 3)
            lvl = self._bits(d, o + 20, 2) + 1
            size = self._bits(d, o + 22, 10)
            if option == 0:
                f["protLevel"] = lvl + 0o100
                f["Length"] = size
                f["BitRate"] = size // {1: 12, 2: 8, 3: 6, 4: 4}[lvl] * 8
            elif option == 1:
                f["protLevel"] = lvl + 0o200
                f["Length"] = size
                f["BitRate"] = size // {1: 27, 2: 21, 3: 18, 4: 15}[lvl] * 32
            o += 32
        return o // 8

    def _fig0_2(self, d, used, pd):                                # :377-418
        o = used * 8
        if pd == 1:
            sid = self._bits(d, o, 32)
            o += 32
        else:
            sid = self._bits(d, o, 16)
            o += 16
        sid = sid - (1 << 32) if sid >= 1 << 31 else sid           # int32_t SId
        n = self._bits(d, o + 4, 4)
        o += 8
        for i in range(n):
            tmid = self._bits(d, o, 2)
            if tmid == 0:
                self._bind(0, sid, i, dict(ASCTy=self._bits(d, o + 2, 6), subchannelId=self._bits(d, o + 8, 6),
                                           PS_flag=self._bits(d, o + 14, 1)))
            elif tmid == 3:
                self._bind(3, sid, i, dict(SCId=self._bits(d, o + 2, 12), PS_flag=self._bits(d, o + 14, 1),
                                           CAflag=self._bits(d, o + 15, 1)))
            o += 16
        return o // 8

    def _fig0_3(self, d, used):                                    # :433-453
        o = used * 8
        scid = self._bits(d, o, 12)
        for c in self.components:                                  # find_packetComponent (:1060-1072)
            if c["inUse"] and c["TMid"] == 3 and c["SCId"] == scid:
                c.update(subchannelId=self._bits(d, o + 24, 6), DSCTy=self._bits(d, o + 18, 6),
                         DGflag=self._bits(d, o + 16, 1), packetAddress=self._bits(d, o + 30, 10))
                break
        return used + 7

    def _label(self, d, off, charset):
        return charset_text([self._bits(d, off + 8 * i, 8) for i in range(16)], charset)

    def _fig1(self, d):                                            # :850-994
        charset = self._bits(d, 8, 4)
        oe = self._bits(d, 12, 1)
        ext = self._bits(d, 13, 3)
        if ext == 0:
            eid = self._bits(d, 16, 16)
            if charset <= 16 and not oe:
                name = self._label(d, 32, charset)
                if self.firstTime:
                    self.events.append(("E", eid, name))
                self.firstTime = False
        elif ext in (1, 5):
            sid = self._bits(d, 16, 16) if ext == 1 else self._bits(d, 16, 32)
            sid = sid - (1 << 32) if sid >= 1 << 31 else sid
            s = self._find_service(sid)
            if not s["hasName"] and charset <= 16:
                s["label"] += self._label(d, 32 if ext == 1 else 48, charset)
                if ext == 5:
                    s["label"] += charset_text(b" (data)\0", charset)
                else:
                    self.events.append(("S", s["label"]))
                s["hasName"] = True

    def _fig2(self, d):                                            # :998-1037
        charset = self._bits(d, 8, 4)
        if self._bits(d, 13, 3) == 5:
            sid = self._bits(d, 16, 32)
            sid = sid - (1 << 32) if sid >= 1 << 31 else sid
            s = self._find_service(sid)
            if not s["hasName"] and charset <= 16:
                s["label"] += self._label(d, 48, charset)
                s["hasName"] = True

    def _find_service(self, sid):                                  # :1041-1058
        for s in self.services:
            if s["inUse"] and s["serviceId"] == sid:
                return s
        for s in self.services:
            if not s["inUse"]:
                s.update(inUse=True, hasName=False, serviceId=sid)
                return s
        return self.services[0]

    def _bind(self, tmid, sid, compnr, fields):                    # :1077-1139
        s = self.services.index(self._find_service(sid))
        first = -1
        for i, c in enumerate(self.components):
            if not c["inUse"]:
                if first < 0:
                    first = i
                continue
            if c["service"] == s and c["componentNr"] == compnr:
                return
        c = self.components[first]
        c.update(fields)
        c.update(inUse=True, TMid=tmid, service=s, componentNr=compnr)

    def setupforNewFrame(self):                                    # :1142-1147
        for c in self.components:
            c["inUse"] = False

    def clearEnsemble(self):                                       # :1149-1163
        self.components = [dict(inUse=False, TMid=0, componentNr=0, service=-1, subchannelId=0, PS_flag=0,
                                ASCTy=0, SCId=0, CAflag=0, DSCTy=0, DGflag=0, packetAddress=0) for _ in range(64)]
        self.ficList = [dict(SubChId=0, StartAddr=0, Length=0, uepFlag=0, protLevel=0, BitRate=0, FEC_scheme=0)
                        for _ in range(64)]
        for s in self.services:                                    # language / programType survive
            s.update(inUse=False, serviceId=-1, label="")
        self.firstTime = True

    def labels(self):
        return [s["label"] for s in self.services if s["inUse"] and s["hasName"]]

    def _lookup(self, label, want):
        for s in self.services:                                    # :1197-1315
            if not s["inUse"] or not s["hasName"] or s["label"] != label:
                continue
            for c in self.components:
                if not c["inUse"] or self.services[c["service"]]["serviceId"] != s["serviceId"]:
                    continue
                if want == "kind":
                    if c["TMid"] == 3:
                        return self.PACKET
                    if c["TMid"] == 0:
                        return self.AUDIO
                    continue
                if c["TMid"] != (0 if want == "audio" else 3):
                    return None                                    # "fatal error, expected ..."
                f = self.ficList[c["subchannelId"]]
                if want == "audio":
                    return [c["subchannelId"], f["StartAddr"], f["uepFlag"], f["protLevel"], f["Length"],
                            f["BitRate"], c["ASCTy"], s["language"], s["programType"]]
                return [c["subchannelId"], f["StartAddr"], f["uepFlag"], f["protLevel"], c["DSCTy"], f["Length"],
                        f["BitRate"], f["FEC_scheme"], c["DGflag"], c["packetAddress"]]
        return self.UNKNOWN if want == "kind" else None

    def kindofService(self, label):
        return self._lookup(label, "kind")

    def dataforAudioService(self, label):
        return self._lookup(label, "audio")

    def dataforDataService(self, label):
        return self._lookup(label, "data")
