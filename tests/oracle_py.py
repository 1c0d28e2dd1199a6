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


def ofdm_run(iq, max_frames, threshold=3, method=1):
    info = (FrameInfo * max_frames)()
    soft = np.zeros((max_frames, 75, 3072), np.int16)
    n = oracle().orc_ofdm_run(P(iq), C.c_int64(len(iq) // 2), threshold, method, max_frames, info, P(soft))
    return n, list(info)[:n], soft[:n]


def null_scan(iq, n, scan=True):
    """ofdmProcessor::run's null search over iq[0, n) with scanMode (ofdm-processor.cpp:259-338):
    (found, attempts, no_signal, pos) where the samples run out or a null's end is found"""
    a, ns, pos = C.c_int32(), C.c_int32(), C.c_int64()
    found = oracle().orc_null_scan(P(iq), C.c_int64(n), int(scan), C.byref(a), C.byref(ns), C.byref(pos))
    return found, a.value, ns.value, pos.value


def process_token(sym_ts, phase_ref):
    """returns ibits, softf; updates phase_ref (cf32 float array [4096]) in place"""
    ib = np.zeros(3072, np.int16)
    sf = np.zeros(3072, np.float32)
    oracle().orc_process_token(P(np.ascontiguousarray(sym_ts, np.float32)), P(phase_ref), P(ib), P(sf))
    return ib, sf


def process_block0(blk, flag=1, method=1):
    pr = np.zeros(4096, np.float32)
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


def fft(x):
    """the oracle's 2048-point FFT (double precision, rounded to float) of cf32 [4096]"""
    out = np.zeros(4096, np.float32)
    oracle().orc_fft2048(P(np.ascontiguousarray(x, np.float32)), P(out), 0)
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
