"""The host MSC consumers of the drop-in (sdr-j-dab_amd/host/msc_consumers.cpp) against
restatements of the reference (tests/oracle_py.py): mp2Processor's MPEG layer II frame
synchroniser (mp2processor.cpp:572-629) and mscDatagroup's packet -> data group
assembly (msc-datagroup.cpp:221-339), on bit streams built here: frames and packets
with valid and corrupted CRCs, padding packets, foreign addresses, lost packets,
garbage between frames, the 24 kHz (MPEG-2) frame length.  No GPU needed; parity
unpinned beyond the restatement (the reference classes need Qt and kjmp2 / MOT)."""
import ctypes as C
import os
import subprocess

import numpy as np

import oracle_py as orc

ROOT = orc.ROOT
LIB = os.path.join(ROOT, "tests", "cpp", "build", "libconsumers.so")


def _lib():
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "cpp", "Makefile"), LIB], check=True)
    l = C.CDLL(LIB)
    l.cw_mp2_new.restype = l.cw_pa_new.restype = C.c_void_p
    for f in (l.cw_mp2_add, l.cw_pa_add):
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    l.cw_pa_crc_errors.argtypes = [C.c_void_p]
    l.cw_item.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
    return l


def _items(l, h, n=40000):
    out, i = [], 0
    buf = np.zeros(n, np.uint8)
    rate = C.c_int()
    while True:
        k = l.cw_item(h, i, orc.P(buf), n, C.byref(rate))
        if k < 0:
            return out
        out.append((bytes(buf[:k]), rate.value))
        i += 1


def _bits(byts):
    return [int(b) for b in np.unpackbits(np.frombuffer(bytes(byts), np.uint8))]


def test_mp2_frame_sync_matches_reference():
    rng = np.random.default_rng(3)
    br = 64
    stream = list(rng.integers(0, 2, 500))            # garbage before sync
    want = []
    for k in range(12):
        mpeg2 = k in (5, 6)                           # 24 kHz: header 0xF4, twice the length
        hdr = bytes([0xFF, 0xF4 if mpeg2 else 0xFC, (0x8 << 4) | (1 << 2)])
        n = 24 * br * (2 if mpeg2 else 1)
        body = bytes(hdr) + bytes(rng.integers(0, 256, n // 8 - 3, dtype=np.uint8))
        stream += _bits(body)
        if k == 8:
            stream += [0, 1, 0]                       # a slip: the synchroniser must recover
    bits = np.array(stream, np.uint8)
    o = orc.MP2(br)
    l = _lib()
    h = l.cw_mp2_new(br)
    for c in range(0, len(bits), 24 * br):            # CIF-sized pieces, like dabConcurrent's
        piece = np.ascontiguousarray(bits[c:c + 24 * br])
        o.add([int(x) for x in piece])
        l.cw_mp2_add(h, orc.P(piece), len(piece))
    got = _items(l, h)
    assert len(o.frames) >= 8
    assert got == o.frames


def _packet(rng, plen_code, fl, addr, payload, corrupt=False):
    nbytes = (plen_code + 1) * 24
    assert len(payload) <= nbytes - 5                 # 3 header bytes + 2 CRC bytes
    bits = [plen_code >> 1, plen_code & 1, 0, 0, fl >> 1, fl & 1]
    bits += [(addr >> (9 - i)) & 1 for i in range(10)] + [0]
    bits += [(len(payload) >> (6 - i)) & 1 for i in range(7)]
    data = _bits(payload)
    bits += data + [0] * (nbytes * 8 - 16 - len(bits) - len(data))
    reg = 0xFFFF                                       # CRC-CCITT, transmitted inverted
    for b in bits:
        top = (reg >> 15) & 1
        reg = (reg << 1) & 0xFFFF
        if top ^ b:
            reg ^= 0x1021
    bits += [((reg >> (15 - i)) & 1) ^ 1 for i in range(16)]
    if corrupt:
        bits[40] ^= 1
    return bits


def test_packet_datagroups_match_reference():
    rng = np.random.default_rng(9)
    br = 32                                            # 768 bits = 96 bytes per CIF
    pk = []
    seq = [(0, 3, 77, 10, False), (0, 0, 0, 0, False),                  # single, padding
           (0, 2, 77, 19, False), (0, 0, 77, 19, False), (0, 1, 77, 5, False),   # first, mid, last
           (0, 2, 77, 19, False), (0, 0, 77, 17, True), (0, 1, 77, 5, False),    # lost middle packet
           (0, 2, 99, 18, False), (0, 3, 99, 8, False),                  # another address: ignored
           (0, 2, 77, 12, False), (0, 2, 77, 12, False), (0, 1, 77, 3, False),   # restart within a series
           (1, 3, 77, 40, False), (0, 3, 77, 1, False), (0, 0, 0, 0, False)]
    for code, fl, addr, n, bad in seq:
        pk += _packet(rng, code, fl, addr, bytes(rng.integers(0, 256, n, dtype=np.uint8)), bad)
    cif = 24 * br
    pk += [0] * ((-len(pk)) % cif)
    bits = np.array(pk, np.uint8)
    o = orc.Datagroups(60, 0)
    l = _lib()
    h = l.cw_pa_new(60, 0)
    for c in range(0, len(bits), cif):
        piece = np.ascontiguousarray(bits[c:c + cif])
        o.add([int(x) for x in piece])
        l.cw_pa_add(h, orc.P(piece), len(piece))
    got = [list(b) for b, _ in _items(l, h)]
    assert len(o.groups) >= 4 and o.crc_errors >= 1
    assert got == o.groups
    assert l.cw_pa_crc_errors(h) == o.crc_errors


def test_transmitter_mp2_and_packet_subchannels():
    """The transmitter's MPEG layer II and packet-mode subchannels (dabsynth content
    MP2 / PACKET): the oracle's consumers find one frame per CIF and whole data groups
    with good CRCs in the transmitted bits, and the product's consumers agree."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sdr-j-dab_amd"))
    from dabamd.synth import Ensemble, MP2, PACKET
    sub = [(0, 96, 128, 0o103, 0, 0, MP2), (96, 24, 32, 0o103, 0, 0, PACKET)]
    ens = Ensemble(6, subch=sub)
    g = ens.generate(5)
    l = _lib()
    m, hm = orc.MP2(128), l.cw_mp2_new(128)
    d, hd = orc.Datagroups(60, 0), l.cw_pa_new(60, 0)
    for c in range(16, 24):
        fb = np.ascontiguousarray(g["msc"][c, 0, :24 * 128])
        pb = np.ascontiguousarray(g["msc"][c, 1, :24 * 32])
        assert bytes(np.packbits(fb)[:4]) == bytes([0xFF, 0xFD, 0x84, 0x04])
        m.add(fb)
        fc, pc = fb.copy(), pb.copy()                  # (the consumers invert CRC bits in place)
        l.cw_mp2_add(hm, orc.P(fc), len(fc))
        d.add(pb)
        l.cw_pa_add(hd, orc.P(pc), len(pc))
    assert len(m.frames) == 8 and all(r == 48000 for _, r in m.frames)
    assert [f for f, _ in m.frames] == [bytes(np.packbits(g["msc"][c, 0, :24 * 128])) for c in range(16, 24)]
    assert _items(l, hm) == m.frames
    assert d.crc_errors == 0 and len(d.groups) >= 2
    assert [list(x) for x, _ in _items(l, hd)] == d.groups
    assert l.cw_pa_crc_errors(hd) == 0
