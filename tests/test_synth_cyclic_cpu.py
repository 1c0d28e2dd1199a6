"""The cyclic transmitter (dabsynth_generate_period): one period of P frames repeated
end to end must be a valid DAB stream everywhere -- the oracle (the reference CPU
path restated) decodes it across the period seams with every FIB CRC good, every
MSC codeword equal to the periodic truth and DAB+ superframes passing RS/fire
code/AU CRCs.  bench.py builds its streams this way (every rank's ensembles from one
period each), so this pins its checked step's truth indexing."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdr-j-dab_amd"), os.path.join(ROOT, "tests")]

import oracle_py as orc  # noqa: E402
from dabamd.synth import Ensemble  # noqa: E402

SUBCH = [(0, 48, 64, 0o103, 0, 2), (48, 96, 128, 3, 1, 0)]   # DAB+ EEP-3A (grid shifted 1 CIF), UEP-3


def _flip():
    m = np.zeros(768, np.uint8)
    for q in range(3):
        m[256 * q + 240:256 * q + 256] = 1
    return m


@pytest.mark.parametrize("cfo", [0.0, 1300.0])
def test_cyclic_stream_decodes_across_seams(cfo):
    P = 5                                                 # 4P = 20 CIFs: superframes tile the period
    nfr = 13 if cfo == 0 else 23
    f0 = 0 if cfo == 0 else 12                            # the AFC converges (reference: ~11 frames at 1.3 kHz)
    ens = Ensemble(nfr, subch=SUBCH, snr_db=30.0, cfo_hz=cfo)
    g = ens.generate_period(77, P, truth=True)
    iq = ens.stream_from_period(g["iq"], P)
    assert len(iq) == 2 * ens.length
    # the runs cover the stream exactly, and period sample 0 sits at TF - pre_offset
    pieces = ens.stream_pieces(P)
    assert pieces[0][0] == 0 and sum(m for _, _, m in pieces) == ens.length
    assert any(p == ens.period_offset() and q == 0 for p, q, _ in pieces)
    ref = orc.decode_stream(iq, nfr, SUBCH)
    n = ref["n"]
    assert n >= nfr - 1
    flip = _flip()
    assert ref["crc"][f0:n].all()
    for f in range(f0, n):
        for b in range(4):
            assert np.array_equal(ref["fic"][f, b] ^ flip, g["fic"][f % P, b]), (f, b)
    checked = 0
    for c in range(max(16, 4 * f0 + 16), 4 * n):           # past the de-interleaver warm-up (and the AFC)
        for k, sc in enumerate(SUBCH):
            nb = 24 * sc[2]
            assert np.array_equal(ref["msc"][c, k, :nb], g["msc"][c % (4 * P), k, :nb]), (c, k)
            checked += 1
    assert checked >= 2 * 20
    mp4 = orc.MP4(SUBCH[0][2])
    st = [mp4.add(ref["msc"][c, 0, :24 * SUBCH[0][2]])["status"] for c in range(max(16, 4 * f0 + 16), 4 * n)]
    # superframes decoded across the seams: once in sync, every superframe decodes (the
    # reference's blocksInBuffer cycle: four 0s then a 3), none fails its fire code or RS
    first = st.index(3)
    assert st.count(3) >= 4 and set(st[first:]) <= {0, 3}, st
    assert all(st[i] == 3 for i in range(first, len(st), 5)), st


def test_period_many_matches_single():
    ens = Ensemble(4, subch=SUBCH[1:], snr_db=25.0)
    many = ens.period_many(3, seed0=10, period=4, threads=3)
    for e in range(3):
        assert np.array_equal(many[e], ens.generate_period(10 + e, 4, truth=False)["iq"])


def test_cyclic_dabplus_needs_whole_superframes():
    ens = Ensemble(4, subch=SUBCH[:1])
    with pytest.raises(Exception):
        ens.generate_period(1, 6)                         # 24 CIFs: not a multiple of 5


def test_cyclic_refuses_packet_mode():
    """packet-mode content does not wrap at the period seam (a data group in flight, the
    continuity counter): generate_period refuses it rather than make an invalid stream"""
    from dabamd.synth import PACKET
    ens = Ensemble(4, subch=[(0, 24, 32, 0o103, 0, 0, PACKET)])
    with pytest.raises(Exception):
        ens.generate_period(1, 4)
