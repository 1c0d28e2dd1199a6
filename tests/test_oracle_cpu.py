"""CPU tests: the oracle against the golden vectors produced by the reference's
own sources, the oracle against the synthetic transmitter end to end, and
the C ABI library's exported surface.  No GPU needed."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle_py as orc

ROOT = orc.ROOT
GOLD = os.path.join(ROOT, "tests", "golden")
P = orc.P


def _g(name):
    return np.load(os.path.join(GOLD, name))


def test_tables_match_reference_fixtures():
    g = _g("tables.npz")
    perm = np.zeros(1536, np.int16)
    orc.oracle().orc_mapper(P(perm))
    assert np.array_equal(perm, g["mapper"])
    phi = np.array([orc.oracle().orc_get_phi(int(k)) for k in g["phi_k"]], np.float32)
    assert np.array_equal(phi, g["phi"])
    for i in range(24):
        row = np.zeros(32, np.int8)
        orc.oracle().orc_pcode(i + 1, P(row))
        assert np.array_equal(row, g["pcodes"][i])


def test_viterbi_matches_reference_fixtures():
    g = _g("viterbi_kat.npz")
    for nb in (768, 3072):
        for soft, want in zip(g[f"in_{nb}"], g[f"out_{nb}"]):
            assert np.array_equal(orc.viterbi(soft, nb), want)


def test_msc_deconvolve_matches_reference_fixtures():
    g = _g("msc_kat.npz")
    for (uf, br, pl), frag, want in zip(g["cases"], g["frags"], g["out"]):
        nb = 24 * int(br)
        got = orc.msc_deconvolve(1 if uf == 0 else 0, int(br), int(pl), frag) ^ orc.prbs(nb)
        assert np.array_equal(got, want[:nb]), (uf, br, pl)


def test_viterbi_int16_extremes_match_reference_fixtures():
    """viterbi.cpp:230-233 (int16_t temp = input + 127 wraps above 32640)"""
    g = _g("viterbi_kat.npz")
    for soft, want in zip(g["in_extreme"], g["out_extreme"]):
        assert np.array_equal(orc.viterbi(soft, 768), want)


def _profile_cases():
    g = _g("profiles_kat.npz")
    return g, [tuple(int(x) for x in c) for c in g["cases"]]


def test_every_profile_matches_reference_fixtures():
    """all 60 UEP rows, the unknown-profile fallback, EEP-A 1-4 (incl. 8 kbit/s level 2)
    and EEP-B 1-4: the oracle's depuncture + Viterbi against the reference's
    uep_/eep_deconvolve output (deconvolve.cpp:39-366)"""
    g, cases = _profile_cases()
    assert sum(1 for c in cases if c[0] == 0) >= 63 and sum(1 for c in cases if c[0] == 1) >= 40
    for i, (uf, br, pl) in enumerate(cases):
        nb = 24 * br
        frag = g["frags"][i, :g["used"][i]].astype(np.int16)
        got = orc.msc_deconvolve(1 if uf == 0 else 0, br, pl, frag) ^ orc.prbs(nb)
        assert np.array_equal(np.packbits(got), g["out"][i, :nb // 8]), (uf, br, pl)


def test_product_profiles_match_oracle():
    """the decoder's own depuncturing table (csrc/dab_tables.h, host make_profile) gives the
    oracle's (L_i, PI_i) segments for every fixture profile -- so the product table is
    pinned to the reference through the oracle, not only through GPU decodes"""
    import dabamd
    g, cases = _profile_cases()
    for i, (uf, br, pl) in enumerate(cases):
        nb, frag, segs, fallback = dabamd.subch_profile(dabamd.Subch(0, 0, br, pl, uf, 0))
        L, PI = np.zeros(4, np.int16), np.zeros(4, np.int16)
        if uf == 0:
            found = orc.oracle().orc_uep_profile(br, pl, P(L), P(PI))
            assert fallback == (found == 0), (br, pl)
        else:
            assert orc.oracle().orc_eep_profile(br, pl, P(L), P(PI))
        want = [(int(L[k]), int(PI[k])) for k in range(4) if L[k] > 0]
        assert nb == 24 * br and segs == want, (uf, br, pl, segs, want)
        assert frag == g["used"][i], (uf, br, pl, frag, g["used"][i])


def test_product_tables_match_reference_fixtures():
    """the product's PRS refTable and frequency de-interleaver (host-built, uploaded to
    the device as they are) against the reference's phasetable/mapper output"""
    import dabamd
    g = _g("tables.npz")
    assert np.array_equal(dabamd.host_table(dabamd.TABLE_PRS), g["ref_table"])
    assert np.array_equal(dabamd.host_table(dabamd.TABLE_MAPPER), g["mapper"])
    ra = np.zeros(18, np.float32)
    ref = g["ref_table"].astype(np.float64)
    # refArg[i] = arg(ref[i] conj(ref[i+1])) (ofdm-decoder.cpp:71-74), recomputed in float
    got = dabamd.host_table(dabamd.TABLE_REFARG)
    z = (g["ref_table"][:18, 0] + 1j * g["ref_table"][:18, 1]).astype(np.complex64) * \
        np.conj((g["ref_table"][1:19, 0] + 1j * g["ref_table"][1:19, 1]).astype(np.complex64))
    assert np.allclose(got, np.angle(z).astype(np.float32), atol=1e-6)


def test_nco_factor_tables_rebuild_oscillator_table_exactly():
    """the front-end kernels' NCO (three double factor tables, fma products, rounded to
    float) equals oscillatorTable (ofdm-processor.cpp:79-81) at all 2048000 indices; the
    product's own table too (tests/cpp/test_nco.c)"""
    import subprocess
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "cpp", "Makefile"),
                    os.path.join(ROOT, "tests", "cpp", "build", "test_nco")], check=True)
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "build", "test_nco")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_rs_matches_reference_fixtures():
    g = _g("rs_kat.npz")
    for cw, dec, ret in zip(g["cw"], g["dec"], g["ret"]):
        out = np.zeros(110, np.uint8)
        r = C.c_int16(orc.oracle().orc_rs_dec(P(np.ascontiguousarray(cw)), P(out))).value
        assert r == ret
        if r >= 0:
            assert np.array_equal(out, dec)


def test_crc_and_firecode_match_reference_fixtures():
    g = _g("crc_kat.npz")
    for fib, ok, mut in zip(g["fibs"], g["crc"], g["mutated"]):
        b = fib.copy()
        assert orc.oracle().orc_check_crc_bits(P(b), 256) == ok
        assert np.array_equal(b, mut)
    for x, ok in zip(g["fire"], g["fire_ok"]):
        assert orc.oracle().orc_firecode_check(P(np.ascontiguousarray(x))) == ok


def test_oracle_decodes_synthetic_ensemble():
    from dabamd.synth import Ensemble
    subch = [(0, 96, 128, 3, 1, 0), (96, 48, 64, 0o103, 0, 0)]
    e = Ensemble(5, subch=subch)
    g = e.generate(7)
    n, info, soft = orc.ofdm_run(g["iq"], 5)
    assert n == 5
    assert all(fi.start_index == 504 for fi in info[1:])
    assert np.array_equal((soft > 0).astype(np.uint8), g["coded"][:n])
    for f in range(n):
        fic = soft[f, 0:3].reshape(-1)
        for b in range(4):
            bits, ok = orc.fic_process(fic[2304 * b:2304 * (b + 1)])
            assert ok.all()
            want = g["fic"][f, b].copy()
            for q in range(3):
                want[256 * q + 240:256 * q + 256] ^= 1
            assert np.array_equal(bits, want)
    cifs = soft[:, 3:75].reshape(4 * n, -1)
    for k, (sa, ln, br, pl, uep, _) in enumerate(subch):
        frag = np.ascontiguousarray(cifs[:, sa * 64:(sa + ln) * 64])
        out = np.zeros((4 * n, 24 * br), np.uint8)
        assert orc.oracle().orc_msc_stream(uep, br, pl, ln * 64, 4 * n, P(frag), P(out)) == 0
        for c in range(16, 4 * n):
            assert np.array_equal(out[c], g["msc"][c, k, :24 * br])


def test_oracle_dabplus_superframe():
    """DAB+ superframes from the transmitter pass fire code, RS and AU CRCs in the oracle
    (mp4processor.cpp:107-230)."""
    from dabamd.synth import Ensemble
    subch = [(0, 48, 64, 0o103, 0, 1)]
    e = Ensemble(7, subch=subch)
    g = e.generate(3)
    bits = g["msc"][:, 0, :24 * 64]                  # CIF n carries encoder CIF n-15
    # encoder CIF e = n - 15 and superframes start at e = -19 + 5m -> n = -4 + 5m
    rs = 8
    good = 0
    for n0 in range(16, 4 * 7 - 4, 5):
        if (n0 + 4) % 5:
            continue
        by = np.packbits(bits[n0:n0 + 5].reshape(-1))
        assert orc.oracle().orc_firecode_check(P(by[:11]))
        out = np.zeros(110 * rs, np.uint8)
        nc = C.c_int16()
        na = C.c_int()
        au = np.zeros(8, np.int16)
        crc = np.zeros(8, np.uint8)
        ok = orc.oracle().orc_superframe(P(by), 0, 64, P(out), C.byref(nc), C.byref(na), P(au), P(crc))
        assert ok == 1 and nc.value == 0 and na.value == 4 and crc[:4].all()
        good += 1
    assert good >= 2


def test_oracle_superframe_au_layouts():
    """The transmitter's AU_MIX superframes (dacRate / SBR cycling through the four
    layouts of mp4processor.cpp:163-195: 4, 2, 6, 3 access units, where their AUs fit the
    reference's limits) decode in the oracle's superframe restatement with every AU CRC
    good, at RS widths 4 (32 kbit/s) to 24 (192 kbit/s: no 2-AU layout, its AUs would
    exceed 960 bytes)."""
    from dabamd.synth import AU_MIX, Ensemble
    for br, cus, pl in ((32, 32, 0o102), (64, 48, 0o103), (128, 96, 0o103), (192, 144, 0o103)):
        rs = br // 8
        e = Ensemble(9, subch=[(0, cus, br, pl, 0, 1, AU_MIX)], snr_db=300.0)
        g = e.generate(11)
        bits = g["msc"][:, 0, :24 * br]
        seen = []
        for n0 in range(16, 4 * 9 - 4):
            by = np.packbits(bits[n0:n0 + 5].reshape(-1))
            if not orc.oracle().orc_firecode_check(P(by[:11])):
                continue
            out = np.zeros(110 * rs, np.uint8)
            nc = C.c_int16()
            na = C.c_int()
            au = np.zeros(8, np.int16)
            crc = np.zeros(8, np.uint8)
            ok = orc.oracle().orc_superframe(P(by), 0, br, P(out), C.byref(nc), C.byref(na), P(au), P(crc))
            assert ok == 1 and nc.value == 0 and crc[:na.value].all(), (br, n0, na.value)
            seen.append(na.value)
        assert set(seen) == ({3, 4, 6} if br == 192 else {2, 3, 4, 6}), (br, seen)


def test_oracle_mp4_state_machine():
    """mp4Processor::addtoFrame (mp4processor.cpp:107-145): with the superframe grid
    shifted by 2 CIFs the fire code fails until the ring is aligned, then every
    fifth CIF completes a superframe whose bytes are the transmitted ones."""
    from dabamd.synth import Ensemble
    e = Ensemble(8, subch=[(0, 48, 64, 0o103, 0, 3)], snr_db=300.0)
    g = e.generate(5)
    m = orc.MP4(64)
    st = []
    for n in range(16, 32):
        r = m.add(g["msc"][n, 0, :24 * 64])
        st.append(r["status"])
        if r["status"] == 3:
            sf = np.packbits(g["msc"][n - 4:n + 1, 0, :24 * 64].reshape(-1))
            assert np.array_equal(r["out"], sf[:110 * 8])
            assert r["num_aus"] == 4 and r["au_crc"][:4].all() and r["n_corrected"] == 0
    assert st == [0, 0, 0, 0, 1, 1, 1, 3, 0, 0, 0, 0, 3, 0, 0, 0]


def test_abi_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "dabgpu.h")).read()
    names = set(re.findall(r"\b(dabgpu_[a-z0-9_]+)\s*\(", hdr))
    assert len(names) >= 25
    import dabamd
    lib = dabamd.lib()
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert lib.dabgpu_abi_version() == 7


def test_abi_fails_loudly_without_device():
    import dabamd
    if dabamd.lib().dabgpu_device_count() > 0:
        pytest.skip("device present")
    with pytest.raises(dabamd.DabError):
        dabamd.Context(0)
