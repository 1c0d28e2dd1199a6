"""Recorded IQ -> cf32 on the GPU (dabgpu_iq_convert) against the
reference readers' scaling: rawFiles::getSamples float(x - 128) / 128.0
(rawfiles.cpp:100-118) and libsndfile's sf_readf_float on PCM16, x / 32768
(wavfiles.cpp readBuffer).  Bit-exact (both are exact in float32).  End to end: an
ensemble written as an .sdr file and read back through the GPU conversion decodes
to the same FIC/MSC bits as the same samples converted on the host."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import dabamd
    c = dabamd.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("n_pairs", [1, 7, 8, 4099, 1 << 16])
def test_iq_convert_exact(ctx, n_pairs):
    import dabamd
    rng = np.random.default_rng(n_pairs)
    u8 = rng.integers(0, 256, 2 * n_pairs, dtype=np.uint8)
    s16 = rng.integers(-32768, 32768, 2 * n_pairs, dtype=np.int16)
    s16[:2] = (-32768, 32767)
    for fmt, src, want in ((dabamd.IQ_U8, u8, (u8.astype(np.float64) - 128) / 128.0),
                           (dabamd.IQ_S16, s16, s16.astype(np.float64) / 32768.0)):
        dsrc = ctx.put(src)
        dst = ctx.buf(8 * n_pairs)
        ctx.iq_convert(fmt, dsrc, n_pairs, dst)
        ctx.sync()
        got = dst.download(np.float32, 2 * n_pairs)
        assert np.array_equal(got, want.astype(np.float32)), fmt
        dsrc.free()
        dst.free()


def test_sdr_file_decodes_like_host_conversion(ctx, tmp_path):
    import dabamd
    from dabamd.synth import Ensemble
    subch = [(0, 96, 128, 3, 1, 0)]
    F, runs = 3, 2
    e = Ensemble(F * runs, subch=subch, snr_db=40.0)
    g = e.generate(5)
    x = g["iq"].astype(np.float64)
    gain = 0.5 * 32767 / np.abs(x).max()
    s16 = np.clip(np.rint(x * gain), -32768, 32767).astype(np.int16)
    p = str(tmp_path / "ens.sdr")
    dabamd.write_sdr(p, s16)
    dfile, n = ctx.load_iq_file(p, chunk_pairs=1 << 18)     # several chunks
    assert n == s16.size // 2
    dhost = ctx.put((s16.astype(np.float32) / 32768.0).astype(np.float32))
    subs = [dabamd.Subch(s[0], s[1], s[2], s[3], 0 if s[4] else 1, 0) for s in subch]
    res = []
    for d in (dfile, dhost):
        pipe = dabamd.Pipeline(ctx, 1, F, subs)
        pipe.acquire(d, n, [0], [n])
        out = [tuple(a.copy() for a in pipe.run(d, n, [n])) for _ in range(runs)]
        pipe.close()
        res.append(out)
    n_valid = 0
    for (fa, ca, ma, va), (fb, cb, mb, vb) in zip(*res):
        assert np.array_equal(fa, fb) and np.array_equal(ca, cb) and np.array_equal(va, vb)
        assert ca.all()
        for c in np.flatnonzero(va[0]):                     # CIFs past the de-interleaver warm-up
            assert np.array_equal(ma[0, c, 0, :24 * 128], mb[0, c, 0, :24 * 128]), c
            n_valid += 1
    assert n_valid == 4 * F * runs - 16
    dfile.free()
    dhost.free()
