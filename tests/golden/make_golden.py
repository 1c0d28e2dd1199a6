"""Generate golden vectors from the REFERENCE's own sources (oracle/_ref/libdabref.so,
compiled from /root/reference by oracle/Makefile: viterbi.cpp + spiral-sse.c,
deconvolve.cpp, protTables.cpp, reed-solomon.cpp, galois.cpp, firecode-checker.cpp,
mapper.cpp, phasetable.cpp).  Inputs are seeded synthetic data; outputs are the
reference's.  Run from the repo root:  python tests/golden/make_golden.py"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "sdr-j-dab_amd"))
import oracle_py  # noqa: E402
from dabamd.synth import conv_encode  # noqa: E402

P = oracle_py.P


def main():
    r = oracle_py.ref()
    if r is None:
        raise SystemExit("oracle/_ref/libdabref.so missing: make -f oracle/Makefile")
    rng = np.random.default_rng(20251015)
    out = {}
    # mapper (mapper.cpp:33-117) and PRS phases (phasetable.cpp:261-274)
    perm = np.zeros(1536, np.int16)
    r.ref_mapper(P(perm))
    out["mapper"] = perm
    ks = np.array(list(range(-768, 0)) + list(range(1, 769)), np.int32)
    out["phi_k"] = ks
    out["phi"] = np.array([r.ref_get_phi(int(k)) for k in ks], np.float32)
    pc = np.zeros((24, 32), np.int8)
    for i in range(24):
        row = np.zeros(32, np.int8)
        r.ref_pcode(i + 1, P(row))
        pc[i] = row
    out["pcodes"] = pc
    np.savez_compressed(os.path.join(HERE, "tables.npz"), **out)

    # Viterbi known answers (viterbi.cpp:225-242 + spiral-sse.c)
    vk = {}
    for nb in (768, 3072):
        rows, outs = [], []
        for i in range(6):
            bits = rng.integers(0, 2, nb).astype(np.uint8)
            coded = conv_encode(bits).astype(np.int32)
            sigma = [0, 80, 160, 240, 320, 400][i]
            soft = np.clip((2 * coded - 1) * 127 + rng.normal(0, sigma, coded.shape), -250, 250).astype(np.int16)
            o = np.zeros(nb, np.uint8)
            r.ref_viterbi(P(soft), nb, P(o))
            rows.append(soft)
            outs.append(o)
        vk[f"in_{nb}"] = np.stack(rows)
        vk[f"out_{nb}"] = np.stack(outs)
    np.savez_compressed(os.path.join(HERE, "viterbi_kat.npz"), **vk)

    # UEP / EEP depuncture + Viterbi (deconvolve.cpp:172-237, 325-366)
    cases = [(0, 128, 3), (0, 32, 5), (0, 64, 4), (0, 192, 2), (1, 64, 0o103), (1, 8, 0o102), (1, 96, 0o204)]
    frags = rng.integers(-127, 128, (len(cases), 20000)).astype(np.int16)
    mo = np.zeros((len(cases), 24 * 192), np.uint8)
    for i, (uf, br, pl) in enumerate(cases):
        o = np.zeros(24 * br, np.uint8)
        fn = r.ref_uep_deconvolve if uf == 0 else r.ref_eep_deconvolve
        fn(br, pl, P(frags[i]), 20000, P(o))
        mo[i, :24 * br] = o
    np.savez_compressed(os.path.join(HERE, "msc_kat.npz"), cases=np.array(cases, np.int32), frags=frags, out=mo)

    # RS(120,110) decode incl. failures (reed-solomon.cpp:129-229)
    n = 64
    cw = np.zeros((n, 120), np.uint8)
    dec = np.zeros((n, 110), np.uint8)
    ret = np.zeros(n, np.int16)
    for i in range(n):
        d = rng.integers(0, 256, 110).astype(np.uint8)
        c = np.zeros(120, np.uint8)
        r.ref_rs_enc(P(d), P(c))
        ne = i % 9
        pos = rng.choice(120, ne, replace=False)
        c[pos] ^= rng.integers(1, 256, ne).astype(np.uint8)
        o = np.zeros(110, np.uint8)
        ret[i] = C.c_int16(r.ref_rs_dec(P(c), P(o))).value
        cw[i], dec[i] = c, o
    np.savez_compressed(os.path.join(HERE, "rs_kat.npz"), cw=cw, dec=dec, ret=ret)

    # FIB CRC (dab-constants.h:310-340) and DAB+ fire code (firecode-checker.cpp:76-94)
    fibs = rng.integers(0, 2, (32, 256)).astype(np.uint8)
    crc = np.zeros(32, np.uint8)
    mut = fibs.copy()
    for i in range(32):
        crc[i] = r.ref_check_crc_bits(P(mut[i]), 256)
    fire = rng.integers(0, 256, (64, 11)).astype(np.uint8)
    fok = np.array([r.ref_firecode_check(P(fire[i])) for i in range(64)], np.uint8)
    np.savez_compressed(os.path.join(HERE, "crc_kat.npz"), fibs=fibs, crc=crc, mutated=mut, fire=fire, fire_ok=fok)
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
