"""FIG parser (sdr-j-dab_amd/host/fib_processor.*) on FIBs built
field by field (tests/cpp/test_fib.cpp): sub-channel and service organisation,
packet components, FEC, programme type/language, labels (EBU Latin), and the
service lookups kindofService / dataforAudioService / dataforDataService with the
reference's loop bounds.  Host code only; parity unpinned (the reference class
needs Qt)."""
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_fib")


def test_fib_processor():
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "cpp", "Makefile"), EXE], check=True,
                   cwd=ROOT, timeout=300)
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout


# ---- the parser against the restatement of fib-processor.cpp on random FIBs ----------
DUMP = os.path.join(ROOT, "tests", "cpp", "build", "fib_dump")


class _Bits:
    def __init__(self):
        self.b = []

    def put(self, v, n):
        self.b += [(v >> (n - 1 - i)) & 1 for i in range(n)]
        return self

    def bytes(self):
        assert len(self.b) % 8 == 0
        return bytes(int("".join(map(str, self.b[i:i + 8])), 2) for i in range(0, len(self.b), 8))


def _fig(t, payload):
    assert len(payload) < 32
    return bytes([(t << 5) | len(payload)]) + payload


def _random_fig(rng, pools):
    """one well-formed FIG (header + payload) of a kind the parser reads, fields drawn
    from small pools so that services, components and sub-channels collide"""
    sids, scids, subs, labels = pools
    k = rng.integers(0, 12)
    if k == 0:                                                   # FIG 0/1, short / long entries
        b = _Bits().put(int(rng.integers(0, 2)), 1).put(0, 1).put(0, 1).put(1, 5)
        for _ in range(rng.integers(1, 4)):
            b.put(int(rng.choice(subs)), 6).put(int(rng.integers(0, 864)), 10)
            if rng.integers(0, 2):
                b.put(0, 1).put(0, 1).put(int(rng.integers(0, 64)), 6)
            else:
                b.put(1, 1).put(int(rng.integers(0, 3)), 3).put(int(rng.integers(0, 4)), 2)
                b.put(int(rng.integers(1, 1024)), 10)
        return _fig(0, b.bytes())
    if k in (1, 2):                                              # FIG 0/2, pd 0 / 1
        pd = int(k == 2)
        b = _Bits().put(0, 1).put(0, 1).put(pd, 1).put(2, 5)
        for _ in range(rng.integers(1, 3)):
            b.put(int(rng.choice(sids)) & (0xFFFFFFFF if pd else 0xFFFF), 32 if pd else 16)
            n = int(rng.integers(1, 4))
            b.put(0, 1).put(0, 3).put(n, 4)
            for _ in range(n):
                tm = int(rng.choice([0, 0, 3, 3, 1, 2]))
                b.put(tm, 2)
                if tm == 3:
                    b.put(int(rng.choice(scids)), 12)
                else:
                    b.put(int(rng.integers(0, 64)), 6).put(int(rng.choice(subs)), 6)
                b.put(int(rng.integers(0, 2)), 1).put(int(rng.integers(0, 2)), 1)
        return _fig(0, b.bytes())
    if k == 3:                                                   # FIG 0/3
        b = _Bits().put(0, 1).put(0, 1).put(0, 1).put(3, 5)
        for _ in range(rng.integers(1, 3)):
            b.put(int(rng.choice(scids)), 12).put(0, 3).put(int(rng.integers(0, 2)), 1).put(int(rng.integers(0, 2)), 1)
            b.put(0, 1).put(int(rng.integers(0, 64)), 6).put(int(rng.choice(subs)), 6)
            b.put(int(rng.integers(0, 1024)), 10).put(int(rng.integers(0, 65536)), 16)
        return _fig(0, b.bytes())
    if k == 4:                                                   # FIG 0/14
        b = _Bits().put(0, 1).put(0, 1).put(0, 1).put(14, 5)
        for _ in range(rng.integers(1, 5)):
            b.put(int(rng.choice(subs + [0, 0])), 6).put(int(rng.integers(0, 4)), 2)
        return _fig(0, b.bytes())
    if k == 5:                                                   # FIG 0/16
        b = _Bits().put(0, 1).put(0, 1).put(0, 1).put(16, 5)
        for _ in range(rng.integers(1, 3)):
            b.put(int(rng.choice(sids)) & 0xFFFF, 16).put(int(rng.integers(0, 65536)), 16).put(0, 40)
        return _fig(0, b.bytes())
    if k == 6:                                                   # FIG 0/17
        b = _Bits().put(0, 1).put(0, 1).put(0, 1).put(17, 5)
        for _ in range(rng.integers(1, 4)):
            lf, cc = int(rng.integers(0, 2)), int(rng.integers(0, 2))
            b.put(int(rng.choice(sids)) & 0xFFFF, 16).put(int(rng.integers(0, 2)), 1).put(0, 1).put(lf, 1).put(cc, 1)
            b.put(0, 4)
            if lf:
                b.put(int(rng.integers(0, 256)), 8)
            b.put(0, 3).put(int(rng.integers(0, 32)), 5)
            if cc:
                b.put(int(rng.integers(0, 256)), 8)
        return _fig(0, b.bytes())
    if k == 7:                                                   # an extension the lookups never read
        ext = int(rng.choice([0, 5, 8, 9, 10, 13, 18, 19, 21, 22]))
        return _fig(0, bytes([ext]) + bytes(rng.integers(0, 256, int(rng.integers(0, 6)), dtype=np.uint8)))
    lab = labels[rng.integers(0, len(labels))]
    cs = int(rng.choice([0, 0, 15, 1, 2]))                       # EBU, UTF-8, "other" values (EBU)
    if cs == 15 and max(lab) >= 0x80:                            # invalid UTF-8: Qt's replacement rules, unpinned
        cs = 0
    if k == 8:                                                   # FIG 1/0 ensemble label
        oe = int(rng.integers(0, 4) == 0)
        return _fig(1, bytes([(cs << 4) | (oe << 3) | 0]) + int(rng.choice(sids) & 0xFFFF).to_bytes(2, "big")
                    + lab + b"\xff\x00")
    if k in (9, 10):                                             # FIG 1/1, FIG 1/5
        if k == 9:
            return _fig(1, bytes([(cs << 4) | 1]) + int(rng.choice(sids) & 0xFFFF).to_bytes(2, "big") + lab
                        + b"\xff\x00")
        return _fig(1, bytes([(cs << 4) | 5]) + int(rng.choice(sids) & 0xFFFFFFFF).to_bytes(4, "big") + lab
                    + b"\x00\x00")
    return _fig(2, bytes([(cs << 4) | 5]) + int(rng.choice(sids) & 0xFFFFFFFF).to_bytes(4, "big") + lab
                + b"\x00\x00")                                   # FIG 2/5


def _random_fib(rng, pools):
    body = b""
    for _ in range(8):
        f = _random_fig(rng, pools)
        if len(body) + len(f) <= 30:
            body += f
    return body + b"\xff" * (30 - len(body)) + b"\x00\x00"


def test_fib_processor_matches_restatement_on_random_fibs():
    """dabgpu::fib_processor and oracle_py.FibProcessor (fib-processor.cpp restated:
    FIG 0/1, 0/2, 0/3, 0/14, 0/16, 0/17, 1/0, 1/1, 1/5, 2/5, the three lookups,
    clearEnsemble / setupforNewFrame) fed the same random well-formed FIBs: equal
    service labels in slot order, nameofEnsemble / addtoEnsemble events, and lookup
    answers for every label after every batch.  Parity against a restatement (the
    reference class needs Qt); includes the reference's quirks: FIG 0/14 applies to
    every entry through its never-set SubChId field, labels are taken once per
    service, language / programme type survive clearEnsemble, FIG 0/16 allocates
    service entries, the first named service with a label wins the lookups."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as orc
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "cpp", "Makefile"), DUMP], check=True,
                   cwd=ROOT, timeout=300)
    rng = np.random.default_rng(2024)
    base = [b"Radio One", b"Radio One", b"Jazz & Blues", b"News 24", b"\x80\x8e\xa9 Caf\x82",
            b"Sport$ ^~`", b"Data Svc", b"Ensemble A", b"With\x00NUL"]
    labels = [l.ljust(16, b" ")[:16] for l in base] + [b"Radio One       ", b"Jazz & Blues    "]
    for trial in range(6):
        sids = [int(x) for x in rng.integers(1, 0xFFFF, 6)] + [0xF0000000 + trial, 0x80001234]
        scids = [int(x) for x in rng.integers(0, 4096, 4)]
        subs = [int(x) for x in rng.integers(0, 64, 6)]
        pools = (sids, scids, subs, labels)
        ref = orc.FibProcessor()
        script, expect = [], []

        def queries():
            qs = sorted(set(ref.labels()) | {"nothing", "Radio One       "})
            for q in qs:
                h = q.encode("utf-8").hex()
                script.append("Q " + h)
                expect.append({"q": h, "kind": ref.kindofService(q), "audio": ref.dataforAudioService(q),
                               "data": ref.dataforDataService(q)})
            script.append("D")
            ev = [["E", e[1], e[2].encode("utf-8").hex()] if e[0] == "E" else ["S", e[1].encode("utf-8").hex()]
                  for e in ref.events]
            ref.events.clear()
            expect.append({"labels": [l.encode("utf-8").hex() for l in ref.labels()], "events": ev})

        for step in range(400):
            r = rng.integers(0, 100)
            if r == 0:
                script.append("C")
                ref.clearEnsemble()
            elif r == 1:
                script.append("N")
                ref.setupforNewFrame()
            else:
                fib = _random_fib(rng, pools)
                script.append("F " + fib.hex())
                ref.process_FIB([(fib[i >> 3] >> (7 - (i & 7))) & 1 for i in range(256)])
            if step % 50 == 49:
                queries()
        queries()
        out = subprocess.run([DUMP], input="\n".join(script) + "\n", capture_output=True, text=True, timeout=60)
        assert out.returncode == 0, out.stderr
        got = [json.loads(l) for l in out.stdout.splitlines()]
        assert len(got) == len(expect), (trial, len(got), len(expect))
        for i, (g, e) in enumerate(zip(got, expect)):
            assert g == e, (trial, i, g, e)
