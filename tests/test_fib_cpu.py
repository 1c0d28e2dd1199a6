"""FIG parser (sdr-j-dab_amd/host/fib_processor.*) on FIBs built
field by field (tests/cpp/test_fib.cpp): sub-channel and service organisation,
packet components, FEC, programme type/language, labels (EBU Latin), and the
service lookups kindofService / dataforAudioService / dataforDataService with the
reference's loop bounds.  Host code only; parity unpinned (the reference class
needs Qt)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_fib")


def test_fib_processor():
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "cpp", "Makefile"), EXE], check=True,
                   cwd=ROOT, timeout=300)
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout
