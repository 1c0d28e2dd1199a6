"""The C++ drop-in classes (sdr-j-dab_amd/host/dabgpu_dropin.h: viterbi,
uep_/eep_deconvolve, reedSolomon, phaseReference, ficHandler and the streaming
ensembleDecoder) on the GPU, checked by tests/cpp/test_dropin.cpp against the CPU
oracle and the transmitter's truth."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_dropin")


@pytest.mark.gpu
def test_cpp_dropin_classes():
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "cpp", "Makefile")], check=True)
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=600)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and "DROPIN OK" in r.stdout, r.stdout + r.stderr


def test_cpp_dropin_builds():
    """the drop-in library and its test link on a host without a GPU"""
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "cpp", "Makefile")], check=True)
    assert os.path.exists(EXE)
