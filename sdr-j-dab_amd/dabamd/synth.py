"""ctypes bindings of the synthetic DAB Mode-I transmitter (synth/dabsynth.h)."""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import SYNTH_PATH, DabError

_lib: Optional[C.CDLL] = None


class SynthSubch(C.Structure):
    _fields_ = [("startAddr", C.c_int16), ("length", C.c_int16), ("bitRate", C.c_int16),
                ("protLevel", C.c_int16), ("uep", C.c_int16), ("dabplus", C.c_int16), ("content", C.c_int16)]


MP2, PACKET, AU_MIX = 2, 3, 4   # SynthSubch.content (dabsynth.h DABSYNTH_MP2 / _PACKET / _AU_MIX)


class SynthCfg(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("pre_offset", C.c_int32), ("snr_db", C.c_float),
                ("cfo_hz", C.c_float), ("amplitude", C.c_float), ("n_subch", C.c_int32),
                ("subch", C.POINTER(SynthSubch)), ("figs", C.c_int32)]


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        try:
            _lib = C.CDLL(SYNTH_PATH)
        except OSError as e:
            raise DabError(f"{SYNTH_PATH}: {e}")
        _lib.dabsynth_stream_len.restype = C.c_int64
        _lib.dabsynth_stream_len.argtypes = [C.c_void_p]
        _lib.dabsynth_generate.argtypes = [C.c_void_p, C.c_uint64] + [C.c_void_p] * 5
        _lib.dabsynth_generate_many.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int] + [C.c_void_p] * 3
        _lib.dabsynth_generate_period.argtypes = [C.c_void_p, C.c_uint64, C.c_int] + [C.c_void_p] * 3
        _lib.dabsynth_period_many.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_void_p]
        _lib.dabsynth_conv_encode.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        _lib.dabsynth_puncture_msc.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        _lib.dabsynth_rs_encode.argtypes = [C.c_void_p, C.c_void_p]
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class Ensemble:
    """Synthetic ensemble generator.  subch: tuples (startAddr, length, bitRate,
    protLevel, uep, dabplus[, content]) -- uep=1 for UEP (uepFlag 0 in the reference);
    content MP2 / PACKET for MPEG layer II frames / packet-mode data groups; AU_MIX
    on a DAB+ subchannel cycles its superframes through the 4 (dacRate, SBR) layouts."""

    def __init__(self, n_frames: int, subch: Sequence[tuple] = (), pre_offset: int = 50000,
                 snr_db: float = 300.0, cfo_hz: float = 0.0, amplitude: float = 1.0, figs: bool = False):
        self.n_frames = n_frames
        self.subch = [SynthSubch(*s) for s in subch]
        self._arr = (SynthSubch * max(1, len(self.subch)))(*self.subch)
        self.cfg = SynthCfg(n_frames, pre_offset, snr_db, cfo_hz, amplitude, len(self.subch),
                            C.cast(self._arr, C.POINTER(SynthSubch)), int(figs))
        self.length = lib().dabsynth_stream_len(C.byref(self.cfg))
        self.maxbits = 24 * max([s.bitRate for s in self.subch] + [8])

    def generate(self, seed: int, truth: bool = True):
        iq = np.zeros(2 * self.length, dtype=np.float32)
        F, NS = self.n_frames, len(self.subch)
        fic = np.zeros((F, 4, 768), np.uint8) if truth else None
        msc = np.zeros((4 * F, NS, self.maxbits), np.uint8) if truth and NS else None
        coded = np.zeros((F, 75, 3072), np.uint8) if truth else None
        f0 = C.c_int64()
        rc = lib().dabsynth_generate(C.byref(self.cfg), seed, _p(iq), _p(fic), _p(msc), _p(coded), C.byref(f0))
        if rc:
            raise DabError(f"dabsynth_generate failed {rc}")
        return dict(iq=iq, fic=fic, msc=msc, coded=coded, frame0=f0.value)

    def generate_many(self, n_ens: int, seed0: int, threads: int = 8) -> np.ndarray:
        iq = np.zeros((n_ens, 2 * self.length), dtype=np.float32)
        rc = lib().dabsynth_generate_many(C.byref(self.cfg), seed0, n_ens, threads, _p(iq), None, None)
        if rc:
            raise DabError(f"dabsynth_generate_many failed {rc}")
        return iq

    # ---- cyclic streams (dabsynth_generate_period) ----------------------------------
    def generate_period(self, seed: int, period: int, truth: bool = True):
        """One period (`period` frames from frame 0's null) of a cyclic stream; truth
        arrays indexed by frame mod period / receiver CIF mod 4*period."""
        TF = 196608
        iq = np.zeros(2 * period * TF, dtype=np.float32)
        NS = len(self.subch)
        fic = np.zeros((period, 4, 768), np.uint8) if truth else None
        msc = np.zeros((4 * period, NS, self.maxbits), np.uint8) if truth and NS else None
        rc = lib().dabsynth_generate_period(C.byref(self.cfg), seed, period, _p(iq), _p(fic), _p(msc))
        if rc:
            raise DabError(f"dabsynth_generate_period failed {rc}")
        return dict(iq=iq, fic=fic, msc=msc, period=period)

    def period_many(self, n_ens: int, seed0: int, period: int, threads: int = 8) -> np.ndarray:
        iq = np.zeros((n_ens, 2 * period * 196608), dtype=np.float32)
        rc = lib().dabsynth_period_many(C.byref(self.cfg), seed0, period, n_ens, threads, _p(iq))
        if rc:
            raise DabError(f"dabsynth_period_many failed {rc}")
        return iq

    def period_offset(self) -> int:
        """stream sample of period sample 0 (frame 0's null start): TF - pre_offset"""
        return 196608 - self.cfg.pre_offset

    def stream_pieces(self, period: int, p0: int = 0, n: Optional[int] = None):
        """(stream sample, period sample, count) runs covering stream samples [p0, p0 + n)
        of the cyclic stream (default: the whole stream of this Ensemble's length)"""
        L = period * 196608
        n = self.length - p0 if n is None else n
        out, p, end = [], p0, p0 + n
        while p < end:
            q = (p - self.period_offset()) % L
            m = min(end - p, L - q)
            out.append((p, q, m))
            p += m
        return out

    def stream_from_period(self, period_iq: np.ndarray, period: int) -> np.ndarray:
        """the whole cyclic stream (this Ensemble's length) from one period"""
        iq = np.empty(2 * self.length, np.float32)
        for p, q, m in self.stream_pieces(period):
            iq[2 * p:2 * (p + m)] = period_iq[2 * q:2 * (q + m)]
        return iq


def conv_encode(bits: np.ndarray) -> np.ndarray:
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    out = np.zeros(4 * (len(bits) + 6), np.uint8)
    lib().dabsynth_conv_encode(_p(bits), len(bits), _p(out))
    return out
