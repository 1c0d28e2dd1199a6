"""dabamd -- Python mirror of the MI355X DAB Mode-I path (include/dabgpu.h).

Thin ctypes layer over lib/libdabgpu.so.  The functions mirror the
sdr-j-dab interfaces they replace (names and argument meaning follow the
reference; file:line in each docstring).  There is no CPU fallback: if the
HIP library or a gfx950 device is missing, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("DABGPU_LIB") or os.path.join(_PKG, "lib", "libdabgpu.so")   # env: A/B of builds (tools/)
SYNTH_PATH = os.path.join(_PKG, "lib", "libdabsynth.so")

TU, TS, TG, TNULL, TF, K, L = 2048, 2552, 504, 2656, 196608, 1536, 76
NSYM = 75
SYMBITS = 2 * K
CIF_BITS = 55296


class DabError(RuntimeError):
    pass


class Subch(C.Structure):
    """audiodata/packetdata subset (dab-constants.h:151-176)."""
    _fields_ = [("startAddr", C.c_int16), ("length", C.c_int16), ("bitRate", C.c_int16),
                ("protLevel", C.c_int16), ("uepFlag", C.c_int16), ("flags", C.c_int16)]


SUBCH_DABPLUS = 1   # Subch.flags: feed the DAB+ superframe layer
SUPERFRAME_DTYPE = np.dtype([("status", "i1"), ("num_aus", "i1"), ("n_corrected", "<i2"), ("au_start", "<i2", (7,)),
                             ("au_crc_ok", "u1"), ("reserved", "u1")])


class Superframe(C.Structure):
    """one CIF of one DAB+ subchannel through mp4Processor (mp4processor.cpp:107-292)"""
    _fields_ = [("status", C.c_int8), ("num_aus", C.c_int8), ("n_corrected", C.c_int16),
                ("au_start", C.c_int16 * 7), ("au_crc_ok", C.c_uint8), ("reserved", C.c_uint8)]


class Frame(C.Structure):
    _fields_ = [("iq_base", C.c_int64), ("n_samples", C.c_int64), ("window", C.c_int64), ("block0", C.c_int64),
                ("lp_window", C.c_int32), ("phase_a", C.c_int32), ("lp_data", C.c_int32),
                ("phase_b", C.c_int32), ("out_slot", C.c_int32), ("flags", C.c_int32)]


class PipeCfg(C.Structure):
    _fields_ = [("n_streams", C.c_int32), ("n_frames", C.c_int32), ("n_subch", C.c_int32),
                ("threshold", C.c_int16), ("freq_sync_method", C.c_int16), ("subch", C.POINTER(Subch))]


class StreamState(C.Structure):
    _fields_ = [("next_pos", C.c_int64), ("local_phase", C.c_int32), ("coarse", C.c_int32),
                ("fine", C.c_int16), ("f2correction", C.c_int16), ("prev1", C.c_int16), ("prev2", C.c_int16),
                ("synced", C.c_int32), ("cif_count", C.c_int64), ("last_start_index", C.c_int32),
                ("resyncs", C.c_int32), ("acquisitions", C.c_int32), ("attempts", C.c_int32),
                ("no_signal", C.c_int32), ("frames_run", C.c_int32), ("acquiring", C.c_int32)]


class FrameInfo(C.Structure):
    """dabgpu_frame_info: per-frame observables of the last run (ofdm-processor.cpp:344-446,
    ofdm-decoder.cpp:93-97)"""
    _fields_ = [("window", C.c_int64), ("start_index", C.c_int32), ("coarse", C.c_int32), ("fine", C.c_int16),
                ("correction", C.c_int16), ("snr", C.c_int16), ("committed", C.c_int16)]


CTL_RESET, CTL_COARSE_ON, CTL_COARSE_OFF, CTL_SCAN_ON, CTL_SCAN_OFF, CTL_RESYNC = 1, 2, 3, 4, 5, 6
CTL_ACQ_ASYNC, CTL_ACQ_SYNC, CTL_INJECT_BOUNDS = 7, 8, 9
PACK_MSC, PACK_FIC = 1, 2          # dabgpu_pipe_set_packed mask


_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Load libdabgpu.so (raises if it is missing: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DabError(f"{LIB_PATH} not built (run __graft_entry__.build())")
        l = C.CDLL(LIB_PATH)
        vp, i32, i64, sz = C.c_void_p, C.c_int, C.c_int64, C.c_size_t
        sig = {
            "dabgpu_abi_version": ([], i32), "dabgpu_last_error": ([], C.c_char_p),
            "dabgpu_host_table": ([i32, vp, sz], i32),
            "dabgpu_subch_profile": ([vp, vp, vp, vp, vp, vp], i32),
            "dabgpu_device_count": ([], i32), "dabgpu_ctx_create": ([i32, C.POINTER(vp)], i32),
            "dabgpu_ctx_destroy": ([vp], i32), "dabgpu_sync": ([vp], i32),
            "dabgpu_alloc": ([vp, sz, C.POINTER(vp)], i32), "dabgpu_free": ([vp, vp], i32),
            "dabgpu_memcpy_h2d": ([vp, vp, vp, sz], i32), "dabgpu_memcpy_d2h": ([vp, vp, vp, sz], i32),
            "dabgpu_memset_d": ([vp, vp, i32, sz], i32),
            "dabgpu_memcpy_d2d": ([vp, vp, vp, sz], i32),
            "dabgpu_ofdm_symbol": ([vp, vp, i32, vp, vp], i32),
            "dabgpu_get_snr": ([vp, vp, vp], i32),
            "dabgpu_nco_eval": ([vp, i32, i32, vp], i32),
            "dabgpu_ofdm_demod_mix": ([vp, vp, i32, vp, i32, i32, C.c_int16, vp, vp, vp, vp], i32),
            "dabgpu_pipe_set_iq_format": ([vp, i32], i32),
            "dabgpu_pipe_acquire_wait": ([vp], i32),
            "dabgpu_pipe_set_display_token": ([vp, i32], i32),
            "dabgpu_iq_convert": ([vp, i32, vp, i64, vp], i32),
            "dabgpu_event_record": ([vp, i32], i32),
            "dabgpu_kernel_errors": ([vp], i32),
            "dabgpu_event_elapsed": ([vp, i32, i32, C.POINTER(C.c_float)], i32),
            "dabgpu_prs_sync": ([vp, vp, vp, i32, C.c_int16, vp, vp, vp], i32),
            "dabgpu_block0": ([vp, vp, vp, i32, i32, vp, vp], i32),
            "dabgpu_ofdm_demod": ([vp, vp, vp, i32, vp, vp, vp], i32),
            "dabgpu_ofdm_sync_demod": ([vp, vp, vp, i32, C.c_int16, vp, vp, vp, vp, vp], i32),
            "dabgpu_viterbi": ([vp, vp, i32, i32, vp], i32),
            "dabgpu_fic_decode": ([vp, vp, i32, vp, vp], i32),
            "dabgpu_fic_decode_frames": ([vp, vp, vp, i32, vp, vp], i32),
            "dabgpu_msc_deconvolve": ([vp, vp, i64, vp, i32, vp, i64], i32),
            "dabgpu_rs_decode": ([vp, vp, i32, vp, vp], i32),
            "dabgpu_pipe_dabplus": ([vp, vp, C.c_int32, vp], i32),
            "dabgpu_pipe_sync": ([vp], i32),
            "dabgpu_pipe_create": ([vp, vp, C.POINTER(vp)], i32), "dabgpu_pipe_destroy": ([vp], i32),
            "dabgpu_pipe_acquire": ([vp, vp, i64, vp, vp], i32),
            "dabgpu_pipe_run": ([vp, vp, i64, vp, vp, vp, vp, C.c_int32, vp], i32),
            "dabgpu_pipe_state": ([vp, i32, vp], i32),
            "dabgpu_pipe_frame_info": ([vp, vp], i32),
            "dabgpu_pipe_control": ([vp, i32, i32], i32),
            "dabgpu_pipe_softbits": ([vp, C.POINTER(vp), C.POINTER(C.c_int32)], i32),
            "dabgpu_pipe_set_dabplus_compact": ([vp, i32], i32),
            "dabgpu_pipe_frame_slot": ([vp, i32, C.POINTER(C.c_int32)], i32),
            "dabgpu_pipe_frames": ([vp, vp, vp], i32),
            "dabgpu_pipe_set_display": ([vp, i32], i32),
            "dabgpu_pipe_set_packed": ([vp, i32], i32),
            "dabgpu_pipe_fetch": ([vp, vp, vp, sz], i32),
            "dabgpu_host_alloc": ([vp, sz, C.POINTER(vp)], i32),
            "dabgpu_host_free": ([vp, vp], i32),
            "dabgpu_pipe_iq_display": ([vp, i32, i32, vp], i32),
            "dabgpu_pipe_set_profiling": ([vp, i32], i32),
            "dabgpu_pipe_timing": ([vp, vp, vp], i32),
        }
        for name, (args, res) in sig.items():
            try:
                f = getattr(l, name)
            except AttributeError:
                if "DABGPU_LIB" in os.environ:           # an older A/B build (tools/): calls to it raise
                    continue
                raise
            f.argtypes, f.restype = args, res
        _lib = l
    return _lib


def _chk(rc: int, what: str) -> None:
    if rc != 0:
        raise DabError(f"{what} failed ({rc}): {lib().dabgpu_last_error().decode()}")


def _p(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


IQ_F32, IQ_U8, IQ_S16 = 0, 1, 2   # sample formats (dabgpu_iq_convert, dabgpu_pipe_set_iq_format)
TABLE_PRS, TABLE_MAPPER, TABLE_REFARG, TABLE_OSC, TABLE_NCO = 1, 2, 3, 4, 5


def host_table(which: int) -> np.ndarray:
    """the product's host-built tables (dabgpu_host_table; no device needed)"""
    shape, dt = {TABLE_PRS: ((2048, 2), np.float32), TABLE_MAPPER: (1536, np.int16),
                 TABLE_REFARG: (18, np.float32), TABLE_OSC: ((2048000, 2), np.float32),
                 TABLE_NCO: ((384, 2), np.float64)}[which]
    out = np.zeros(shape, dt)
    _chk(lib().dabgpu_host_table(which, _p(out), out.nbytes), "dabgpu_host_table")
    return out


def subch_profile(sub: "Subch"):
    """(nbits, fragment size, [(L_i, PI_i)...], fallback) of the decoder's depuncturing
    profile for a subchannel (dabgpu_subch_profile)"""
    nb, fr, ns = C.c_int32(), C.c_int32(), C.c_int32()
    L, PI = np.zeros(4, np.int32), np.zeros(4, np.int32)
    rc = lib().dabgpu_subch_profile(C.byref(sub), C.byref(nb), C.byref(fr), C.byref(ns), _p(L), _p(PI))
    if rc < 0:
        _chk(rc, "dabgpu_subch_profile")
    return nb.value, fr.value, [(int(L[k]), int(PI[k])) for k in range(ns.value)], rc == 1


def read_raw(path: str) -> np.ndarray:
    """.raw recording (rawfiles.cpp): interleaved unsigned 8-bit I/Q, no header.
    Returns the bytes memory-mapped (an odd trailing byte is dropped)."""
    a = np.memmap(path, dtype=np.uint8, mode="r")
    return a[: a.size & ~1]


def read_sdr(path: str) -> np.ndarray:
    """.sdr recording (wavfiles.cpp:56-69): a WAV file with 2 channels (I, Q) of
    PCM16 at 2048000 samples/s.  Returns the interleaved int16 samples
    memory-mapped; raises ValueError for any other WAV layout, as the reference
    refuses it ("This is not a recorded dab file")."""
    import struct
    with open(path, "rb") as f:
        head = f.read(12)
        if len(head) < 12 or head[:4] != b"RIFF" or head[8:12] != b"WAVE":
            raise ValueError(f"{path}: not a RIFF/WAVE file")
        fmt = None
        off = 12
        while True:
            ck = f.read(8)
            if len(ck) < 8:
                raise ValueError(f"{path}: no data chunk")
            cid, n = ck[:4], struct.unpack("<I", ck[4:])[0]
            off += 8
            if cid == b"fmt ":
                b = f.read(n)
                tag, ch, rate, _, _, bits = struct.unpack("<HHIIHH", b[:16])
                if tag == 0xFFFE and n >= 26:              # WAVE_FORMAT_EXTENSIBLE: subformat GUID
                    tag = struct.unpack("<H", b[24:26])[0]
                fmt = (tag, ch, rate, bits)
            elif cid == b"data":
                if fmt is None:
                    raise ValueError(f"{path}: data before fmt chunk")
                if fmt != (1, 2, 2048000, 16):
                    raise ValueError(f"{path}: not a recorded DAB file (format/channels/rate/bits {fmt}); "
                                     "need PCM16, 2 channels, 2048000 Hz")
                size = os.path.getsize(path)
                n = min(n, size - off) & ~3
                return np.memmap(path, dtype="<i2", mode="r", offset=off, shape=(n // 2,))
            else:
                f.seek(n + (n & 1), 1)
            off += n + (n & 1)


def write_sdr(path: str, iq_s16: np.ndarray) -> None:
    """write interleaved int16 I/Q as an .sdr WAV (2 channels, PCM16, 2048000 Hz):
    the recording format of gui.cpp:880-883"""
    import wave
    with wave.open(path, "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(2048000)
        w.writeframes(np.ascontiguousarray(iq_s16, dtype="<i2").tobytes())


class DevBuf:
    """HBM buffer owned by a Context."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx, self.nbytes = ctx, int(nbytes)
        p = C.c_void_p()
        _chk(lib().dabgpu_alloc(ctx.h, max(self.nbytes, 16), C.byref(p)), "dabgpu_alloc")
        self.ptr = p

    def upload(self, a: np.ndarray) -> "DevBuf":
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        _chk(lib().dabgpu_memcpy_h2d(self.ctx.h, self.ptr, _p(a), a.nbytes), "h2d")
        return self

    def upload_at(self, a: np.ndarray, offset: int) -> "DevBuf":
        """copy `a` to byte `offset` of the buffer"""
        a = np.ascontiguousarray(a)
        assert offset >= 0 and offset + a.nbytes <= self.nbytes
        _chk(lib().dabgpu_memcpy_h2d(self.ctx.h, C.c_void_p(self.ptr.value + offset), _p(a), a.nbytes), "h2d")
        return self

    def download(self, dtype, shape) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        assert out.nbytes <= self.nbytes
        _chk(lib().dabgpu_memcpy_d2h(self.ctx.h, _p(out), self.ptr, out.nbytes), "d2h")
        return out

    def zero(self) -> "DevBuf":
        _chk(lib().dabgpu_memset_d(self.ctx.h, self.ptr, 0, self.nbytes), "memset")
        return self

    def free(self) -> None:
        if self.ptr:
            lib().dabgpu_free(self.ctx.h, self.ptr)
            self.ptr = None


class HostBuf:
    """page-locked host memory (dabgpu_host_alloc): the target of Pipeline.fetch"""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx, self.nbytes = ctx, int(nbytes)
        p = C.c_void_p()
        _chk(lib().dabgpu_host_alloc(ctx.h, max(self.nbytes, 16), C.byref(p)), "dabgpu_host_alloc")
        self.ptr = p

    def view(self, dtype, shape, offset: int = 0) -> np.ndarray:
        """a numpy view of the memory (valid until free)"""
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        assert offset + n <= self.nbytes
        raw = (C.c_uint8 * n).from_address(self.ptr.value + offset)
        return np.frombuffer(raw, dtype=dtype).reshape(shape)

    def free(self) -> None:
        if self.ptr:
            lib().dabgpu_host_free(self.ctx.h, self.ptr)
            self.ptr = None


class Context:
    """One HIP device + stream (dabgpu_ctx)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _chk(lib().dabgpu_ctx_create(device, C.byref(h)), "dabgpu_ctx_create")
        self.h = h

    def buf(self, nbytes: int) -> DevBuf:
        return DevBuf(self, nbytes)

    def put(self, a: np.ndarray) -> DevBuf:
        a = np.ascontiguousarray(a)
        return DevBuf(self, a.nbytes).upload(a)

    def sync(self) -> None:
        _chk(lib().dabgpu_sync(self.h), "sync")

    def iq_convert(self, fmt: int, src: "DevBuf", n_pairs: int, dst: "DevBuf", src_off: int = 0,
                   dst_off: int = 0) -> None:
        """dabgpu_iq_convert: recorded samples (IQ_U8 / IQ_S16) in src -> cf32 in dst"""
        _chk(lib().dabgpu_iq_convert(self.h, fmt, C.c_void_p(src.ptr.value + src_off), n_pairs,
                                     C.c_void_p(dst.ptr.value + dst_off)), "dabgpu_iq_convert")

    def load_iq_file(self, path: str, max_pairs: Optional[int] = None, chunk_pairs: int = 1 << 25):
        """Read a .raw (u8) or .sdr (WAV PCM16) recording into HBM as interleaved cf32,
        converting on the GPU; streamed in chunks (host memory stays at one chunk).
        Returns (DevBuf, n_pairs)."""
        if path.endswith(".raw"):
            src, fmt, w = read_raw(path), IQ_U8, 1
        else:
            src, fmt, w = read_sdr(path), IQ_S16, 2
        n = src.size // 2
        if max_pairs is not None:
            n = min(n, int(max_pairs))
        dst = self.buf(max(8 * n, 16))
        stage = self.buf(2 * w * min(n, chunk_pairs) + 16)
        try:
            for p0 in range(0, n, chunk_pairs):
                m = min(chunk_pairs, n - p0)
                stage.upload(np.ascontiguousarray(src[2 * p0: 2 * (p0 + m)]))
                self.iq_convert(fmt, stage, m, dst, dst_off=8 * p0)
                self.sync()
        finally:
            stage.free()
        return dst, n

    def load_recording(self, path: str, max_pairs: Optional[int] = None, chunk_pairs: int = 1 << 25):
        """Read a .raw (u8) or .sdr (WAV PCM16) recording into HBM as the file holds it
        (2 or 4 bytes per I/Q pair, a quarter / half of cf32): the pipeline converts it in
        its kernels' loads (Pipeline.set_iq_format(fmt), exactly as the reference's readers
        do, rawfiles.cpp:115-117 / wavfiles.cpp:172).  Streamed in chunks from the
        memory-mapped file.  Returns (DevBuf, n_pairs, fmt)."""
        if path.endswith(".raw"):
            src, fmt, w = read_raw(path), IQ_U8, 1
        else:
            src, fmt, w = read_sdr(path), IQ_S16, 2
        n = src.size // 2
        if max_pairs is not None:
            n = min(n, int(max_pairs))
        dst = self.buf(max(2 * w * n, 16))
        for p0 in range(0, n, chunk_pairs):
            m = min(chunk_pairs, n - p0)
            dst.upload_at(np.ascontiguousarray(src[2 * p0: 2 * (p0 + m)]), 2 * w * p0)
        return dst, n, fmt

    def check(self) -> None:
        """raise if a kernel refused out-of-bounds work since the last check"""
        _chk(lib().dabgpu_kernel_errors(self.h), "kernel bounds check")

    def close(self) -> None:
        if self.h:
            lib().dabgpu_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- operators mirroring the reference interfaces -------------------------
    def viterbi(self, soft: np.ndarray, nbits: int) -> np.ndarray:
        """viterbi::deconvolve (viterbi.cpp:225-242) for each row of soft [n, 4*(nbits+6)]."""
        soft = np.ascontiguousarray(soft, dtype=np.int16).reshape(-1, 4 * (nbits + 6))
        n = soft.shape[0]
        din, dout = self.put(soft), self.buf(n * nbits)
        try:
            _chk(lib().dabgpu_viterbi(self.h, din.ptr, n, nbits, dout.ptr), "dabgpu_viterbi")
            r = dout.download(np.uint8, (n, nbits))
            self.check()
            return r
        finally:
            din.free(); dout.free()

    def fic_process(self, blocks: np.ndarray):
        """ficHandler::process_ficInput (fic-handler.cpp:241-321) for [n, 2304] soft bits.
        Returns (bits [n,768] after energy dispersal and the CRC check's inversion, crc_ok [n,3])."""
        blocks = np.ascontiguousarray(blocks, dtype=np.int16).reshape(-1, 2304)
        n = blocks.shape[0]
        din, db, dc = self.put(blocks), self.buf(n * 768), self.buf(n * 3)
        try:
            _chk(lib().dabgpu_fic_decode(self.h, din.ptr, n, db.ptr, dc.ptr), "dabgpu_fic_decode")
            return db.download(np.uint8, (n, 768)), dc.download(np.uint8, (n, 3))
        finally:
            din.free(); db.free(); dc.free()

    def msc_deconvolve(self, frags: np.ndarray, subch: Sequence[Subch]) -> list:
        """uep_/eep_deconvolve::deconvolve + energy dispersal (deconvolve.cpp:172,325;
        dab-concurrent.cpp:183-190): one already de-interleaved fragment per row."""
        frags = np.ascontiguousarray(frags, dtype=np.int16)
        n, stride = frags.shape
        arr = (Subch * n)(*subch)
        maxbits = max(24 * s.bitRate for s in subch)
        din, dout = self.put(frags), self.buf(n * maxbits)
        try:
            _chk(lib().dabgpu_msc_deconvolve(self.h, din.ptr, stride, C.cast(arr, C.c_void_p), n, dout.ptr, maxbits),
                 "dabgpu_msc_deconvolve")
            out = dout.download(np.uint8, (n, maxbits))
            return [out[i, :24 * subch[i].bitRate] for i in range(n)]
        finally:
            din.free(); dout.free()

    def rs_decode(self, cw: np.ndarray):
        """reedSolomon::dec(rsIn, rsOut, 135) per row (reed-solomon.cpp:129-141):
        [n, 120] bytes -> ([n, 110] corrected bytes, [n] symbols corrected or -1)."""
        cw = np.ascontiguousarray(cw, dtype=np.uint8)
        n = cw.shape[0]
        din, dout, dr = self.put(cw), self.buf(max(1, 110 * n)), self.buf(max(2, 2 * n))
        try:
            _chk(lib().dabgpu_rs_decode(self.h, din.ptr, n, dout.ptr, dr.ptr), "dabgpu_rs_decode")
            return dout.download(np.uint8, (n, 110)), dr.download(np.int16, n)
        finally:
            din.free(); dout.free(); dr.free()

    def prs_sync(self, iq: DevBuf, frames: Sequence[Frame], level: int = 3):
        """phaseReference::findIndex (phasereference.cpp:60-88) per frame window."""
        n = len(frames)
        fa = (Frame * n)(*frames)
        dfr = DevBuf(self, C.sizeof(fa)).upload(np.frombuffer(fa, dtype=np.uint8))
        dsi, dmx, dsm = self.buf(4 * n), self.buf(4 * n), self.buf(4 * n)
        try:
            _chk(lib().dabgpu_prs_sync(self.h, iq.ptr, dfr.ptr, n, level, dsi.ptr, dmx.ptr, dsm.ptr), "prs_sync")
            r = (dsi.download(np.int32, n), dmx.download(np.float32, n), dsm.download(np.float32, n))
            self.check()
            return r
        finally:
            for b in (dfr, dsi, dmx, dsm):
                b.free()

    def block0(self, iq: DevBuf, frames: Sequence[Frame], method: int = 1, with_snr: bool = False):
        """ofdmDecoder::processBlock_0 (ofdm-decoder.cpp:85-162): coarse offset of
        freqSyncMethod `method` (frames with flags & 1), and get_snr when with_snr."""
        n = len(frames)
        fa = (Frame * n)(*frames)
        dfr = DevBuf(self, C.sizeof(fa)).upload(np.frombuffer(fa, dtype=np.uint8))
        dc, ds = self.buf(2 * n), self.buf(2 * n)
        try:
            _chk(lib().dabgpu_block0(self.h, iq.ptr, dfr.ptr, n, method, dc.ptr, ds.ptr), "block0")
            r = dc.download(np.int16, n)
            snr = ds.download(np.int16, n)
            self.check()
            return (r, snr) if with_snr else r
        finally:
            dfr.free(); dc.free(); ds.free()

    def demod(self, iq: DevBuf, frames: Sequence[Frame], with_float: bool = False):
        """ofdmDecoder::processToken for symbols 1..75 (ofdm-decoder.cpp:167-190).
        Frame i must have out_slot == i.  Returns (ibits [n,75,3072], softf or None, freqcorr [n] complex)."""
        n = len(frames)
        fa = (Frame * n)(*frames)
        dfr = DevBuf(self, C.sizeof(fa)).upload(np.frombuffer(fa, dtype=np.uint8))
        ds = self.buf(2 * n * NSYM * SYMBITS)
        df = self.buf(4 * n * NSYM * SYMBITS) if with_float else None
        dfc = self.buf(8 * n)
        try:
            _chk(lib().dabgpu_ofdm_demod(self.h, iq.ptr, dfr.ptr, n, ds.ptr, df.ptr if df else None, dfc.ptr),
                 "ofdm_demod")
            soft = ds.download(np.int16, (n, NSYM, SYMBITS))
            softf = df.download(np.float32, (n, NSYM, SYMBITS)) if df else None
            fc = dfc.download(np.float32, (n, 2))
            self.check()
            return soft, softf, fc[:, 0] + 1j * fc[:, 1]
        finally:
            for b in (dfr, ds, df, dfc):
                if b is not None:
                    b.free()


    def demod_mix(self, iq: DevBuf, frames: Sequence[Frame], chunks: int = 1, fmt: int = None, level: int = 3,
                  with_spec: bool = False):
        """dabgpu_ofdm_demod_mix: the fused demod's NCO-mixed FFT input of every data
        symbol, float32 [n, 75, 2048, 2] (samples [T_g, T_s) of symbol l after getSamples'
        NCO), and the soft bits; `chunks` workgroups per frame.
        fmt None: the operator form (cf32 in, frames give block0; int16 soft bits [n, 75, 3072]).
        fmt IQ_F32 / IQ_S16 / IQ_U8: the pipeline's instantiation (findIndex on each frame's
        window, samples read in that format, RING8 soft bytes [n, 75, 3072] u8); the start
        indices are returned too.  Returns (mix, soft) -- (mix, soft, start_index) with fmt --
        and the FFT output [n, 75, 2048] complex64 (natural bins) last when with_spec."""
        n = len(frames)
        fa = (Frame * n)(*frames)
        dfr = DevBuf(self, C.sizeof(fa)).upload(np.frombuffer(fa, dtype=np.uint8))
        dm = self.buf(8 * n * NSYM * 2048)
        dp = self.buf(8 * n * NSYM * 2048)
        sync = fmt is not None
        ds = self.buf((1 if sync else 2) * n * NSYM * SYMBITS)
        dsi = self.buf(4 * n) if sync else None
        try:
            _chk(lib().dabgpu_ofdm_demod_mix(self.h, iq.ptr, IQ_F32 if fmt is None else fmt, dfr.ptr, n, chunks, level,
                                             dsi.ptr if sync else None, dm.ptr, dp.ptr, ds.ptr), "ofdm_demod_mix")
            mix = dm.download(np.float32, (n, NSYM, 2048, 2))
            soft = ds.download(np.uint8 if sync else np.int16, (n, NSYM, SYMBITS))
            out = (mix, soft) + ((dsi.download(np.int32, n),) if sync else ())
            if with_spec:
                sp = dp.download(np.float32, (n, NSYM, 2048, 2))
                out += (sp[..., 0] + 1j * sp[..., 1],)
            self.check()
            return out
        finally:
            for b in (dfr, dm, dp, ds, dsi):
                if b is not None:
                    b.free()

    def ofdm_symbol(self, samples: np.ndarray, kind: int = 0, spectrum: Optional[np.ndarray] = None):
        """dabgpu_ofdm_symbol (ofdmDecoder::processBlock_0 / processToken one symbol at a
        time): kind 0 = FFT of T_u samples (complex64 [2048]) -> the spectrum in natural bin
        order; kind 1 = a data symbol (T_s samples) against `spectrum` -> (ibits [3072],
        the new spectrum)."""
        x = np.ascontiguousarray(samples, dtype=np.complex64).view(np.float32)
        ds, dsp = self.put(x), self.buf(8 * 2048)
        db = self.buf(2 * SYMBITS) if kind else None
        try:
            if spectrum is not None:
                dsp.upload(np.ascontiguousarray(spectrum, dtype=np.complex64).view(np.float32))
            _chk(lib().dabgpu_ofdm_symbol(self.h, ds.ptr, kind, dsp.ptr, db.ptr if db else None), "ofdm_symbol")
            sp = dsp.download(np.float32, (2048, 2))
            self.check()
            spec = sp[:, 0] + 1j * sp[:, 1]
            return (db.download(np.int16, SYMBITS), spec) if kind else spec
        finally:
            for b in (ds, dsp, db):
                if b is not None:
                    b.free()

    def nco_eval(self, first: int = 0, n: int = 2048000) -> np.ndarray:
        """oscillatorTable[first:first+n] as the front-end kernels compute it
        (dabgpu_nco_eval): float32 [n, 2]"""
        d = self.buf(8 * n)
        try:
            _chk(lib().dabgpu_nco_eval(self.h, first, n, d.ptr), "nco_eval")
            out = d.download(np.float32, (n, 2))
            self.check()
            return out
        finally:
            d.free()

    def sync_demod(self, iq: DevBuf, frames: Sequence[Frame], level: int = 3, with_float: bool = False):
        """findIndex + get_snr + processToken x 75 in one launch (dabgpu_ofdm_sync_demod).
        Frame i must have out_slot == i.  Returns (start_index [n], snr [n], ibits [n,75,3072],
        softf or None, freqcorr [n] complex)."""
        n = len(frames)
        fa = (Frame * n)(*frames)
        dfr = DevBuf(self, C.sizeof(fa)).upload(np.frombuffer(fa, dtype=np.uint8))
        dsi, dsn = self.buf(4 * n), self.buf(2 * n)
        ds = self.buf(2 * n * NSYM * SYMBITS)
        df = self.buf(4 * n * NSYM * SYMBITS) if with_float else None
        dfc = self.buf(8 * n)
        try:
            _chk(lib().dabgpu_ofdm_sync_demod(self.h, iq.ptr, dfr.ptr, n, level, dsi.ptr, dsn.ptr, ds.ptr,
                                              df.ptr if df else None, dfc.ptr), "ofdm_sync_demod")
            si = dsi.download(np.int32, n)
            snr = dsn.download(np.int16, n)
            soft = ds.download(np.int16, (n, NSYM, SYMBITS))
            softf = df.download(np.float32, (n, NSYM, SYMBITS)) if df else None
            fc = dfc.download(np.float32, (n, 2))
            self.check()
            return si, snr, soft, softf, fc[:, 0] + 1j * fc[:, 1]
        finally:
            for b in (dfr, dsi, dsn, ds, df, dfc):
                if b is not None:
                    b.free()


class Pipeline:
    """ofdmProcessor::run + ficHandler + mscHandler for n_streams ensembles
    (ofdm-processor.cpp:247-474, fic-handler.cpp:192-321, msc-handler.cpp:125-193,
    dab-concurrent.cpp:144-193), n_frames frames per run() call."""

    def __init__(self, ctx: Context, n_streams: int, n_frames: int, subch: Sequence[Subch],
                 threshold: int = 3, freq_sync_method: int = 1):
        self.ctx, self.S, self.F, self.subch = ctx, n_streams, n_frames, list(subch)
        self._arr = (Subch * max(1, len(self.subch)))(*self.subch)
        cfg = PipeCfg(n_streams, n_frames, len(self.subch), threshold, freq_sync_method,
                      C.cast(self._arr, C.POINTER(Subch)))
        h = C.c_void_p()
        _chk(lib().dabgpu_pipe_create(ctx.h, C.byref(cfg), C.byref(h)), "dabgpu_pipe_create")
        self.h = h
        self.msc_stride = max([24 * s.bitRate for s in self.subch] + [768])
        self.msc_stride = (self.msc_stride + 15) // 16 * 16
        self.msc_stride_packed = self.msc_stride // 8        # bytes per codeword with set_packed
        self.packed = False
        self.fic_packed = False
        self.iq_format = IQ_F32                              # dabgpu_pipe_set_iq_format's default
        # consecutive runs decode concurrently on two back-end streams (dabgpu.h,
        # dabgpu_pipe_sync): outputs alternate between two buffer sets
        self._outs = [(ctx.buf(n_streams * n_frames * 4 * 768), ctx.buf(n_streams * n_frames * 12),
                       ctx.buf(max(1, n_streams * 4 * n_frames * len(self.subch) * self.msc_stride)))
                      for _ in range(2)]
        self._run = 0
        self.fic_d, self.crc_d, self.msc_d = self._outs[0]
        self.dp = [s for s in self.subch if s.flags & SUBCH_DABPLUS]
        self.sf_stride = max([110 * (s.bitRate // 8) for s in self.dp] + [16])
        if self.dp:
            # two sets as well: run r's records may still be copied out (fetch) while
            # run r+1's DAB+ layer writes
            nrec = n_streams * 4 * n_frames * len(self.dp)
            self._sf = [(ctx.buf(nrec * self.sf_stride), ctx.buf(nrec * C.sizeof(Superframe))) for _ in range(2)]
            self.sf_d, self.sfi_d = self._sf[0]

    def acquire(self, iq: DevBuf, stride: int, start: Sequence[int], n_avail: Sequence[int]) -> None:
        st = np.asarray(start, dtype=np.int64)
        na = np.asarray(n_avail, dtype=np.int64)
        _chk(lib().dabgpu_pipe_acquire(self.h, iq.ptr, stride, _p(st), _p(na)), "dabgpu_pipe_acquire")

    def run(self, iq: DevBuf, stride: int, n_avail: Sequence[int], download: bool = True, partial: bool = False):
        """one dabgpu_pipe_run; partial=True accepts a run in which a stream ran out of
        samples (DABGPU_E_STATE: its decoded frames are still delivered)"""
        na = np.asarray(n_avail, dtype=np.int64)
        valid = np.zeros((self.S, 4 * self.F), dtype=np.uint8)
        self.fic_d, self.crc_d, self.msc_d = self._outs[self._run & 1]
        self._run += 1
        ms = self.msc_stride_packed if self.packed else self.msc_stride
        rc = lib().dabgpu_pipe_run(self.h, iq.ptr, stride, _p(na), self.fic_d.ptr, self.crc_d.ptr,
                                   self.msc_d.ptr if self.subch else None, ms, _p(valid))
        if not (partial and rc == -6):
            _chk(rc, "dabgpu_pipe_run")
        if not download:
            return valid
        self.sync()
        fic = self.fic_d.download(np.uint8, (self.S, self.F, 4, 96 if self.fic_packed else 768))
        crc = self.crc_d.download(np.uint8, (self.S, self.F, 12))
        msc = self.msc_d.download(np.uint8, (self.S, 4 * self.F, len(self.subch), ms)) if self.subch else None
        return fic, crc, msc, valid

    def set_dabplus_compact(self, on: bool = True) -> None:
        """compact superframe bytes (dabgpu_pipe_set_dabplus_compact): dabplus() then returns
        bytes [S, n_dabplus, sf_slots, sf_stride], the run's superframes in CIF order, and
        each record's `reserved` is its slot"""
        _chk(lib().dabgpu_pipe_set_dabplus_compact(self.h, int(on)), "dabgpu_pipe_set_dabplus_compact")
        self.dp_compact = bool(on)

    @property
    def sf_slots(self) -> int:
        return (4 * self.F + 4) // 5 + 1                  # DABGPU_SF_SLOTS

    def dabplus(self, download: bool = True):
        """DAB+ superframe layer over the CIFs of the last run() (mp4processor.cpp:107-292).
        Returns (info [S, 4F, n_dabplus] Superframe records, bytes [S, 4F, n_dabplus, sf_stride]
        -- or [S, n_dabplus, sf_slots, sf_stride] with set_dabplus_compact)."""
        self.sf_d, self.sfi_d = self._sf[(self._run - 1) & 1]
        _chk(lib().dabgpu_pipe_dabplus(self.h, self.sf_d.ptr, self.sf_stride, self.sfi_d.ptr), "dabgpu_pipe_dabplus")
        if not download:
            return None
        self.sync()
        nd = len(self.dp)
        raw = self.sfi_d.download(np.uint8, self.S * 4 * self.F * nd * C.sizeof(Superframe))
        info = np.frombuffer(raw.tobytes(), dtype=SUPERFRAME_DTYPE).reshape(self.S, 4 * self.F, nd)
        if getattr(self, "dp_compact", False):
            sf = self.sf_d.download(np.uint8, (self.S, nd, self.sf_slots, self.sf_stride))
        else:
            sf = self.sf_d.download(np.uint8, (self.S, 4 * self.F, nd, self.sf_stride))
        return info, sf

    STAGES = ("prs_sync", "block0", "demod", "fic", "msc_acs", "msc_traceback", "dabplus")

    def sync(self) -> None:
        """wait for every stage of the last run (channel decoding runs on the
        pipeline's own stream, overlapping the next run's front end)"""
        _chk(lib().dabgpu_pipe_sync(self.h), "dabgpu_pipe_sync")

    def set_profiling(self, on=True) -> None:
        """True/1: time the last run; 2: accumulate over every run from now on; 3: as 2
        with every stage run alone on the device (roofline timing); False/0: off"""
        mode = 0 if on is False else 1 if on is True else int(on)
        _chk(lib().dabgpu_pipe_set_profiling(self.h, mode), "set_profiling")

    def timing(self) -> dict:
        """per-stage kernel milliseconds and launch counts (last run, or summed since
        set_profiling(2))"""
        ms = np.zeros(len(self.STAGES), np.float32)
        n = np.zeros(len(self.STAGES), np.int32)
        _chk(lib().dabgpu_pipe_timing(self.h, _p(ms), _p(n)), "timing")
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.STAGES)}

    def state(self, s: int) -> StreamState:
        o = StreamState()
        _chk(lib().dabgpu_pipe_state(self.h, s, C.byref(o)), "dabgpu_pipe_state")
        return o

    def frame_info(self):
        """[S][F] FrameInfo records of the last run"""
        n = self.S * self.F
        fi = (FrameInfo * n)()
        _chk(lib().dabgpu_pipe_frame_info(self.h, C.cast(fi, C.c_void_p)), "dabgpu_pipe_frame_info")
        return [list(fi)[s * self.F:(s + 1) * self.F] for s in range(self.S)]

    def control(self, op: int, stream: int = -1) -> None:
        """ofdmProcessor's reset / coarseCorrectorOn/Off / set_scanMode (dabgpu_pipe_control)"""
        _chk(lib().dabgpu_pipe_control(self.h, stream, op), "dabgpu_pipe_control")

    def frames(self):
        n = self.S * self.F
        fr = (Frame * n)()
        si = np.zeros(n, dtype=np.int32)
        _chk(lib().dabgpu_pipe_frames(self.h, C.cast(fr, C.c_void_p), _p(si)), "dabgpu_pipe_frames")
        return list(fr), si.reshape(self.S, self.F)

    def set_packed(self, on=True) -> None:
        """output format of the following runs (dabgpu_pipe_set_packed): True / PACK_MSC:
        MSC 8 bits per byte, msb first (packbits order) instead of one bit per byte -- run()
        then returns msc [S, 4F, n_subch, msc_stride_packed] bytes; | PACK_FIC: the FIC as
        FIB bytes, fic [S, F, 4, 96]"""
        m = PACK_MSC if on is True else 0 if on is False else int(on)
        _chk(lib().dabgpu_pipe_set_packed(self.h, m), "dabgpu_pipe_set_packed")
        self.packed = bool(m & PACK_MSC)
        self.fic_packed = bool(m & PACK_FIC)

    def acquire_wait(self) -> None:
        """wait for a background null search in flight and apply it (dabgpu_pipe_acquire_wait)"""
        _chk(lib().dabgpu_pipe_acquire_wait(self.h), "dabgpu_pipe_acquire_wait")

    def set_display_token(self, token: int) -> None:
        """the symbol (1..75) the display feed keeps (ofdmDecoder::set_displayToken)"""
        _chk(lib().dabgpu_pipe_set_display_token(self.h, int(token)), "dabgpu_pipe_set_display_token")

    def set_iq_format(self, fmt: int) -> None:
        """sample format of the streams acquire() / run() read: IQ_F32 (default), IQ_S16
        (.sdr PCM16) or IQ_U8 (.raw), converted exactly in the kernels' loads
        (dabgpu_pipe_set_iq_format); strides and n_avail stay in samples"""
        _chk(lib().dabgpu_pipe_set_iq_format(self.h, int(fmt)), "dabgpu_pipe_set_iq_format")
        self.iq_format = int(fmt)

    def fetch(self, dst: "HostBuf", src: DevBuf, nbytes: int, dst_off: int = 0) -> None:
        """asynchronous copy of an output of the last run to pinned host memory, behind
        that run's channel decoding (dabgpu_pipe_fetch)"""
        _chk(lib().dabgpu_pipe_fetch(self.h, C.c_void_p(dst.ptr.value + dst_off), src.ptr, nbytes),
             "dabgpu_pipe_fetch")

    def set_display(self, on: bool = True) -> None:
        """keep symbol 2's display carriers of every decoded frame (dabgpu_pipe_set_display)"""
        _chk(lib().dabgpu_pipe_set_display(self.h, int(on)), "dabgpu_pipe_set_display")

    def iq_display(self, stream: int, frame: int) -> np.ndarray:
        """processToken's iqBuffer values (ofdm-decoder.cpp:197-205) of (stream, frame) of
        the last run: complex64 [1536]"""
        out = np.zeros((K, 2), np.float32)
        _chk(lib().dabgpu_pipe_iq_display(self.h, stream, frame, _p(out)), "dabgpu_pipe_iq_display")
        return out[:, 0] + 1j * out[:, 1]

    def softbits(self) -> np.ndarray:
        """the soft-bit ring of the last run as [stream][slot][75][3072] ibits rows (the ring
        holds ibits + 127 as bytes, dabgpu.h dabgpu_pipe_softbits)"""
        p, r = C.c_void_p(), C.c_int32()
        _chk(lib().dabgpu_pipe_softbits(self.h, C.byref(p), C.byref(r)), "softbits")
        n = self.S * r.value * NSYM * SYMBITS
        raw = np.empty(n, dtype=np.uint8)
        _chk(lib().dabgpu_memcpy_d2h(self.ctx.h, _p(raw), p, raw.nbytes), "d2h")
        return (raw.astype(np.int16) - 127).reshape(self.S, r.value, NSYM, SYMBITS)

    def close(self) -> None:
        if self.h:
            for o in self._outs + (self._sf if self.dp else []):
                for b in o:
                    b.free()
            lib().dabgpu_pipe_destroy(self.h)
            self.h = None
