"""TEST INFRASTRUCTURE: run the GPU streaming pipeline (dabgpu_pipe_*, through the C
ABI) over whole synthetic streams and compare every committed frame with the
oracle's sequential restatement of the reference CPU path (oracle_py.decode_stream):
frame placement and correctors, int16 soft bits, FIC bits + CRCs, MSC bits, DAB+
superframes.  Used by the -m gpu tests and by bench.py's checked step."""
import time

import numpy as np

import oracle_py as orc

IQ_F32, IQ_U8, IQ_S16 = 0, 1, 2                  # dabgpu.h DABGPU_IQ_*


def quantize(iq, fmt):
    """the cf32 samples a recorded format carries: .sdr PCM16 (x -> round(32768 x),
    read back as / 32768, wavfiles.cpp:172) or .raw u8 (x -> round(128 x + 128), read back
    as float(v - 128) / 128.0, rawfiles.cpp:115-117), clipped to the format's range; F32
    unchanged.  The oracle decodes these floats, the GPU the raw samples (to_raw)."""
    x = np.asarray(iq, np.float32)
    if fmt == IQ_S16:
        return (np.clip(np.rint(x * 32768.0), -32768, 32767) / 32768.0).astype(np.float32)
    if fmt == IQ_U8:
        return ((np.clip(np.rint(x * 128.0 + 128.0), 0, 255) - 128.0) / 128.0).astype(np.float32)
    return x


def to_raw(iq, fmt):
    """the raw samples of quantize(iq, fmt) (exact: asserts that iq is representable)"""
    x = np.asarray(iq, np.float32)
    if fmt == IQ_S16:
        r = np.rint(x * 32768.0).astype(np.int16)
        assert np.array_equal(r.astype(np.float32) / 32768.0, x)
        return r
    if fmt == IQ_U8:
        r = np.rint(x * 128.0 + 128.0).astype(np.uint8)
        assert np.array_equal((r.astype(np.float32) - 128.0) / 128.0, x)
        return r
    return x


def gpu_decode(ctx, iqs, F, runs, subch, method=1, n_avail=None, soft_streams=(), dabplus=False, packed=False,
               acq="sync", packed_pad=0, iq_format=IQ_F32, dev_iq=None):
    """Decode `runs` x F frames of every stream.  iqs: list of float32 IQ arrays
    (interleaved); n_avail: optional list (per run) of per-stream available sample
    counts.  iq_format: the streams go to the GPU as that recorded format (iqs must be
    representable: quantize()), read by the kernels through dabgpu_pipe_set_iq_format.
    dev_iq: (DevBuf, stride) already in HBM in that format (e.g. Context.load_recording)
    instead of uploading iqs (which then only give the stream lengths).
    acq: the re-acquisition mode -- "sync" (DABGPU_CTL_ACQ_SYNC: the reference's in-run
    search, so every stream's frames per run are the oracle's ofdmProcessor::run's, which
    the frame-count assertions check); "default" (the engine's default, a stream that loses
    sync is searched in the background, DABGPU_CTL_ACQ_ASYNC; between runs the caller waits
    up to 50 ms for a search in flight, a real-time feed's pace); "async" (explicit
    DABGPU_CTL_ACQ_ASYNC after a synchronous first acquisition, 50 ms between runs).
    Returns per stream: dict(info [frames], fic, crc, msc {cif: [nsub][nb]},
    soft {frame: [75][3072]} for soft_streams, sf {cif: [(info, bytes)...]})."""
    import dabamd
    S = len(iqs)
    lens = [len(x) // 2 for x in iqs]
    stride = max(lens)
    if dev_iq is not None:
        diq, stride = dev_iq
    else:
        dt = {IQ_F32: np.float32, IQ_S16: np.int16, IQ_U8: np.uint8}[iq_format]
        buf = np.zeros((S, 2 * stride), dt)
        for s, x in enumerate(iqs):
            buf[s, :len(x)] = to_raw(x, iq_format)
        diq = ctx.put(buf)
        del buf
    subs = [dabamd.Subch(sc[0], sc[1], sc[2], sc[3], 0 if sc[4] else 1,
                         dabamd.SUBCH_DABPLUS if (len(sc) > 5 and sc[5]) else 0) for sc in subch]
    dpi = [k for k, sc in enumerate(subch) if len(sc) > 5 and sc[5]]
    pipe = dabamd.Pipeline(ctx, S, F, subs, freq_sync_method=method)
    if iq_format != IQ_F32:
        pipe.set_iq_format(iq_format)
    if packed:                  # MSC bits 8 per byte (dabgpu_pipe_set_packed), unpacked here;
        # packed == "fic": the FIC as FIB bytes too (DABGPU_PACK_FIC)
        pipe.set_packed(dabamd.PACK_MSC | (dabamd.PACK_FIC if packed == "fic" else 0))
        pipe.msc_stride_packed += packed_pad    # a row stride that is not a multiple of 4 bytes
    if acq == "async":          # null searches in the background (DABGPU_CTL_ACQ_ASYNC) after the first
        pipe.acquire(diq, stride, [0] * S, lens)
        pipe.control(dabamd.CTL_ACQ_ASYNC)
    elif acq == "sync":         # the reference's in-run search
        pipe.control(dabamd.CTL_ACQ_SYNC)
    out = [dict(info=[], fic=[], crc=[], msc={}, soft={}, sf={}, states=[]) for _ in range(S)]
    nfr = [0] * S
    try:
        for r in range(runs):
            na = n_avail[r] if n_avail is not None else lens
            if acq == "async" and r:
                time.sleep(0.05)    # a background search finishes between runs (a real-time feed's pace)
            elif acq == "default" and r:
                t0 = time.time()
                while any(pipe.state(s).acquiring for s in range(S)) and time.time() - t0 < 0.05:
                    time.sleep(0.001)
            fic, crc, msc, valid = pipe.run(diq, stride, na, partial=True)
            if packed and msc is not None:
                msc = np.unpackbits(msc, axis=-1)
            if packed == "fic":
                fic = np.unpackbits(fic, axis=-1)
            dp = pipe.dabplus() if dpi else None
            fi = pipe.frame_info()
            frames, _ = pipe.frames()
            ring = pipe.softbits() if soft_streams else None
            for s in range(S):
                st = pipe.state(s)
                out[s]["states"].append(st)
                nf = st.frames_run
                cif0 = st.cif_count - 4 * nf
                for f in range(nf):
                    g = nfr[s] + f
                    assert fi[s][f].committed
                    out[s]["info"].append(fi[s][f])
                    out[s]["fic"].append(fic[s, f].copy())
                    out[s]["crc"].append(crc[s, f].copy())
                    if s in soft_streams:
                        slot = frames[s * F + f].out_slot - s * ring.shape[1]
                        out[s]["soft"][g] = ring[s, slot].copy()
                for f in range(nf, F):
                    assert not fi[s][f].committed and not crc[s, f].any()
                for c in range(4 * F):
                    assert valid[s, c] == (c < 4 * nf and cif0 + c >= 16), (s, r, c)
                    if valid[s, c] and msc is not None:
                        out[s]["msc"][cif0 + c] = msc[s, c].copy()
                    if dp is not None and c < 4 * nf:
                        info, sfb = dp
                        out[s]["sf"][cif0 + c] = [(info[s, c, k].copy(), sfb[s, c, k].copy()) for k in range(len(dpi))]
                nfr[s] += nf
    finally:
        pipe.close()
        if dev_iq is None:
            diq.free()
    for s in range(S):
        out[s]["fic"] = np.array(out[s]["fic"]).reshape(-1, 4, 768)
        out[s]["crc"] = np.array(out[s]["crc"]).reshape(-1, 12)
    return out


def compare(gpu, ref, subch, check_soft=True):
    """GPU results of one stream against oracle_py.decode_stream's.  Returns a dict of
    counts; decoded-bit mismatches are the numbers the tests require to be zero."""
    n = len(gpu["info"])
    r = dict(frames=n, oracle_frames=ref["n"], placement=0, fic_cw=0, fic_bad=0, crc_bad=0, msc_cw=0,
             msc_bad=0, soft=0, soft_bad=0, soft_offby1_only=True, snr=[])
    assert n <= ref["n"], (n, ref["n"])
    for g in range(n):
        a, b = gpu["info"][g], ref["info"][g]
        if (a.window, a.start_index, a.coarse, a.fine, a.correction) != (
                b.window_start, b.start_index, b.coarse, b.fine, b.correction):
            r["placement"] += 1
    for g in range(n):
        for blk in range(4):
            r["fic_cw"] += 1
            if not np.array_equal(gpu["fic"][g, blk], ref["fic"][g, blk]):
                r["fic_bad"] += 1
        r["crc_bad"] += int(np.count_nonzero(gpu["crc"][g] != ref["crc"][g]))
        if check_soft and g in gpu["soft"]:
            d = gpu["soft"][g].astype(np.int32) - ref["soft"][g]
            r["soft"] += d.size
            r["soft_bad"] += int(np.count_nonzero(d))
            if np.abs(d).max(initial=0) > 1:
                r["soft_offby1_only"] = False
    for c, bits in gpu["msc"].items():
        for k, sc in enumerate(subch):
            nb = 24 * sc[2]
            r["msc_cw"] += 1
            if not np.array_equal(bits[k, :nb], ref["msc"][c, k, :nb]):
                r["msc_bad"] += 1
    return r


def compare_dabplus(gpu, ref, subch):
    """superframe records of the GPU's DAB+ layer against the oracle's mp4Processor
    state machine fed with the ORACLE's MSC bits (the reference CPU path end to end).
    Returns (records compared, mismatches, superframes decoded)."""
    dpi = [k for k, sc in enumerate(subch) if len(sc) > 5 and sc[5]]
    mp4 = [orc.MP4(subch[k][2]) for k in dpi]
    n = bad = ok3 = 0
    for c in sorted(gpu["sf"]):
        for j, k in enumerate(dpi):
            rec, sfb = gpu["sf"][c][j]
            if c < 16:
                bad += int(rec["status"] != -1)
                continue
            o = mp4[j].add(ref["msc"][c, k, :24 * subch[k][2]])
            n += 1
            same = rec["status"] == o["status"]
            if same and o["status"] >= 2:
                same = rec["n_corrected"] == o["n_corrected"] and rec["num_aus"] == o["num_aus"]
            if same and o["status"] == 3:
                na = o["num_aus"]
                nb = 110 * (subch[k][2] // 8)
                same = (np.array_equal(rec["au_start"][:na + 1], o["au_start"][:na + 1]) and
                        rec["au_crc_ok"] == sum(int(o["au_crc"][a]) << a for a in range(na)) and
                        np.array_equal(sfb[:nb], o["out"][:nb]))
                ok3 += 1
            bad += int(not same)
    return n, bad, ok3
