"""bench.py -- DAB Mode-I symbols/s on MI355X (BASELINE.json metric, config C3).

Workload (config C3): E synthetic Mode-I ensembles per GPU (default 64), each with
9 UEP-3 128 kbit/s subchannels filling all 864 CUs.  One step decodes F frames
(default 24) of every ensemble through the full hot path: findIndex, block 0,
FFT + DQPSK + frequency de-interleave of 75 symbols, FIC depuncture/Viterbi/PRBS/
CRC, MSC 16-CIF time de-interleave + UEP depuncture + Viterbi + PRBS for every
subchannel.  IQ (cf32) is resident in HBM before the timed region; the streams were
acquired (null search) during warm-up.  --cfo HZ runs the same workload through a
carrier frequency offset (the general NCO path: per-sample oscillator indices,
running coarse/fine AFC).

Synthetic streams are cyclic (dabsynth_generate_period): each ensemble is one period
of P = 2F frames (5F with DAB+) repeated end to end -- the time interleaver and the
superframe grid wrap around the period, so the stream is valid across the seams and
the decoder does the same work everywhere; synthesis costs P frames per ensemble
instead of the whole run's.

The streams sit in HBM as recorded samples (--iq-format: s16 = .sdr PCM16 by default,
f32, u8 = .raw) that the kernels convert exactly in their loads.

Multi-GPU (C4): one process per GPU.  `python bench.py --gpus N` starts the N ranks
itself (torch.distributed.run, 127.0.0.1) unless it already runs under a launcher.
value: each rank decodes its own ensembles (seeded by rank) from its own HBM -- no
data-path collective, weak scaling.  Then the "c4_fed" leg runs BASELINE configs[3] as
named: rank 0 holds every rank's recorded streams (--fed-format, u8 .raw by default) and
sends each rank chunk k + 2 of ITS streams over RCCL (xGMI) while step k decodes
(FedSplit); the receivers' pipelines read the samples in place.  It is link-bound by
design and reported beside value.  Every rank checks one step of its
ensemble 0 against the transmitted bits in both legs.  value = symbols decoded by all
ranks / max-over-ranks time.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sdr-j-dab_amd"))

TF, TNULL, TU, TS = 196608, 2656, 2048, 2552
RT_SYMBOLS = 76 / 0.096            # symbols/s of one real-time Mode-I ensemble (791.67)
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md chip table (spec)
SYMBOL_BYTES = 8 * TS + 2 * 3072   # algorithmic bytes per OFDM symbol (26,560)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # int32 lane-ops/s: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz
C3_SUBCH = [(96 * i, 96, 128, 3, 1, 0) for i in range(9)]   # (startAddr, CUs, kbps, level, uep, dab+)
# C5: 16 ensembles x 16 DAB+ subchannels (64 kbit/s EEP-3A, 48 CUs, RSDims 8) = 256
C5_SUBCH = [(48 * i, 48, 64, 0o103, 0, 1) for i in range(16)]
WORKLOADS = {
    "c2": ([], 64, "C2 at scale: 64 concurrent Mode-I ensembles/GPU, full frames (76 FFT'd symbols), FIC decode only"),
    "c3": (C3_SUBCH, 64, "C3: 64 concurrent Mode-I ensembles/GPU, FIC + full MSC (9 x UEP-3 128 kbps)"),
    "c5": (C5_SUBCH, 16, "C5: 256 DAB+ subchannels/GPU (16 ensembles x 16 x 64 kbps EEP-3A), FIC + MSC Viterbi "
                         "+ superframe sync + RS(120,110) + AU CRC"),
}


# ------------------------------------------------------------------ processes
def launch_ranks(n):
    """Start n ranks of this command under torch.distributed.run (one process per GPU)
    and return its exit code.  Called before this process touches the GPU; the ranks
    are child processes (no exec)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def dist_setup(n_gpus):
    """rank, local rank, world size and the torch.distributed module (None for 1 rank).
    RCCL ("nccl") when every local rank has its own GPU; gloo when ranks share one (a
    rehearsal of the N > 1 path on a 1-GPU box) or there is no GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world}")
    dist = None
    # DAB_DIST_FORCE=1: a one-rank process group too (RCCL on a GPU box) -- a rehearsal of the
    # N > 1 code paths (collectives, the C4 leg's transport) on one GPU
    if world > 1 or os.environ.get("DAB_DIST_FORCE") == "1":
        import torch
        import torch.distributed as td
        ngpu = torch.cuda.device_count()
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        backend = os.environ.get("DAB_DIST_BACKEND") or ("nccl" if ngpu >= lws and ngpu > 0 else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        td.init_process_group(backend=backend)
        dist = td
        # the ranks' barriers, time reductions and check gathers go through a gloo group on
        # the host: an RCCL communicator, once created, slows this process's pipeline by ~9 %
        # (profiles/r05_rccl_overhead_ab.txt), so RCCL is used only where the data moves (the C4
        # leg's transfers, after the rank-local legs)
        global _CTL
        # (DAB_CTL_RCCL=1, A/B only: the control collectives on the RCCL group, as round 5's
        # first N > 1 path ran them -- tools/rccl_overhead.sh)
        _CTL = td.new_group(backend="gloo") if backend == "nccl" and os.environ.get("DAB_CTL_RCCL") != "1" else None
        if backend == "nccl" and os.environ.get("DAB_RCCL_EARLY") == "1":
            # A/B hook (tools/rccl_overhead.sh): create the RCCL communicator before the
            # rank-local legs, as round 5's first N > 1 path did
            t = torch.ones(1, device=f"cuda:{local}")
            td.all_reduce(t)
            torch.cuda.synchronize()
    return rank, local, world, dist


_CTL = None     # the control group (gloo) beside an RCCL default group


def rank_device(local):
    """GPU of a local rank (ranks share GPUs round-robin when there are fewer GPUs)"""
    try:
        import torch
        n = torch.cuda.device_count()
    except ImportError:
        n = 1
    return local % max(n, 1)


def rank_seed0(rank, ensembles):
    """First ensemble seed of a rank: ranks decode disjoint ensemble sets (weak scaling)."""
    return 1000 + rank * ensembles


def barrier(dist):
    if dist is not None:
        dist.barrier(group=_CTL)


def allreduce_max(dist, x):
    if dist is None:
        return x
    import torch
    dev = "cuda" if _CTL is None and dist.get_backend() == "nccl" else "cpu"   # (DAB_CTL_RCCL A/B)
    t = torch.tensor([x], dtype=torch.float64, device=dev)   # on the host: the gloo control group
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=_CTL)
    return float(t.item())


# ------------------------------------------------------------ sample formats
# recorded-IQ formats the pipeline reads straight from HBM (dabgpu_pipe_set_iq_format):
# name -> (DABGPU_IQ_* code, bytes per I/Q pair, numpy dtype of one value)
FORMATS = {"f32": (0, 8, np.float32), "u8": (1, 2, np.uint8), "s16": (2, 4, np.int16)}
FORMAT_DESC = {"f32": "cf32 (virtualInput::getSamples' DSPCOMPLEX)",
               "s16": ".sdr PCM16 (wavfiles.cpp:172: x / 32768, converted in the kernels' loads)",
               "u8": ".raw u8 (rawfiles.cpp:115-117: float(x - 128) / 128, converted in the kernels' loads)"}
# transmitter amplitude of the synthetic streams: peaks inside +-1, as a recording's gain
# sets them (unit-power OFDM at 1.0 would clip in the PCM16 / u8 formats)
AMPLITUDE = 0.25


def to_raw(iq, fmt):
    """cf32 IQ -> the samples of a recorded format: s16 round(32768 x), u8 round(128 x + 128),
    clipped to the format's range (what the readers turn back into x exactly)"""
    x = np.asarray(iq, np.float32)
    if fmt == "s16":
        return np.clip(np.rint(x * 32768.0), -32768, 32767).astype(np.int16)
    if fmt == "u8":
        return np.clip(np.rint(x * 128.0 + 128.0), 0, 255).astype(np.uint8)
    return x


def to_s16(iq):
    return to_raw(iq, "s16")


# --------------------------------------------------------------- stream split
def chunk_layout(stream_len, F):
    """samples per stream chunk (F frames) and the number of chunks covering a stream"""
    cs = F * TF
    return cs, (stream_len + cs - 1) // cs


def period_frames(F, dabplus):
    """Frames of the cyclic period every synthetic stream repeats (dabsynth_generate_period):
    a multiple of the step's F frames (the stream split then ships P / F distinct chunk
    phases) whose 4P CIFs hold whole DAB+ superframes (5 CIFs)."""
    m = 2
    while dabplus and (4 * F * m) % 5:
        m += 1
    return F * m


def fill_chunk_phases(out, per, ens, P, cs, g0, fmt):
    """out[j, g0 + e] = stream samples [j cs, (j+1) cs) of the cyclic stream whose period
    is per[e] (interleaved cf32), as format fmt -- chunk k of the stream is phase k % m"""
    for j in range(out.shape[0]):
        for p, q, c in ens.stream_pieces(P, j * cs, cs):
            o = p - j * cs
            out[j, g0:g0 + len(per), 2 * o:2 * (o + c)] = to_raw(per[:, 2 * q:2 * (q + c)], fmt)


def chunk_phases(ens, P, cs, E, seed0, threads, fmt="s16"):
    """the P * TF / cs distinct stream chunks of E cyclic streams (seeds seed0 + e) in a
    recorded format: [phase j][ensemble][2 * cs] values"""
    m = P * TF // cs
    out = np.zeros((m, E, 2 * cs), FORMATS[fmt][2])
    for g0 in range(0, E, 8):
        n = min(8, E - g0)
        fill_chunk_phases(out, ens.period_many(n, seed0=seed0 + g0, period=P, threads=threads), ens, P, cs, g0, fmt)
    return out


def p2p_batch(dist, sends, recvs):
    """One grouped batch of point-to-point transfers, sends / recvs = [(tensor, peer)], in
    posting order per peer.  Under RCCL ("nccl") one ncclGroupStart/End: every transfer
    on its own xGMI link, received in place.  Under gloo with device tensors (ranks sharing
    one GPU: the rehearsal of this path) staged through host copies.  Returns waitables."""
    import torch
    import torch.distributed as td
    staged = td.get_backend() == "gloo" and any(t.is_cuda for t, _ in list(sends) + list(recvs))

    # the wire carries bytes: a recording's int16 samples travel as their bytes (the NCCL
    # process group refuses int16 tensors; the view is the same memory, received in place)
    def wire(t):
        return t if t.dtype in (torch.uint8, torch.int8) else t.view(torch.uint8)
    sends = [(wire(t), p) for t, p in sends]
    recvs = [(wire(t), p) for t, p in recvs]
    if not staged:
        ops = [td.P2POp(td.isend, t, p) for t, p in sends] + [td.P2POp(td.irecv, t, p) for t, p in recvs]
        return td.batch_isend_irecv(ops) if ops else []
    hs = [(t.cpu(), p) for t, p in sends]
    hr = [(torch.empty(t.shape, dtype=t.dtype), t, p) for t, p in recvs]
    ops = [td.P2POp(td.isend, h, p) for h, p in hs] + [td.P2POp(td.irecv, h, p) for h, _, p in hr]
    reqs = td.batch_isend_irecv(ops) if ops else []

    class _Staged:
        def wait(self):
            for q in reqs:
                q.wait()
            for h, t, _ in hr:
                t.copy_(h)
    return [_Staged()]


class FedSplit:
    """The C4 stream split (BASELINE configs[3]: "512 ensembles sharded across
    8 MI355X via RCCL ... of IQ chunks over xGMI").  Rank 0 holds every rank's recorded
    streams: src[r] = [phases][E][2 * cs] values of rank r's ensembles.  begin(k) moves
    chunk k of every stream of every rank r >= 1 from rank 0 straight into rank r's stream
    buffer -- dst(e, k) is the [2 * cs] view of stream e's samples [k cs, (k+1) cs) -- as
    one grouped batch (E sends per destination on rank 0, E receives on each rank: a
    scatter, each destination over its own link, not a ring broadcast of all 512
    ensembles); end(reqs) waits for it.  Rank 0 reads its own streams in place."""

    def __init__(self, dist, rank, world, E, phases, src=None, dst=None):
        self.dist, self.rank, self.world, self.E, self.phases = dist, rank, world, E, phases
        self.src, self.dst = src, dst

    def begin(self, k):
        if self.rank == 0:
            sends = [(self.src[r][k % self.phases][e], r) for r in range(1, self.world) for e in range(self.E)]
            return p2p_batch(self.dist, sends, [])
        return p2p_batch(self.dist, [], [(self.dst(e, k), 0) for e in range(self.E)])

    def end(self, reqs):
        for r in reqs or []:
            r.wait()
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.current_stream().synchronize()       # the chunk has landed before a run reads it


def gather_to_rank0(dist, rank, world, mine):
    """setup (untimed): every rank's chunk phases to rank 0 (one transfer per rank);
    returns the list [rank 0's, rank 1's, ...] on rank 0, None elsewhere"""
    import torch
    if rank == 0:
        got = [mine] + [torch.empty_like(mine) for _ in range(1, world)]
        for r in p2p_batch(dist, [], [(got[q], q) for q in range(1, world)]):
            r.wait()
        return got
    for r in p2p_batch(dist, [(mine, 0)], []):
        r.wait()
    return None


def check_step(truth, P, st0, st1, fic, crc, msc, valid, subch):
    """The checked step of ensemble 0: decoded FIC blocks (CRC field restored) and MSC
    codewords against the transmitted bits of its cyclic stream (frame f of the stream
    is frame f mod P of the period, receiver CIF n carries CIF n mod 4P's truth)."""
    f0 = st1.frames_run
    cif0 = st0.cif_count
    flip = _crc_flip()
    fic_ok = all(np.array_equal(fic[0, f, b] ^ flip, truth["fic"][(cif0 // 4 + f) % P, b])
                 for f in range(f0) for b in range(4))
    msc_ok = msc_n = 0
    for c in range(4 * f0):
        if not valid[0, c]:
            continue
        for k, sc in enumerate(subch):
            nb = 24 * sc[2]
            msc_n += 1
            msc_ok += int(np.array_equal(msc[0, c, k, :nb], truth["msc"][(cif0 + c) % (4 * P), k, :nb]))
    return {"ensemble": 0, "frames": int(f0), "fic_blocks_equal_transmitted": bool(fic_ok),
            "fic_crc_pass_rate": float(crc[0, :f0].mean()) if f0 else 0.0, "msc_codewords": msc_n,
            "msc_equal_transmitted": msc_ok}


def gather_objects(dist, obj):
    """obj of every rank, in rank order (a one-element list for one rank)"""
    if dist is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj, group=_CTL)
    return out


# ----------------------------------------------------------------- CPU side
def pmc_traffic(kernel, workload):
    """HBM bytes per full-batch launch of `kernel` from the newest committed PMC
    summary for this workload (profiles/rNN_traffic_<workload>.json, made by
    tools/pmc_traffic.py from the FETCH_SIZE / WRITE_SIZE passes of this bench
    command at its default size), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{workload}.json")))
    if not files:
        return None
    try:
        k = json.load(open(files[-1]))["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    return None if k is None else {"bytes": k["hbm_bytes"], "fetch_bytes": k["fetch_bytes"],
                                   "write_bytes": k["write_bytes"], "source": os.path.basename(files[-1])}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """the cgroup's CPU quota in cores (cpu.max), or None when unlimited / unreadable"""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def gen_threads(world):
    """synthesis threads per rank: the job's CPU share (the cgroup quota when one is set, else
    OMP_NUM_THREADS, else the affinity set) split over the ranks of this node, at most 16 --
    8 ranks x 16 threads on a 16-core share would time-slice 8x"""
    q = cpu_quota()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    share = int(q) if q is not None else (omp if omp > 0 else len(os.sched_getaffinity(0)))
    return max(1, min(16, share // max(world, 1)))


def cpu_cores():
    """the cores the workers run on: the process's affinity set, capped at the box's CPU
    share (OMP_NUM_THREADS, which the GPU box sets to its share, and the cgroup quota) --
    more workers than the share only time-slice the same cores"""
    cores = sorted(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    q = cpu_quota()
    if q is not None:
        cap = min(cap, int(q)) if cap > 0 else int(q)
    return cores[:cap] if cap > 0 else cores


def cpu_baseline(frames=20, budget_s=20.0, workload="c3", cfo=0.0):
    """The reference CPU path on the host cores: one worker process per
    core, pinned (sched_setaffinity = taskset), each decoding its own synthetic ensemble
    of the workload for a bounded time.  Stages: OFDM front end = the oracle's C
    restatement of ofdmProcessor::run/ofdmDecoder with the reference's oscillatorTable and
    an fp32 radix-4 FFT (orc_fft2048_f32: FFTW3f, absent here, is an fp32 transform); FIC = restated depuncture + the reference's
    viterbi.cpp + spiral-sse.c + check_CRC_bits; MSC = restated 16-CIF de-interleave +
    the reference's deconvolve.cpp (UEP/EEP + Viterbi) + PRBS; DAB+ = the reference's
    firecode_checker + reedSolomon inside the restated mp4Processor glue
    (oracle/ref_wrap.cpp: ref_mp4_add)."""
    import multiprocessing as mp
    cores = cpu_cores()
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(w, core, frames, budget_s, q, workload, cfo))
             for w, core in enumerate(cores)]
    for p in procs:
        p.start()
    res = [q.get() for _ in procs]
    for p in procs:
        p.join()
    secs = max(r["secs"] for r in res)
    tot = {k: sum(r[k] for r in res) for k in ("symbols", "fic_bits", "msc_bits", "rs_cw", "t_ofdm", "t_fic",
                                               "t_msc", "t_dabplus")}
    # the OFDM front end (most of the CPU time) is the oracle's C restatement -- the
    # reference's ofdm-decoder.cpp / fft.cpp need Qt and FFTW3f, absent here (building
    # them against stand-in headers is not allowed) -- so the whole
    # chain is labelled a port; its FIC/MSC/DAB+ back end is the reference's own code
    kind = "port"
    return dict(value=tot["symbols"] / secs, cores=len(cores), kind=kind, tot=tot, secs=secs,
                nproc=os.cpu_count(), cpu=cpu_model(), affinity=len(os.sched_getaffinity(0)),
                omp=os.environ.get("OMP_NUM_THREADS"), quota=cpu_quota())


def _cpu_worker(w, core, frames, budget_s, q, workload, cfo):
    os.sched_setaffinity(0, {core})
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    import oracle_py as orc
    from dabamd.synth import Ensemble
    ref = orc.ref()
    subch = WORKLOADS[workload][0]
    # a cyclic stream (as the GPU side's) of frames + 4 frames: long enough for the AFC to
    # converge under the carrier offset (~11 frames at 1.3 kHz) and for DAB+ superframes
    # to decode after the 16-CIF de-interleaver warm-up -- every stage does its real work
    e = Ensemble(frames + 4, subch=subch, snr_db=30.0, cfo_hz=cfo)
    per = 10                                           # 40 CIFs: whole DAB+ superframes
    g = {"iq": e.stream_from_period(e.generate_period(9000 + w, per, truth=False)["iq"], per)}
    prbs = orc.prbs(24 * 384)
    P = orc.P
    st = dict(symbols=0, fic_bits=0, msc_bits=0, rs_cw=0, t_ofdm=0.0, t_fic=0.0, t_msc=0.0, t_dabplus=0.0)

    class Mp4(C.Structure):
        _fields_ = [("bitRate", C.c_int), ("fill", C.c_int), ("blocks", C.c_int), ("ring", C.c_uint8 * (120 * 48))]

    delay = np.array([orc.oracle().orc_interleave_delay(i) for i in range(16)])
    crc_fn = ref.ref_check_crc_bits if ref is not None else orc.oracle().orc_check_crc_bits
    t0 = time.perf_counter()
    while True:
        a = time.perf_counter()
        n, info, soft = orc.ofdm_run(g["iq"], frames + 4, fft_kind=1)
        b = time.perf_counter()
        st["t_ofdm"] += b - a
        for f in range(n):                               # ficHandler: 4 blocks per frame
            fic = soft[f, 0:3].reshape(-1)
            for blk in range(4):
                vb = np.zeros(3096, np.int16)
                orc.oracle().orc_fic_depuncture(P(np.ascontiguousarray(fic[2304 * blk:2304 * (blk + 1)])), P(vb))
                bits = np.zeros(768, np.uint8)
                if ref is not None:
                    ref.ref_viterbi(P(vb), 768, P(bits))
                else:
                    orc.oracle().orc_viterbi(P(vb), 768, P(bits))
                bits ^= prbs[:768]
                for k in range(3):
                    crc_fn(P(bits[256 * k:]), 256)
                st["fic_bits"] += 768
        c = time.perf_counter()
        st["t_fic"] += c - b
        cifs = soft[:, 3:75].reshape(4 * n, -1)
        mp4 = [Mp4(sc[2], 0, 0) if sc[5] else None for sc in subch]
        tm = 0.0
        for k, (sa, ln, br, pl, uep, dp) in enumerate(subch):
            frags = cifs[:, sa * 64:(sa + ln) * 64]
            idx = np.arange(ln * 64)
            d = delay[idx & 15]
            for cc in range(16, 4 * n):                   # dabConcurrent: 16-CIF de-interleave
                frag = np.ascontiguousarray(frags[cc - d, idx])
                out = np.zeros(24 * br, np.uint8)
                if ref is not None:
                    fn = ref.ref_uep_deconvolve if uep else ref.ref_eep_deconvolve
                    fn(br, pl, P(frag), len(frag), P(out))
                    out ^= prbs[:24 * br]
                else:
                    out = orc.msc_deconvolve(uep, br, pl, frag)
                st["msc_bits"] += 24 * br
                if mp4[k] is not None:
                    t1 = time.perf_counter()
                    nok = C.c_int()
                    if ref is not None and ref.ref_mp4_add(C.byref(mp4[k]), P(out), C.byref(nok)) == 3:
                        st["rs_cw"] += br // 8
                    tm += time.perf_counter() - t1
        dd = time.perf_counter()
        st["t_msc"] += dd - c - tm
        st["t_dabplus"] += tm
        st["symbols"] += n * 76
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    st["secs"] = el
    st["ref"] = ref is not None
    q.put(st)


# ----------------------------------------------------------------------- main
def acs_clock_issue():
    """The ACS's achieved clock and VALU issue utilisation from the newest committed PMC
    summary (profiles/rNN_acs_clock_issue.json, tools/acs_clock_issue.py over one
    rocprofv3 --pmc pass of this bench command: GRBM_GUI_ACTIVE / 8 / kernel duration and
    4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x cycles)), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_acs_clock_issue.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
    except (OSError, ValueError):
        return None
    d["source"] = os.path.basename(files[-1])
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--ensembles", type=int, default=0, help="ensembles per GPU (default: C3 64, C5 16)")
    ap.add_argument("--frames", type=int, default=24,
                    help="frames per ensemble per step (the pipeline's batch: 24 frames = 2.3 s of air time; "
                         "throughput saturates from ~24 on MI355X, profiles/r01_frames_sweep.txt)")
    ap.add_argument("--cfo", type=float, default=1300.0,
                    help="carrier frequency offset of the synthetic IQ (Hz); nonzero by default: a receiver's NCO "
                         "always runs (phase = coarse + fine correction), 0 takes the constant-phase shortcut")
    ap.add_argument("--iq-format", choices=["s16", "f32", "u8"], default="s16",
                    help="how the streams sit in HBM: s16 = .sdr PCM16 samples (default; SURVEY 8(d)'s int16 "
                         "transport), f32 = cf32, u8 = .raw samples -- read by the kernels through "
                         "dabgpu_pipe_set_iq_format, converted exactly in their loads")
    ap.add_argument("--fed-format", choices=["u8", "s16"], default="u8",
                    help="the C4 stream split's wire format (N > 1): u8 = .raw (2 B per sample over xGMI)")
    ap.add_argument("--fed-steps", type=int, default=8,
                    help="timed steps of the C4 leg (N > 1): rank 0 feeding every rank its ensembles over RCCL")
    ap.add_argument("--no-c4-fed", action="store_true", help="skip the C4 leg when N > 1")
    ap.add_argument("--fed-timeout", type=float, default=240.0,
                    help="seconds after which the C4 leg is abandoned (the line is printed with its error)")
    ap.add_argument("--msc-format", choices=["bits", "packed"], default="packed",
                    help="MSC output of the timed steps: one bit per byte as the reference's deconvolve delivers it "
                         "(viterbi.cpp:240-241), or 8 bits per byte (dabgpu_pipe_set_packed; the DAB+ layer reads "
                         "either)")
    ap.add_argument("--solo-steps", type=int, default=2,
                    help="steps after the timed region with every kernel alone on the device (profiling mode 3): "
                         "per-kernel times without overlap, to name the dominant kernel")
    ap.add_argument("--delivered-mode", choices=["fetch", "direct"], default="fetch",
                    help="delivered leg: copies behind the decoding (dabgpu_pipe_fetch) or the decoders writing "
                         "pinned host memory directly")
    ap.add_argument("--delivered-fic", choices=["bytes", "bits"], default="bytes",
                    help="FIC format of the delivered leg: FIB bytes (DABGPU_PACK_FIC) or one bit per byte")
    ap.add_argument("--delivered-steps", type=int, default=10,
                    help="timed steps after the main measurement whose FIC bits + CRCs and MSC bytes (8 bits per "
                         "byte) are copied to pinned host memory while the next step decodes (dabgpu_pipe_fetch): "
                         "the delivered rate, reported beside value")
    ap.add_argument("--sync-loss-steps", type=int, default=8,
                    help="timed steps (per acquisition mode) in which one stream every 2 steps loses sync (an "
                         "interferer over 1.5 frames: findIndex fails, goto notSynced) -- the price of a sync loss, "
                         "with the null search inside the run and in the background (DABGPU_CTL_ACQ_ASYNC)")
    ap.add_argument("--c5-steps", type=int, default=12,
                    help="timed steps of the C5 leg (BASELINE configs[4], 16 ensembles x 16 DAB+ subchannels) run "
                         "after the C3 measurement at N = 1, reported as c5 in the same line (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    rank, local, world, dist = dist_setup(args.gpus)
    cpu = None
    if rank == 0 and world == 1 and dist is None and not args.no_cpu_baseline:
        # before this process touches the GPU: the workers are forked children
        cpu = cpu_baseline(budget_s=args.cpu_seconds, workload=args.workload, cfo=args.cfo)
    import dabamd
    from dabamd.synth import Ensemble

    SUBCH, E_default, wl_desc = WORKLOADS[args.workload]
    dabplus = any(s[5] for s in SUBCH)
    E, F = args.ensembles or E_default, args.frames
    fmt_code, bps, _ = FORMATS[args.iq_format]
    # +1 step: the checked pass; then the solo steps
    deliv_steps = args.delivered_steps + 1 if args.delivered_steps > 0 else 0     # + one untimed warm-up
    loss_steps = 2 * (args.sync_loss_steps + 1) if args.sync_loss_steps > 0 else 0  # two modes, + one each
    # (+ 2F: a stream that loses sync skips frames and reaches the end of its samples sooner)
    total_frames = F * (args.warmup + args.steps + 1 + args.solo_steps + deliv_steps + loss_steps + (2 if loss_steps else 0)) + 1
    ens = Ensemble(total_frames, subch=SUBCH, snr_db=30.0, cfo_hz=args.cfo, amplitude=AMPLITUDE)
    P = period_frames(F, dabplus)
    ctx = dabamd.Context(rank_device(local))
    stride = ens.length
    threads = gen_threads(world)
    fed = (world > 1 or dist is not None) and not args.no_c4_fed
    cs, _ = chunk_layout(stride, F)
    fed_ph = np.zeros((P * TF // cs, E, 2 * cs), FORMATS[args.fed_format][2]) if fed else None
    # Every stream is cyclic (dabsynth_generate_period: P frames repeated end to end, a
    # valid DAB stream across the seams), stored in HBM as the chosen recorded format;
    # ensemble 0 of each rank is generated with its transmitted bits for the checked step.
    t0 = time.time()
    diq = ctx.buf(E * stride * bps)
    seed0 = rank_seed0(rank, E)
    truth = ens.generate_period(seed0, P, truth=True)
    truth.pop("iq")
    for g0 in range(0, E, 8):
        n = min(8, E - g0)
        per = ens.period_many(n, seed0=seed0 + g0, period=P, threads=threads)
        for e in range(n):
            raw = to_raw(per[e], args.iq_format)          # once per period, not per repeated piece
            for p, q, m in ens.stream_pieces(P):
                diq.upload_at(raw[2 * q:2 * (q + m)], ((g0 + e) * stride + p) * bps)
            del raw
        if fed:
            fill_chunk_phases(fed_ph, per, ens, P, cs, g0, args.fed_format)
        del per
    gen_s = time.time() - t0
    subs = [dabamd.Subch(s[0], s[1], s[2], s[3], 0 if s[4] else 1, dabamd.SUBCH_DABPLUS if s[5] else 0)
            for s in SUBCH]
    pipe = dabamd.Pipeline(ctx, E, F, subs)
    pipe.set_iq_format(fmt_code)
    if args.msc_format == "packed":
        pipe.set_packed(True)

    # the initial null search of every stream (k_acquire, one wave per stream): the cost a
    # sync loss pays before the pipeline resumes (ofdm-processor.cpp:298-357), reported beside
    # the steady state, never inside the timed region
    pipe.sync()
    t_acq = time.perf_counter()
    pipe.acquire(diq, stride, [0] * E, [stride] * E)
    pipe.sync()
    acquire_ms = (time.perf_counter() - t_acq) * 1e3

    def step(k, download=False, partial=False):
        try:
            r = pipe.run(diq, stride, [stride] * E, download=download, partial=partial)
        except dabamd.DabError:
            # which stream, where: every stream's state to stderr before the error ends the run
            for s in range(E):
                x = pipe.state(s)
                print(f"rank {rank} step {k} stream {s}: next_pos {x.next_pos} of {stride} "
                      f"frames_run {x.frames_run} cif_count {x.cif_count} synced {x.synced} "
                      f"acquiring {x.acquiring} resyncs {x.resyncs} acquisitions {x.acquisitions}", file=sys.stderr)
            raise
        d = pipe.dabplus(download=download) if dabplus else None
        return r, d

    for i in range(args.warmup):
        step(i)
    pipe.sync()
    # per-kernel HIP events on each launch's stream over the timed steps (recording
    # adds no synchronisation); summed and counted by the pipeline
    pipe.set_profiling(2)
    barrier(dist)
    pipe.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    pipe.sync()
    el = time.perf_counter() - t0
    barrier(dist)
    el = allreduce_max(dist, el)
    tsum = pipe.timing()
    pipe.set_profiling(False)
    # kernel time per step and per launch over the timed region
    tm = {k: (v[0] / args.steps, v[0] / max(v[1], 1)) for k, v in tsum.items()}

    # one extra step (outside the timed region) whose outputs are checked against the
    # transmitted bits of ensemble 0 of every rank: every FIB, every MSC subchannel
    ck = args.warmup + args.steps
    st0 = pipe.state(0)
    (fic, crc, msc, valid), dp = step(ck, download=True)
    if pipe.packed:
        msc = np.unpackbits(msc, axis=-1)
    # every rank checks its ensemble 0 against the transmitted bits; rank 0 reports all
    st1 = pipe.state(0)
    check = check_step(truth, P, st0, st1, fic, crc, msc, valid, SUBCH)
    check["rank"] = rank
    check["seed"] = seed0
    checks = gather_objects(dist, check)
    # the same workload with every kernel alone (after the measurement: never timed)
    tm_alone = {}
    if args.solo_steps > 0:
        pipe.sync()
        pipe.set_profiling(3)
        for i in range(args.solo_steps):
            step(ck + 1 + i)
        pipe.sync()
        tm_alone = {k: v[0] / max(v[1], 1) for k, v in pipe.timing().items()}
        pipe.set_profiling(False)
    # the delivered leg: every step's results leave the GPU (FIC bits + CRC flags, the MSC
    # packed 8 bits per byte, DAB+ superframe records + bytes) into pinned host memory,
    # each copy queued behind its run's channel decoding while the next run decodes
    delivered = None
    if deliv_steps:
        k0 = ck + 1 + args.solo_steps
        delivered = delivered_leg(dabamd, ctx, pipe, step, k0, deliv_steps - 1, E, F, SUBCH, dabplus, dist, truth, P,
                                  fic_bytes=args.delivered_fic == "bytes", direct=args.delivered_mode == "direct")
    sync_loss = None
    if loss_steps and E >= 2:
        k0 = ck + 1 + args.solo_steps + deliv_steps
        sync_loss = sync_loss_leg(dabamd, ctx, pipe, step, k0, args.sync_loss_steps, E, F, stride, diq, dist,
                                  el / args.steps * 1e3, args.iq_format)
    c5 = None
    if args.c5_steps > 0 and args.workload == "c3" and world == 1 and dist is None:
        # BASELINE configs[4] in the same run (its own pipeline, after every C3 leg: never timed with
        # them; the C3 pipeline and its streams are released first -- no C4 leg at N = 1)
        pipe.close()
        diq.free()
        try:
            c5 = c5_leg(dabamd, Ensemble, ctx, args.c5_steps, max(args.warmup, 3), F, args.cfo, args.iq_format,
                        args.msc_format, threads)
        except Exception as e:                          # noqa: BLE001 -- reported in the line
            c5 = {"error": repr(e)[:300]}
    sf_ok = None
    if dp is not None:
        info = dp[0]
        sf_ok = {"superframes": int((info["status"] == 3).sum()),
                 "au_crc_pass": int(sum(bin(int(x)).count("1") for x in info["au_crc_ok"][info["status"] == 3])),
                 "cif_records": int((info["status"] >= 0).sum())}
    symbols = world * E * F * 76 * args.steps
    value = symbols / el
    # dominant kernel + its roofline.  Launches overlap in the pipeline (the next run's
    # demod starts beside the ACS and shares the SIMDs with it and the traceback), so the
    # in-pipeline spans include shared time; the dominant kernel is the one with the most
    # GPU time when every kernel runs alone (solo steps), its roofline is priced on its
    # in-pipeline launch duration over the timed region (and, beside it, alone)
    per_step_alone = {k: tm_alone.get(k, 0.0) * (tm[k][0] / tm[k][1] if tm[k][1] else 0.0) for k in tm}
    dom = max(per_step_alone, key=per_step_alone.get) if tm_alone else max(tm, key=lambda k: tm[k][0])
    # the pipeline decodes the FIC in the MSC's ACS launch (dabgpu.h, DABGPU_STAGE_FIC)
    acs_steps = E * 4 * F * sum(24 * s[2] + 6 for s in SUBCH) + E * F * 4 * (768 + 6)
    # (without MSC subchannels the FIC has launches of its own, k_acs<2>)
    acs_stage, acs_kernel = ("msc_acs", "dab::k_acs2<3, 2, true>") if SUBCH else ("fic", "dab::k_acs<2, true>")
    acs_ms = max(tm[acs_stage][1], 1e-9)            # average launch duration
    acs_ops = acs_steps * 64 * 4                    # 2 adds + compare + select per ACS
    demod_ms = max(tm["demod"][1], 1e-9)
    # the recorded samples in + the pipeline's RING8 soft bits out (one byte each: ibits +
    # 127) + the findIndex window; SURVEY 8(d)'s 26,560 B/symbol counts cf32 in, int16 out
    demod_bytes = E * F * (75 * (bps * TS + 3072) + bps * TU)
    demod_kernel = "dab::k_demod_wg<%s, true, true, %d, false>" % ("true" if args.cfo else "false", fmt_code)
    roof_valu = {"kernel": f"{acs_kernel[5:]} (Viterbi ACS)", "bound": "valu",
                 "achieved": acs_ops / (acs_ms * 1e-3) / 1e12, "peak": VALU_PEAK_TOPS, "unit": "TOP/s",
                 "traffic": pmc_traffic(acs_kernel, args.workload),
                 "note": "4 int ops per add-compare-select x 64 states per trellis step; peak = 256 CU x 4 SIMD x "
                         "32 lanes x 2.4 GHz (the 32-bit rate). Formulation ceiling ~0.6 of it: the exact u16x2 ACS "
                         "word is 6 VALU per wave-step (2 codeword steps = 512 ops), of which the packed-16, DPP, "
                         "v_perm and v_bfi ops issue at half rate (profiles/r02_valu_rate.txt), ~24 issue cycles + "
                         "~2 for the loader: 512 / 26 / 32 = 0.62 at 100 % issue; frac_of_ceiling = frac / 0.62.  "
                         "clock_ghz / issue_utilisation: the kernel's PMC pass (GRBM_GUI_ACTIVE / 8 / duration; "
                         "4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x cycles)); frac_at_clock = frac x 2.4 / clock_ghz",
                 "formulation_ceiling_frac": 0.62}
    roof_valu["frac"] = roof_valu["achieved"] / roof_valu["peak"]
    roof_valu["frac_of_ceiling"] = roof_valu["frac"] / roof_valu["formulation_ceiling_frac"]
    ci = acs_clock_issue()
    if ci is not None:
        roof_valu["clock_ghz"] = ci["clock_ghz"]
        roof_valu["issue_utilisation"] = ci["valu_issue_utilisation"]
        roof_valu["frac_at_clock"] = roof_valu["frac"] * 2.4 / ci["clock_ghz"]
        roof_valu["clock_source"] = ci["source"]
    if tm_alone.get(acs_stage):
        roof_valu["ms_per_launch"] = acs_ms
        roof_valu["ms_per_launch_alone"] = tm_alone[acs_stage]
        roof_valu["frac_alone"] = acs_ops / (tm_alone[acs_stage] * 1e-3) / 1e12 / VALU_PEAK_TOPS
    roof_hbm = {"kernel": f"{demod_kernel[5:]} (findIndex + FFT + DQPSK)", "bound": "hbm",
                "achieved": demod_bytes / (demod_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "traffic": pmc_traffic(demod_kernel, args.workload), "algorithmic_bytes": demod_bytes,
                "note": f"algorithmic bytes: {bps}*T_s of {args.iq_format} samples in + 2K soft bits out as RING8 "
                        "bytes (ibits + 127) per data symbol + the findIndex window's T_u samples per frame "
                        "(SURVEY 8(d)'s 26,560 B/symbol counts cf32 in, int16 out).  ms_per_launch is the launch's "
                        "span on its stream: the demod is queued once run r-2's ACS is done, so its span includes "
                        "the time its workgroups wait for the slots the running ACS still holds; frac_alone is the "
                        "kernel's own rate.  The demod is not HBM-bound: halving its input bytes (PCM16) left its "
                        "time alone unchanged (profiles/r05_iq_format_ab.txt); it answers partly to VALU count (its "
                        "SIMDs' VALU busy ~70 % of the time at the measured per-opcode rates; round 5's instruction "
                        "cuts, -16 % SQ_INSTS_VALU in the same dispatch, made it 8 % faster: "
                        "profiles/r05e_pmc_issue_c3.txt vs r05w_pmc_issue_c3.txt, DESIGN section 9)"}
    roof_hbm["frac"] = roof_hbm["achieved"] / roof_hbm["peak"]
    if tm_alone.get("demod"):
        roof_hbm["ms_per_launch"] = demod_ms
        roof_hbm["ms_per_launch_alone"] = tm_alone["demod"]
        roof_hbm["frac_alone"] = demod_bytes / (tm_alone["demod"] * 1e-3) / 1e9 / HBM_PEAK_GBS
    roofline = roof_valu if dom in ("msc_acs", "fic") else roof_hbm

    out = {
        "metric": "DAB Mode-I symbols/sec (and real-time ensembles/GPU) at 1/2/4/8 MI355X",
        "value": value, "unit": "symbols/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32 (OFDM) + u8 soft bits (ring) + u16x2 packed path metrics (Viterbi, exact)",
        "data": f"synthetic (dabsynth transmitter, 30 dB SNR, CFO {args.cfo:g} Hz, amplitude {AMPLITUDE}), "
                f"stored as {FORMAT_DESC[args.iq_format]}",
        "config": {"workload": wl_desc, "ensembles_per_gpu": E, "frames_per_step": F,
                   "parallelism": f"ensemble-shard x{world}", "iq_source": "rank-local",
                   "iq_format": args.iq_format, "cfo_hz": args.cfo, "msc_output": args.msc_format},
        "realtime_ensembles_per_gpu": value / world / RT_SYMBOLS,
        "roofline": roofline,
        "roofline_hbm_demod": roof_hbm,
        "kernel_ms_per_step": {k: v[0] for k, v in tm.items()},
        "kernel_ms_per_launch": {k: v[1] for k, v in tm.items()},
        "kernel_ms_per_launch_alone": tm_alone,
        "kernel_timing": "HIP events on each launch's stream over the timed steps (rocprofv3 --kernel-trace agrees)",
        "checked_step": checks[0] if world == 1 else checks,
        "dabplus_last_step": sf_ok,
        "gen_seconds": gen_s,
        "acquire_ms": {"streams": E, "ms": acquire_ms, "note": "initial null search of every stream (host-timed, first launch)"},
        # the whole step priced at the front end's algorithmic bytes
        "hbm_frac_step": value / world * SYMBOL_BYTES / (HBM_PEAK_GBS * 1e9),
        "hbm_frac_step_note": "BASELINE.md 4.4's definition: symbols/s per GPU x 26,560 B (8 T_s cf32 in + 2 x 3072 "
                              "int16 out per symbol) / 8 TB/s; the bytes the front end moves per symbol here: "
                              f"{bps} T_s in + 3072 out = {bps * TS + 3072} B",
    }
    if delivered is not None:
        out["delivered_symbols_per_s"] = delivered.pop("value")
        out["delivered"] = delivered
    if sync_loss is not None:
        out["sync_loss"] = sync_loss
    if c5 is not None:
        out["c5"] = c5
    if cpu is not None:
        t = cpu["tot"]
        out["cpu_baseline"] = {
            "value": cpu["value"], "unit": "symbols/s", "cores": cpu["cores"], "kind": cpu["kind"],
            "affinity_cores": cpu["affinity"], "omp_num_threads": cpu["omp"],
            "fft": "fp32 radix-4 Stockham (oracle orc_fft2048_f32, FFTW3f's precision class; FFTW3f absent)",
            "cpu_quota_cores": cpu["quota"],
            "sample": f"{cpu['cores']} workers pinned one per core (affinity lists {cpu['affinity']} of nproc "
                      f"{cpu['nproc']}, {cpu['cpu']}; the box's CPU share: OMP_NUM_THREADS {cpu['omp']}, cgroup "
                      f"quota {cpu['quota']} cores), each its own synthetic "
                      f"{args.workload.upper()} ensemble (24 frames per pass incl. the AFC's convergence, "
                      f"{len(SUBCH)} subch) for ~{args.cpu_seconds:.0f}s: {t['symbols']} symbols.  FIC/MSC Viterbi "
                      "+ depuncture = reference viterbi.cpp+spiral-sse.c+deconvolve.cpp, DAB+ = reference "
                      "reed-solomon.cpp+firecode-checker.cpp (compiled from /root/reference in oracle/_ref); OFDM = "
                      "the oracle's C restatement of ofdm-processor.cpp/ofdm-decoder.cpp/phasereference.cpp with "
                      "the reference's 2.048 M-entry oscillatorTable and an fp32 radix-4 FFT standing in for "
                      "FFTW3f (FFTW3f and Qt absent): kind 'port'",
            "stages_cpu_seconds": {"ofdm": t["t_ofdm"], "fic": t["t_fic"], "msc": t["t_msc"],
                                   "dabplus": t["t_dabplus"]},
            "decoded_mbit_per_s": (t["fic_bits"] + t["msc_bits"]) / cpu["secs"] / 1e6,
            "rs_codewords_per_s": t["rs_cw"] / cpu["secs"],
            "realtime_ensembles": cpu["value"] / RT_SYMBOLS,
        }
    if fed:
        # the C4 leg last (its RCCL communicator would slow the rank-local legs), under a
        # watchdog: a transfer that never completes must not cost the line -- every rank
        # leaves after --fed-timeout seconds, rank 0 printing the line with the leg's error
        import threading
        once = threading.Lock()          # the line is printed once: by the leg or by the watchdog

        def abandon():
            if not once.acquire(blocking=False):
                return
            if rank == 0:
                out["c4_fed"] = {"error": f"no result within {args.fed_timeout:g} s: the leg was abandoned"}
                print(json.dumps(out), flush=True)
            sys.stdout.flush()
            os._exit(3)                  # non-zero on every rank: a hung leg is a failed run
        guard = threading.Timer(args.fed_timeout, abandon)
        guard.daemon = True
        guard.start()
        pipe.close()
        diq.free()
        try:
            c4 = c4_fed_leg(dabamd, ctx, dist, rank, world, local, E, F, subs, SUBCH, dabplus, P, cs,
                            fed_ph, args.fed_format, args.fed_steps, truth, seed0, args.msc_format)
        except Exception as e:           # noqa: BLE001 -- recorded in the line, printed once below
            c4 = {"error": f"rank {rank}: {e!r}"[:300]}
        if not once.acquire(blocking=False):
            time.sleep(3600)             # the watchdog fired meanwhile: it prints and exits
        guard.cancel()
        out["c4_fed"] = c4
    if rank == 0:
        print(json.dumps(out))


def c5_leg(dabamd, Ensemble, ctx, steps, warmup, F, cfo, iq_format, msc_format, threads, seed0=7000):
    """BASELINE configs[4] beside the headline: 16 ensembles x 16 DAB+ subchannels (64 kbps
    EEP-3A) -- FIC + MSC Viterbi, superframe sync, RS(120,110), AU CRC -- on this GPU, with
    the streams resident in HBM as in the main leg; `steps` timed steps after `warmup`, then
    one step whose FIC, MSC and superframes of ensemble 0 are checked against the
    transmitted bits.  The same measurement as `bench.py --workload c5`, fewer steps."""
    subch, E, desc = WORKLOADS["c5"]
    fmt_code, bps, _ = FORMATS[iq_format]
    P = period_frames(F, True)
    ens = Ensemble(F * (warmup + steps + 1) + 1, subch=subch, snr_db=30.0, cfo_hz=cfo, amplitude=AMPLITUDE)
    stride = ens.length
    diq = ctx.buf(E * stride * bps)
    pipe = None
    try:
        truth = ens.generate_period(seed0, P, truth=True)
        truth.pop("iq")
        for g0 in range(0, E, 8):
            n = min(8, E - g0)
            per = ens.period_many(n, seed0=seed0 + g0, period=P, threads=threads)
            for e in range(n):
                raw = to_raw(per[e], iq_format)
                for p, q, m in ens.stream_pieces(P):
                    diq.upload_at(raw[2 * q:2 * (q + m)], ((g0 + e) * stride + p) * bps)
                del raw
            del per
        subs = [dabamd.Subch(s[0], s[1], s[2], s[3], 0 if s[4] else 1, dabamd.SUBCH_DABPLUS if s[5] else 0)
                for s in subch]
        pipe = dabamd.Pipeline(ctx, E, F, subs)
        pipe.set_iq_format(fmt_code)
        if msc_format == "packed":
            pipe.set_packed(True)
        pipe.acquire(diq, stride, [0] * E, [stride] * E)

        def step(download=False):
            r = pipe.run(diq, stride, [stride] * E, download=download)
            return r, pipe.dabplus(download=download)
        for _ in range(warmup):
            step()
        pipe.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        pipe.sync()
        el = time.perf_counter() - t0
        st0 = pipe.state(0)
        (fic, crc, msc, valid), dp = step(download=True)
        if pipe.packed:
            msc = np.unpackbits(msc, axis=-1)
        check = check_step(truth, P, st0, pipe.state(0), fic, crc, msc, valid, subch)
        info = dp[0]
        done = info["status"] == 3
        check["superframes"] = int(done.sum())
        check["au_crc_pass"] = int(sum(bin(int(x)).count("1") for x in info["au_crc_ok"][done]))
        check["cif_records"] = int((info["status"] >= 0).sum())
    finally:
        if pipe is not None:
            pipe.close()
        diq.free()
    return {"value": E * F * 76 * steps / el, "unit": "symbols/s", "ms_per_step": el / steps * 1e3, "steps": steps,
            "warmup": warmup, "workload": desc, "ensembles": E, "frames_per_step": F,
            "dabplus_subchannels": E * len(subch), "checked_step": check}


def c4_fed_leg(dabamd, ctx, dist, rank, world, local, E, F, subs, SUBCH, dabplus, P, cs, fed_ph, fmt, steps,
               truth, seed0, msc_format, warmup=2):
    """BASELINE configs[3] end to end: every rank decodes its E ensembles from samples rank
    0 sends it over RCCL (FedSplit: chunk k + 2 of every stream travels while step k
    decodes; the ranks' chunk phases reach rank 0 once, untimed -- rank 0 holds the
    recordings).  Each rank's stream buffer is a torch tensor the pipeline reads in place
    (dabgpu_pipe_set_iq_format).  Fails soft: an error on any rank before the timed
    steps is agreed on by all ranks and reported instead of a rate."""
    import torch
    fcode, bps, dt = FORMATS[fmt]
    err = None
    nch = warmup + steps + 4                             # + the checked step, the acquisition, 2 ahead
    stride_f = nch * cs
    try:
        dev = torch.device(f"cuda:{rank_device(local)}") if torch.cuda.is_available() else torch.device("cpu")
        mine = torch.from_numpy(fed_ph).to(dev)
        tdt = {np.uint8: torch.uint8, np.int16: torch.int16}[dt]
        fiq = torch.zeros((E, 2 * stride_f), dtype=tdt, device=dev)
    except Exception as e:                              # noqa: BLE001 -- reported in the line
        err = repr(e)[:300]
    if allreduce_max(dist, 1.0 if err else 0.0) > 0:
        return {"error": err or "another rank failed its setup"}
    src = gather_to_rank0(dist, rank, world, mine)      # setup: rank 0 now holds every rank's streams
    phases = fed_ph.shape[0]
    split = FedSplit(dist, rank, world, E, phases, src=src,
                     dst=lambda e, k: fiq[e, 2 * k * cs:2 * (k + 1) * cs])
    if rank == 0:                                       # rank 0 reads its own recordings in place
        for k in range(nch):
            fiq[:, 2 * k * cs:2 * (k + 1) * cs].copy_(src[0][k % phases])
    got = [nch if rank == 0 else 0]

    def feed(k):                                        # chunk k: begin ... end
        if k < nch:
            reqs = split.begin(k)
            return lambda: (split.end(reqs), got.__setitem__(0, max(got[0], k + 1)))
        return lambda: None
    for k in range(2):
        feed(k)()
    pipe = dabamd.Pipeline(ctx, E, F, subs)
    pipe.set_iq_format(fcode)
    if msc_format == "packed":
        pipe.set_packed(True)
    buf = _TorchBuf(fiq)

    def avail():
        return [min(stride_f, got[0] * cs)] * E

    def step(k, download=False):
        done = feed(k + 2)                               # chunk k + 2 travels while step k decodes
        r = pipe.run(buf, stride_f, avail(), download=download)
        if dabplus:
            pipe.dabplus(download=download)
        done()
        return r
    pipe.acquire(buf, stride_f, [0] * E, avail())
    for i in range(warmup):
        step(i)
    pipe.sync()
    barrier(dist)
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    pipe.sync()
    el = time.perf_counter() - t0
    barrier(dist)
    el = allreduce_max(dist, el)
    st0 = pipe.state(0)
    fic, crc, msc, valid = step(warmup + steps, download=True)
    if pipe.packed:
        msc = np.unpackbits(msc, axis=-1)
    check = check_step(truth, P, st0, pipe.state(0), fic, crc, msc, valid, SUBCH)
    check["rank"] = rank
    check["seed"] = seed0
    checks = gather_objects(dist, check)
    pipe.close()
    nbytes = E * cs * bps
    ms = el / steps * 1e3
    return {"value": world * E * F * 76 * steps / el, "unit": "symbols/s", "ms_per_step": ms, "steps": steps,
            "ensembles": world * E, "format": FORMAT_DESC[fmt], "backend": dist.get_backend(),
            "bytes_per_rank_per_step": nbytes, "GBps_per_destination": nbytes / (ms * 1e-3) / 1e9,
            "GBps_out_of_rank0": (world - 1) * nbytes / (ms * 1e-3) / 1e9,
            "checked_steps": checks,
            "note": "rank 0 holds every rank's recorded streams and sends each rank chunk k + 2 of ITS ensembles "
                    "(E grouped sends per destination: a scatter, each destination over its own xGMI link) while "
                    "step k decodes; the receivers' pipelines read the samples in place (u8/s16 converted in the "
                    "kernels' loads).  Link-bound by design: DESIGN.md section 7"}


class _HostOut:
    """pinned host memory (dabgpu_host_alloc) as a pipeline output buffer: the kernels write it
    through its device address (hipHostGetDevicePointer; the same address under ROCm's unified
    addressing, asked anyway)"""

    def __init__(self, hb):
        import ctypes as C
        hip = C.CDLL("libamdhip64.so")
        d = C.c_void_p()
        if hip.hipHostGetDevicePointer(C.byref(d), hb.ptr, 0) != 0 or not d.value:
            raise RuntimeError("pinned host buffer has no device address")
        self.hb, self.ptr = hb, d


def delivered_leg(dabamd, ctx, pipe, step, k0, steps, E, F, subch, dabplus, dist, truth, P, fic_bytes=True,
                  direct=False):
    """`steps` timed steps whose outputs are copied to pinned host memory (two sets,
    alternating like the pipeline's device outputs), each copy on its run's back-end
    stream behind the channel decoding (dabgpu_pipe_fetch), overlapping the next run --
    or (direct) written there by the decoders themselves: the run's FIC, CRC and MSC
    output pointers are dabgpu_host_alloc memory (zero copy; not with DAB+ subchannels,
    whose layer reads the MSC bytes back).
    The last step's host copy of ensemble 0 is checked against the transmitted bits."""
    pipe.sync()
    msc_packed = pipe.packed
    pipe.set_packed(dabamd.PACK_MSC | (dabamd.PACK_FIC if fic_bytes else 0))    # MSC bytes, FIBs as bytes
    ns = len(subch)
    fb = 96 if fic_bytes else 768                               # bytes per FIC block
    n_fic, n_crc = E * F * 4 * fb, E * F * 12
    n_msc = E * 4 * F * ns * pipe.msc_stride_packed
    nd = len(pipe.dp)
    if nd:                                                      # only the run's superframes travel
        pipe.set_dabplus_compact(True)
    n_sfi = E * 4 * F * nd * 16 if nd else 0                     # dabgpu_superframe records
    n_sf = E * nd * pipe.sf_slots * pipe.sf_stride if nd else 0  # compact: DABGPU_SF_SLOTS per subchannel
    total = n_fic + n_crc + n_msc + n_sfi + n_sf
    direct = direct and not nd
    if direct:
        hb = [dabamd.HostBuf(ctx, n) for _ in range(2) for n in (n_fic, n_crc, n_msc)]
        saved = pipe._outs
        pipe._outs = [tuple(_HostOut(hb[3 * q + r]) for r in range(3)) for q in range(2)]
    else:
        hb = [dabamd.HostBuf(ctx, total) for _ in range(2)]
    valids = [None, None]

    def one(k, i):
        valid, _ = step(k)
        valids[i & 1] = valid
        if direct:
            return
        h = hb[i & 1]
        o = 0
        for src, n in ((pipe.fic_d, n_fic), (pipe.crc_d, n_crc), (pipe.msc_d, n_msc)) + \
                (((pipe.sfi_d, n_sfi), (pipe.sf_d, n_sf)) if nd else ()):
            if n:
                pipe.fetch(h, src, n, o)
            o += n

    one(k0, 0)                                                  # untimed: the packed format's first run
    pipe.sync()
    barrier(dist)
    t0 = time.perf_counter()
    for i in range(steps - 1):
        one(k0 + 1 + i, i + 1)
    st0 = pipe.state(0)
    one(k0 + steps, steps)
    pipe.sync()
    el = allreduce_max(dist, time.perf_counter() - t0)
    barrier(dist)
    st1 = pipe.state(0)
    if direct:                                                  # the last run's own buffers
        fic = pipe.fic_d.hb.view(np.uint8, (E, F, 4, fb))
        crc = pipe.crc_d.hb.view(np.uint8, (E, F, 12))
        msc = pipe.msc_d.hb.view(np.uint8, (E, 4 * F, ns, pipe.msc_stride_packed))
    else:
        h = hb[steps & 1]
        fic = h.view(np.uint8, (E, F, 4, fb))
        crc = h.view(np.uint8, (E, F, 12), n_fic)
        msc = h.view(np.uint8, (E, 4 * F, ns, pipe.msc_stride_packed), n_fic + n_crc)
    if fic_bytes:
        fic = np.unpackbits(fic, axis=-1)
    msc = np.unpackbits(msc, axis=-1)
    check = check_step(truth, P, st0, st1, fic, crc, msc, valids[steps & 1], subch)
    pipe.sync()
    if direct:
        pipe._outs = saved
        pipe.fic_d, pipe.crc_d, pipe.msc_d = saved[0]
    for b in hb:
        b.free()
    pipe.set_packed(dabamd.PACK_MSC if msc_packed else 0)      # the timed legs' format again
    if nd:
        pipe.set_dabplus_compact(False)
    world = dist.get_world_size() if dist is not None else 1
    return {"value": world * E * F * 76 * steps / el, "ms_per_step": el / steps * 1e3, "steps": steps,
            "bytes_to_host_per_step": total, "pcie_GBps": total * steps / el / 1e9,
            "msc_format": "8 bits per byte, msb first (dabgpu_pipe_set_packed)",
            "fic_format": "FIB bytes, 96 per FIC block (DABGPU_PACK_FIC)" if fic_bytes else "1 bit per byte",
            "checked_last_step_from_host_memory": check, "mode": "direct" if direct else "fetch",
            "note": "FIC + CRC flags + packed MSC bytes" + (" + DAB+ superframe records and the run's "
                                                                 "superframe bytes (compact)" if nd else "")
                    + (" of every step written to pinned host memory by the decoders themselves (the run's "
                       "output pointers are dabgpu_host_alloc memory)" if direct else
                       " of every step copied to pinned host memory behind its run's channel decoding "
                       "(dabgpu_pipe_fetch), overlapping the next run")}


def sync_loss_leg(dabamd, ctx, pipe, step, k0, steps, E, F, stride, diq, dist, base_ms, fmt="f32"):
    """The price of a sync loss (ofdm-processor.cpp:354-357: findIndex fails -> notSynced,
    the null search from where the stream is).  Before step k0 + 2j + 1 of each mode, stream
    j gets an interferer over 300,000 samples (1.5 frames) in the middle of that step's
    frames: a carrier at +100 kHz whose PRS correlation is flat.  Mode "sync": the run waits
    for the stream's null search (k_acquire, one wave) and still delivers F frames of every
    stream; mode "async" (DABGPU_CTL_ACQ_ASYNC): the search runs in the background and the
    run goes on without that stream.  Reported: ms per step against the loss-free steps
    (base_ms), the hit per loss, and the frames decoded."""
    n = 300000
    rng = np.random.default_rng(11)
    ph = 2 * np.pi * 100e3 / 2048000 * np.arange(n)
    jam = np.empty((n, 2), np.float32)
    jam[:, 0] = AMPLITUDE * (np.cos(ph) + rng.normal(0, 0.1, n))
    jam[:, 1] = AMPLITUDE * (np.sin(ph) + rng.normal(0, 0.1, n))
    jam = to_raw(jam.reshape(-1), fmt)
    bps = FORMATS[fmt][1]
    res = {}
    j = 0
    for mode in ("sync", "async"):
        pipe.sync()
        pipe.control(dabamd.CTL_ACQ_ASYNC if mode == "async" else dabamd.CTL_ACQ_SYNC)
        # partial: a stream may not get back (below) -- the run still delivers the others
        step(k0, partial=True)                             # untimed
        k0 += 1
        frames0 = [pipe.state(s).cif_count // 4 for s in range(E)]
        pos0 = [pipe.state(s).next_pos for s in range(E)]
        losses = 0
        jammed = []
        for i in range(0, steps, 2):
            # stream j: the interferer half-way through the frames of step k0 + i + 1
            s = j % E
            at = pos0[s] + (i + 1) * F * TF + F // 2 * TF + 40000
            if at + n < stride:
                diq.upload_at(jam, (s * stride + at) * bps)
                losses += 1
                jammed.append(s)
            j += 1
        pipe.sync()
        barrier(dist)
        t0 = time.perf_counter()
        for i in range(steps):
            # A stream whose search starts where the end of a null is detected just too late
            # (the PRS's first 50 samples below 0.75 sLevel) restarts every T_F and can lock
            # onto the frame period for good -- the reference's ofdmProcessor::run does the
            # same on the same samples (the oracle never re-acquires either): that stream
            # runs out of samples, the others go on (partial)
            step(k0 + i, partial=True)
        pipe.sync()
        el = allreduce_max(dist, time.perf_counter() - t0)
        barrier(dist)
        k0 += steps
        st = [pipe.state(s) for s in range(E)]
        frames = sum(st[s].cif_count // 4 - frames0[s] for s in range(E))
        ms = el / steps * 1e3
        # lost for good: a search that reached the end of the stream's samples (a search still
        # running at the end of the leg is acquiring_at_end; one that found its null resumes)
        lost = [s for s in jammed if st[s].next_pos + TF > stride]
        res[mode] = {"steps": steps, "losses": losses, "ms_per_step": ms, "streams_not_back": len(lost),
                     "hit_ms_per_loss": (ms - base_ms) * steps / max(losses, 1),
                     "hit_steps_per_loss": (ms - base_ms) * steps / max(losses, 1) / base_ms,
                     "frames_decoded": int(frames), "frames_loss_free": E * F * steps,
                     "resyncs": int(sum(x.resyncs for x in st)), "acquiring_at_end": int(sum(x.acquiring for x in st))}
    pipe.sync()
    pipe.control(dabamd.CTL_ACQ_ASYNC)                     # the engine's default again
    res["base_ms_per_step"] = base_ms
    res["default_mode"] = "async"
    res["note"] = ("one stream every 2 steps loses sync (interferer over 1.5 frames, findIndex fails); sync "
                   "(DABGPU_CTL_ACQ_SYNC, the reference's order): the run waits for its null search (k_acquire); "
                   "async (DABGPU_CTL_ACQ_ASYNC, the engine's default since round 6): the search runs in the background "
                   "and that stream rejoins a later run (its frames delivered later, frame for frame the same); "
                   "streams_not_back: this rank's jammed streams whose search reached the end of their samples "
                   "(it locked onto the frame period -- the end of the null detected just after T_null + 50 samples "
                   "at every attempt -- as the reference's ofdmProcessor::run does on the same samples); searches "
                   "still running at the end of the leg are acquiring_at_end")
    return res


def _crc_flip():
    """the FIC output carries each FIB's CRC field inverted, as check_CRC_bits leaves it
    (dab-constants.h:316-317): xor-ing this restores the transmitted bits"""
    m = np.zeros(768, np.uint8)
    for q in range(3):
        m[256 * q + 240:256 * q + 256] = 1
    return m


class _TorchBuf:
    """a torch tensor's device memory seen as a dabamd buffer (same device and process)"""

    def __init__(self, t):
        import ctypes as C
        self.ptr = C.c_void_p(t.data_ptr())


if __name__ == "__main__":
    main()
