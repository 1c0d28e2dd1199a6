"""bench.py -- DAB Mode-I symbols/s on MI355X (BASELINE.json metric, config C3).

Workload (config C3): E synthetic Mode-I ensembles per GPU (default 64), each with
9 UEP-3 128 kbit/s subchannels filling all 864 CUs.  One step decodes F frames
(default 8) of every ensemble through the full hot path: PRS sync (findIndex),
block-0 AFC, FFT + DQPSK + frequency de-interleave of 75 symbols, FIC
depuncture/Viterbi/PRBS/CRC, MSC 16-CIF time de-interleave + UEP depuncture +
Viterbi + PRBS for every subchannel.  IQ (cf32) is resident in HBM before the
timed region; the streams were acquired (null search) during warm-up.

Multi-GPU: one process per GPU; ensembles are sharded by rank (independent
streams, no data-path collective -> weak scaling); barrier + max-over-ranks
timing.  value = symbols decoded by all ranks / max time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sdr-j-dab_amd"))

RT_SYMBOLS = 76 / 0.096            # symbols/s of one real-time Mode-I ensemble (791.67)
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md chip table (spec)
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


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as td
        # RCCL when every local rank has its own GPU (the driver's 1..8-GPU node runs);
        # gloo when ranks share one (a rehearsal of the N > 1 path on a 1-GPU box) or
        # there is no GPU.  The path itself has no collective: only the start/stop
        # barriers and the max-over-ranks time go through torch.distributed.
        ngpu = torch.cuda.device_count()
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        backend = os.environ.get("DAB_DIST_BACKEND") or ("nccl" if ngpu >= lws and ngpu > 0 else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        td.init_process_group(backend=backend)
        dist = td
    return rank, local, world, dist


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
        dist.barrier()


def allreduce_max(dist, x):
    if dist is None:
        return x
    import torch
    dev = "cuda" if torch.cuda.is_available() and dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


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


def cpu_baseline(frames=2, budget_s=20.0, workers=None, workload="c3"):
    """Reference CPU path on the host cores: MSC/FIC depuncture+Viterbi through the
    reference's own compiled viterbi.cpp+spiral-sse.c+deconvolve.cpp (oracle/_ref);
    OFDM front end through the oracle's C restatement (FFTW3f absent).  One worker
    per core, each decoding its own synthetic ensemble for a bounded time."""
    import multiprocessing as mp
    workers = workers or min(16, os.cpu_count() or 1)
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(w, frames, budget_s, q, workload)) for w in range(workers)]
    for p in procs:
        p.start()
    res = [q.get() for _ in procs]
    for p in procs:
        p.join()
    syms = sum(r[0] for r in res)
    secs = max(r[1] for r in res)
    kind = "reference" if all(r[2] for r in res) else "port"
    return syms / secs, workers, kind, syms


def _cpu_worker(w, frames, budget_s, q, workload="c3"):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as orc
    from dabamd.synth import Ensemble
    ref = orc.ref()
    subch = WORKLOADS[workload][0]
    e = Ensemble(frames + 4, subch=subch, snr_db=300.0)
    g = e.generate(9000 + w, truth=False)
    prbs = orc.prbs(3072)
    t0 = time.perf_counter()
    done = 0
    while True:
        n, info, soft = orc.ofdm_run(g["iq"], frames + 4)
        cifs = soft[:, 3:75].reshape(4 * n, -1)
        for f in range(n):
            fic = soft[f, 0:3].reshape(-1)
            for b in range(4):
                orc.fic_process(fic[2304 * b:2304 * (b + 1)])
        mp4 = [orc.MP4(sc[2]) if sc[5] else None for sc in subch]
        for c in range(4 * n):
            for k, (sa, ln, br, pl, uep, dp) in enumerate(subch):
                frag = np.ascontiguousarray(cifs[c, sa * 64:(sa + ln) * 64])
                out = np.zeros(24 * br, np.uint8)
                if ref is not None:
                    if uep:
                        ref.ref_uep_deconvolve(br, pl, orc.P(frag), len(frag), orc.P(out))
                    else:
                        ref.ref_eep_deconvolve(br, pl, orc.P(frag), len(frag), orc.P(out))
                    out ^= prbs[:24 * br]
                else:
                    out = orc.msc_deconvolve(uep, br, pl, frag)
                if mp4[k] is not None:
                    mp4[k].add(out)
        done += n * 76
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    q.put((done, el, ref is not None))


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
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    rank, local, world, dist = dist_setup(args.gpus)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before this process touches the GPU: the workers are forked children
        cpu = cpu_baseline(budget_s=args.cpu_seconds, workload=args.workload)
    import dabamd
    from dabamd.synth import Ensemble

    SUBCH, E_default, wl_desc = WORKLOADS[args.workload]
    dabplus = any(s[5] for s in SUBCH)
    E, F = args.ensembles or E_default, args.frames
    total_frames = F * (args.warmup + args.steps + 1) + 1   # +1 step: the profiled pass
    ens = Ensemble(total_frames, subch=SUBCH, snr_db=30.0)
    ctx = dabamd.Context(rank_device(local))
    stride = ens.length
    # generated in groups straight into HBM: host memory stays at one group (~2 GB)
    # however many ensembles and frames the run decodes
    t0 = time.time()
    diq = ctx.buf(E * 2 * stride * 4)
    group = 8
    for g0 in range(0, E, group):
        n = min(group, E - g0)
        part = ens.generate_many(n, seed0=rank_seed0(rank, E) + g0, threads=min(16, os.cpu_count() or 1))
        diq.upload_at(part, g0 * 2 * stride * 4)
        del part
    gen_s = time.time() - t0
    subs = [dabamd.Subch(s[0], s[1], s[2], s[3], 0 if s[4] else 1, dabamd.SUBCH_DABPLUS if s[5] else 0)
            for s in SUBCH]
    pipe = dabamd.Pipeline(ctx, E, F, subs)
    pipe.acquire(diq, stride, [0] * E, [stride] * E)
    n_avail = [stride] * E

    def step(download=False):
        r = pipe.run(diq, stride, n_avail, download=download)
        if dabplus:
            return r, pipe.dabplus(download=download)
        return r, None

    for _ in range(args.warmup):
        step()
    pipe.sync()
    # per-kernel HIP events on each launch's stream over the timed steps (recording
    # adds no synchronisation); summed and counted by the pipeline
    pipe.set_profiling(2)
    barrier(dist)
    pipe.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    pipe.sync()
    el = time.perf_counter() - t0
    barrier(dist)
    el = allreduce_max(dist, el)
    tsum = pipe.timing()
    pipe.set_profiling(False)
    # kernel time per step and per launch over the timed region
    tm = {k: (v[0] / args.steps, v[0] / max(v[1], 1)) for k, v in tsum.items()}

    # one extra step (outside the timed region) whose outputs are checked
    (fic, crc, msc, valid), dp = step(download=True)
    crc_ok = float(crc.mean())
    sf_ok = None
    if dp is not None:
        info = dp[0]
        sf_ok = {"superframes": int((info["status"] == 3).sum()),
                 "au_crc_pass": int(sum(bin(int(x)).count("1") for x in info["au_crc_ok"][info["status"] == 3])),
                 "cif_records": int((info["status"] >= 0).sum())}

    symbols = world * E * F * 76 * args.steps
    value = symbols / el
    if rank != 0:
        return
    # dominant kernel + its roofline
    dom = max(tm, key=lambda k: tm[k][0])
    # the pipeline decodes the FIC in the MSC's ACS launch (dabgpu.h, DABGPU_STAGE_FIC)
    acs_steps = E * 4 * F * sum(24 * s[2] + 6 for s in SUBCH) + E * F * 4 * (768 + 6)
    # (without MSC subchannels the FIC has launches of its own, k_acs<2>)
    acs_stage, acs_kernel = ("msc_acs", "dab::k_acs2<3, 2>") if SUBCH else ("fic", "dab::k_acs<2>")
    acs_ms = max(tm[acs_stage][1], 1e-9)            # average launch duration
    acs_ops = acs_steps * 64 * 4                    # 2 adds + compare + select per ACS
    demod_ms = max(tm["demod"][1], 1e-9)
    demod_bytes = E * F * 75 * (8 * 2552 + 2 * 3072)
    roof_valu = {"kernel": f"{acs_kernel[5:]} (Viterbi ACS)", "bound": "valu", "achieved": acs_ops / (acs_ms * 1e-3) / 1e12,
                 "peak": VALU_PEAK_TOPS, "unit": "TOP/s", "traffic": pmc_traffic(acs_kernel, args.workload),
                 "note": "4 int ops per add-compare-select x 64 states per trellis step; peak = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz"}
    roof_valu["frac"] = roof_valu["achieved"] / roof_valu["peak"]
    roof_hbm = {"kernel": "k_demod_wg (FFT+DQPSK)", "bound": "hbm",
                "achieved": demod_bytes / (demod_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "traffic": pmc_traffic("dab::k_demod_wg<false>", args.workload), "algorithmic_bytes": demod_bytes,
                "note": "algorithmic bytes: 8*T_s cf32 in + 2*2K int16 out per data symbol"}
    roof_hbm["frac"] = roof_hbm["achieved"] / roof_hbm["peak"]
    roofline = roof_valu if dom in ("msc_acs", "fic") else roof_hbm

    out = {
        "metric": "DAB Mode-I symbols/sec (and real-time ensembles/GPU) at 1/2/4/8 MI355X",
        "value": value, "unit": "symbols/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32+u32",
        "data": "synthetic (dabsynth transmitter, 30 dB SNR)",
        "config": {"workload": wl_desc,
                   "ensembles_per_gpu": E, "frames_per_step": F, "parallelism": f"ensemble-shard x{world}"},
        "realtime_ensembles_per_gpu": value / world / RT_SYMBOLS,
        "roofline": roofline,
        "roofline_hbm_demod": roof_hbm,
        "kernel_ms_per_step": {k: v[0] for k, v in tm.items()},
        "kernel_ms_per_launch": {k: v[1] for k, v in tm.items()},
        "kernel_timing": "HIP events on each launch's stream over the timed steps (rocprofv3 --kernel-trace agrees)",
        "fic_crc_pass_rate": crc_ok,
        "dabplus_last_step": sf_ok,
        "gen_seconds": gen_s,
    }
    if cpu is not None:
        v, cores, kind, syms = cpu
        out["cpu_baseline"] = {"value": v, "unit": "symbols/s", "cores": cores, "kind": kind,
                               "sample": f"{cores} workers x own synthetic {args.workload.upper()} ensemble "
                                         f"(6 frames, {len(SUBCH)} subch), ~{args.cpu_seconds:.0f}s each, {syms} "
                                         "symbols total; Viterbi/depuncture = reference viterbi.cpp+spiral-sse.c+"
                                         "deconvolve.cpp, OFDM (and DAB+ RS/superframe) = oracle C restatement "
                                         "(FFTW3f absent)"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
