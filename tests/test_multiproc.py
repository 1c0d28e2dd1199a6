"""bench.py's multi-process path on CPU: world_size 2 over gloo (127.0.0.1).

Covers what the N-GPU bench relies on: torch.distributed rendezvous from the
launcher's env vars, the start/stop barrier, the max-over-ranks time, the disjoint
per-rank ensemble seeds (rank-local mode: each rank decodes its own ensembles) and
the C4 stream split (the c4_fed leg) through the bench's own code (bench.chunk_phases,
bench.gather_to_rank0, bench.FedSplit): every rank's recorded streams (u8 .raw and s16
.sdr) reach rank 0, which sends each rank chunk k of its OWN ensembles into its stream
buffer per step; every rank must receive exactly its own streams, byte for byte, which
must decode (oracle) to its own transmitted FIBs, and the per-rank checks gather on
every rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "sdr-j-dab_amd")]
    import bench
    import oracle_py as orc
    from dabamd.synth import Ensemble
    r, local, w, dist = bench.dist_setup(world)
    assert (r, local, w) == (rank, rank, world) and dist is not None
    assert dist.get_backend() == "gloo"
    seed0 = bench.rank_seed0(rank, 4)
    g = Ensemble(1, snr_db=300.0).generate(seed0)
    n, info, soft = orc.ofdm_run(g["iq"], 1)
    bench.barrier(dist)
    el = 0.5 + rank                      # this rank's "elapsed time"
    m = bench.allreduce_max(dist, el)
    bench.barrier(dist)
    q.put((rank, m, seed0, n, hash(soft[:n].tobytes())))
    dist.destroy_process_group()


def _split_worker(rank, world, port, q, fmt):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "sdr-j-dab_amd")]
    import torch
    import bench
    import oracle_py as orc
    from dabamd.synth import Ensemble
    r, local, w, dist = bench.dist_setup(world)
    E, F = 2, 2
    ens = Ensemble(7, snr_db=30.0, amplitude=bench.AMPLITUDE)
    stride = ens.length
    P = bench.period_frames(F, False)
    cs, nchunks = bench.chunk_layout(stride, F)
    seed0 = bench.rank_seed0(rank, E)
    # the bench's own C4 feed: every rank's chunk phases reach rank 0 (setup), then rank 0
    # sends each rank chunk k of its OWN streams straight into that rank's stream buffer
    mine = torch.from_numpy(bench.chunk_phases(ens, P, cs, E, seed0, 2, fmt))
    src = bench.gather_to_rank0(dist, rank, world, mine)
    dt = {"u8": torch.uint8, "s16": torch.int16}[fmt]
    fiq = torch.zeros((E, 2 * nchunks * cs), dtype=dt)
    split = bench.FedSplit(dist, rank, world, E, mine.shape[0], src=src,
                           dst=lambda e, k: fiq[e, 2 * k * cs:2 * (k + 1) * cs])
    if rank == 0:
        for k in range(nchunks):
            fiq[:, 2 * k * cs:2 * (k + 1) * cs].copy_(src[0][k % mine.shape[0]])
    for k in range(nchunks):
        split.end(split.begin(k))
    got = fiq.numpy()
    per = ens.period_many(E, seed0=seed0, period=P, threads=2)
    want = np.stack([bench.to_raw(ens.stream_from_period(per[e], P), fmt) for e in range(E)])
    same = bool(np.array_equal(got[:, :2 * stride], want))           # byte-identical
    # the received samples, read back as the format's reader does, decode to this rank's
    # own transmitted bits
    truth = ens.generate_period(seed0, P, truth=True)
    g0 = got[0, :2 * stride]
    iq = (g0.astype(np.float32) / 32768.0) if fmt == "s16" else ((g0.astype(np.float32) - 128.0) / 128.0)
    ref = orc.decode_stream(iq, 7, [])
    flip = np.zeros(768, np.uint8)
    for b in range(3):
        flip[256 * b + 240:256 * b + 256] = 1
    fic_ok = ref["n"] >= 6 and ref["crc"][:ref["n"]].all() and all(
        np.array_equal(ref["fic"][f, b] ^ flip, truth["fic"][f % P, b]) for f in range(ref["n"]) for b in range(4))
    bench.barrier(dist)
    checks = bench.gather_objects(dist, {"rank": rank, "fic_ok": bool(fic_ok)})
    q.put((rank, same, bool(fic_ok), hash(got.tobytes()), checks))
    dist.destroy_process_group()


@pytest.mark.parametrize("fmt,world", [("u8", 2), ("s16", 2), ("u8", 3)])
def test_stream_split_scatter_gloo(fmt, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q, fmt)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [{"rank": r, "fic_ok": True} for r in range(world)]
    for r, same, ok, h, checks in res:
        assert same                          # every rank got exactly its own streams, byte for byte
        assert ok                            # which decode to its own transmitted FIBs
        assert checks == want                # gathered checks, on every rank
    assert len({h for _, _, _, h, _ in res}) == world    # disjoint ensembles per rank


def test_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, m0, s0, n0, c0), (r1, m1, s1, n1, c1) = res
    assert m0 == m1 == 1.5                 # max over ranks, seen by every rank
    assert s0 != s1 and abs(s1 - s0) >= 4  # disjoint ensemble sets
    assert n0 == n1 == 1
    assert c0 != c1                        # independent inputs per rank
