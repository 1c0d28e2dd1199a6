"""bench.py's multi-process path on CPU: world_size 2 over gloo (127.0.0.1).

Covers what the N-GPU bench relies on: torch.distributed rendezvous from the
launcher's env vars, the start/stop barrier, the max-over-ranks time, the disjoint
per-rank ensemble seeds (rank-local mode: each rank decodes its own ensembles) and
the C4 stream split (--iq-source rccl): rank 0 holds the int16 IQ of the ranks'
ensembles in the chunk-major layout and scatters each chunk with one grouped
send/recv; every rank must receive its own streams byte-identical, and the
received chunks, converted back, must decode (oracle) like the rank's own IQ."""
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


def _split_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "sdr-j-dab_amd")]
    import torch
    import bench
    import oracle_py as orc
    from dabamd.synth import Ensemble
    r, local, w, dist = bench.dist_setup(world)
    E, F = 2, 1
    ens = Ensemble(3, snr_db=300.0)
    stride = ens.length
    cs, nchunks = bench.chunk_layout(stride, F)

    def chunked(seed0):
        iq = ens.generate_many(E, seed0=seed0, threads=2)
        p16 = np.zeros((E, nchunks * 2 * cs), np.int16)
        p16[:, :2 * stride] = bench.to_s16(iq)
        return torch.from_numpy(p16.reshape(E, nchunks, 2 * cs).transpose(1, 0, 2).copy())
    # rank 0 holds every rank's streams ([rank][chunk][ensemble][2*cs]); rank r decodes
    # the ensembles of seed rank_seed0(r)
    src = [chunked(bench.rank_seed0(d, E)) for d in range(world)] if rank == 0 else None
    recv = torch.zeros((E, 2 * cs), dtype=torch.int16)
    got = np.zeros((E, nchunks * 2 * cs), np.int16)
    for k in range(nchunks):
        reqs = bench.scatter_chunk(dist, rank, world, [src[d][k] for d in range(world)] if rank == 0 else None, recv)
        for q_ in reqs:
            q_.wait()
        got[:, 2 * k * cs:2 * (k + 1) * cs] = (src[0][k] if rank == 0 else recv).numpy()
    mine = chunked(bench.rank_seed0(rank, E)).numpy().transpose(1, 0, 2).reshape(E, -1)
    same = bool(np.array_equal(got, mine))
    iq = got[0, :2 * stride].astype(np.float32) / 32768.0
    n, info, soft = orc.ofdm_run(iq, 2)
    bench.barrier(dist)
    q.put((rank, same, n, hash(got.tobytes())))
    dist.destroy_process_group()


def test_stream_split_scatter_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, same0, n0, h0), (r1, same1, n1, h1) = res
    assert same0 and same1                   # every rank got exactly its own streams
    assert n0 == n1 == 2                     # and they decode
    assert h0 != h1                          # disjoint ensembles per rank


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
