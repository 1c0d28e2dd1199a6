"""bench.py's multi-process path on CPU: world_size 2 over gloo (127.0.0.1).

Covers what the N-GPU bench relies on: torch.distributed rendezvous from the
launcher's env vars, the start/stop barrier, the max-over-ranks time and the
disjoint per-rank ensemble seeds (each rank decodes its own ensembles; no
data-path collective).  Each rank also decodes its own tiny synthetic ensemble
through the oracle so the per-rank inputs are shown to be independent."""
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
