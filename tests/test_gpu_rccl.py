"""The RCCL ("nccl") branch of the C4 stream split's transport on device tensors
(bench.p2p_batch, the grouped batch_isend_irecv that FedSplit and gather_to_rank0 use),
exercised on the one GPU a test box has: a one-rank RCCL process group sending chunks to
itself in one group, as rank 0 does to every peer.  The multi-rank split itself is covered
by tests/test_multiproc.py (gloo, world size 2 and 3) and by the bench rehearsals; this
checks that the same code path runs under RCCL with device tensors and delivers the bytes."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, torch, torch.distributed as td
sys.path.insert(0, ROOT)
import bench
torch.cuda.set_device(0)
td.init_process_group(backend="nccl")
assert td.get_backend() == "nccl"
g = torch.Generator(device="cpu").manual_seed(5)
# the wire format of the split: u8 .raw chunks (one stream's chunk per send), s16 too
for dt in (torch.uint8, torch.int16):
    src = [torch.randint(0, 255, (4097 + 64 * e,), generator=g).to(dt).cuda() for e in range(6)]
    dst = [torch.zeros_like(t) for t in src]
    reqs = bench.p2p_batch(td, [(t, 0) for t in src], [(t, 0) for t in dst])
    for r in reqs:
        r.wait()
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(src, dst)), dt
# FedSplit.end's wait + stream sync on the receiving side, and the setup gather
got = bench.gather_to_rank0(td, 0, 1, src[0])
assert got is not None and len(got) == 1 and torch.equal(got[0], src[0])
print("RCCL_P2P_OK", torch.cuda.get_device_name(0))
td.destroy_process_group()
"""


@pytest.mark.gpu
def test_p2p_batch_runs_over_rccl_on_device_tensors():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + SCRIPT], env=env, capture_output=True,
                       text=True, timeout=180)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0 and "RCCL_P2P_OK" in r.stdout
