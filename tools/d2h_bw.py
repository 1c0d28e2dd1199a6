"""PCIe device-to-host bandwidth of the box (pinned host memory), for the delivered leg's
ceiling: one hipMemcpyAsync D2H of `mb` MB (dabgpu_pipe_fetch uses the same copy), timed
over reps, plus the same split into 4 concurrent copies on 4 streams (torch)."""
import sys
import time

import torch

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n = mb << 20
d = torch.empty(n, dtype=torch.uint8, device="cuda")
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
for _ in range(2):
    h.copy_(d, non_blocking=True)
torch.cuda.synchronize()
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"D2H {mb} MB pinned: {n / min(ts) / 1e9:.1f} GB/s (best of 5)")
ss = [torch.cuda.Stream() for _ in range(4)]
q = n // 4
ts = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, s in enumerate(ss):
        with torch.cuda.stream(s):
            h[i * q:(i + 1) * q].copy_(d[i * q:(i + 1) * q], non_blocking=True)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"D2H {mb} MB pinned on 4 streams: {n / min(ts) / 1e9:.1f} GB/s")
