#!/usr/bin/env python3
"""Per-block phase timeline of the last thin-factor solve launch (k_gemm_thin).

Runs the resnet18 mode-2 (I = 9) problems of the bench workload for a few ADMM
iterations and prints, relative to the earliest block start (100 MHz ticks -> us):
start, P/U/stop-test loads in, FMA done (M rows consumed), end, for all blocks and
for the finishing (last-arriving) blocks."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq import _lib, synthetic  # noqa: E402
from admmq.admm import admm_iteration_batched  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
probs = []
for s in synthetic.resnet18_layers():
    R = s.rank()
    I = s.shape[2]
    B = torch.randn(R, 2 * R, generator=g) / (2 * R) ** 0.5
    G = (B @ B.T + 0.5 * torch.eye(R)).to(dev)
    F = torch.randn(I, R, generator=g).to(dev)
    H = torch.randn(I, R, generator=g).to(dev) * 0.1
    probs.append((H, torch.zeros(I, R, device=dev), F, G))
for _ in range(2):
    admm_iteration_batched(probs, 6, 0.0, 4, "tensor_mseminmax_symmetric", check_spd=False)
torch.cuda.synchronize()
lib = _lib.load()
lib.admmq_debug_thin_trace.restype = ctypes.c_int32
n = 4096
buf = (ctypes.c_ulonglong * (5 * n))()
got = lib.admmq_debug_thin_trace(buf, n)
recs = []
for b in range(got):
    r = [buf[5 * b + k] for k in range(5)]
    if r[0] == 0:
        break
    recs.append((b, r[0], r[1], r[2], r[3], r[4] >> 32, r[4] & 0xFFFF))
t0 = min(r[1] for r in recs)


def stats(name, xs):
    xs = sorted(xs)
    print(f"  {name:22s} min {xs[0]:6.2f} med {xs[len(xs) // 2]:6.2f} max {xs[-1]:6.2f} us")


print(f"blocks {len(recs)}; span {(max(r[4] for r in recs) - t0) / 100:.2f} us")
for label, sel in (("all", recs), ("finishers", [r for r in recs if r[5]])):
    print(label, len(sel))
    stats("start", [(r[1] - t0) / 100 for r in sel])
    stats("loads in (P/U/test)", [(r[2] - t0) / 100 for r in sel])
    stats("FMA done", [(r[3] - t0) / 100 for r in sel])
    stats("end", [(r[4] - t0) / 100 for r in sel])
    stats("FMA - loads in", [(r[3] - r[2]) / 100 for r in sel])
    stats("end - FMA", [(r[4] - r[3]) / 100 for r in sel])
