#!/usr/bin/env python3
"""Phase durations of the fused small-job kernel (k_mse_small_admm) of the last launch of
one mode (diagnostics): loads, table setup, insert, suffix sums, selection, stage 2, finalize."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq import _lib, synthetic  # noqa: E402
from admmq.admm import admm_iteration_batched  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", type=int, default=2)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
probs = []
for s in synthetic.resnet18_layers():
    R, I = s.rank(), s.shape[a.mode]
    B = torch.randn(R, 2 * R, generator=g) / (2 * R) ** 0.5
    G = (B @ B.T + 0.5 * torch.eye(R)).to(dev)
    probs.append((torch.randn(I, R, generator=g).to(dev) * 0.1, torch.zeros(I, R, device=dev),
                  torch.randn(I, R, generator=g).to(dev), G))
admm_iteration_batched(probs, a.iters, 0.0, 4, "tensor_mseminmax_symmetric", check_spd=False)
torch.cuda.synchronize()
lib = _lib.load()
fn = lib.admmq_debug_small_trace
fn.restype = ctypes.c_int32
n = 64
buf = (ctypes.c_ulonglong * (9 * n))()
got = fn(buf, n)
rows = [[buf[9 * b + k] for k in range(9)] for b in range(got) if buf[9 * b] and buf[9 * b + 7] >= buf[9 * b]]
names = ["loads+flag", "setup", "insert", "suffix", "select", "stage 2", "finalize"]
print(f"blocks {len(rows)}  (R per problem: {[p[0].shape[1] for p in probs]})")
t0 = min(r[0] for r in rows)
for b, r in enumerate(rows):
    ph = " ".join(f"{(r[k + 1] - r[k]) / 100:6.2f}" for k in range(7))
    print(f"  blk {b:2d} start {(r[0] - t0) / 100:6.2f} end {(r[7] - t0) / 100:6.2f} nsel {r[8]:4d} | {ph}")
for k, nm in enumerate(names):
    d = [(r[k + 1] - r[k]) / 100 for r in rows]
    print(f"  {nm:12s} avg {sum(d) / len(d):6.2f}  max {max(d):6.2f} us")
