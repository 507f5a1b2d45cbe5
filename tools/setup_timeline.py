#!/usr/bin/env python3
"""Phase durations of the stage-1 table setup (h3_setup) of the last stage-1 launch of
one mode (diagnostics): {thresholds + host order, tie groups, L, cells}."""
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
ap.add_argument("--mode", type=int, default=0)
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
admm_iteration_batched(probs, 4, 0.0, 4, "tensor_mseminmax_symmetric", check_spd=False)
torch.cuda.synchronize()
lib = _lib.load()
fn = lib.admmq_debug_setup_trace
fn.restype = ctypes.c_int32
n = 4096
buf = (ctypes.c_ulonglong * (5 * n))()
got = fn(buf, n)
rows = [[buf[5 * b + k] for k in range(5)] for b in range(got) if buf[5 * b] and buf[5 * b + 4] >= buf[5 * b]]
names = ["thresholds+scatter", "ties", "check+L+cells", "(fallback)"]
print(f"blocks {len(rows)}")
for k, nm in enumerate(names):
    d = [(r[k + 1] - r[k]) / 100 for r in rows]
    print(f"  {nm:18s} avg {sum(d) / len(d):6.2f}  max {max(d):6.2f} us")
