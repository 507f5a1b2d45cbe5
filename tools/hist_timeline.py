#!/usr/bin/env python3
"""Per-block phase timeline of one stage-1 (k_mse_hist) launch (diagnostics).

Same problem set as tools/gemm_timeline.py; prints, over the blocks of the last
hist launch, the phase durations {threshold fill, elements, flush+ticket, select}
and the kernel span."""
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
ap.add_argument("--iters", type=int, default=4)
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
probs = []
for s in synthetic.resnet18_layers():
    R = s.rank()
    I = s.shape[a.mode]
    B = torch.randn(R, 2 * R, generator=g) / (2 * R) ** 0.5
    G = (B @ B.T + 0.5 * torch.eye(R)).to(dev)
    F = torch.randn(I, R, generator=g).to(dev)
    H = torch.randn(I, R, generator=g).to(dev) * 0.1
    U = torch.zeros(I, R, device=dev)
    probs.append((H, U, F, G))
admm_iteration_batched(probs, a.iters, 0.0, 4, "tensor_mseminmax_symmetric", check_spd=False)
torch.cuda.synchronize()
lib = _lib.load()
n = 8192
buf = (ctypes.c_ulonglong * (6 * n))()
got = lib.admmq_debug_hist_trace(buf, n)
rows = []
for b in range(got):
    r = [buf[6 * b + j] for j in range(6)]
    if r[0] == 0 or r[4] < r[0]:
        break
    rows.append(r)
t0 = min(r[0] for r in rows)
t1 = max(r[4] for r in rows)
print(f"blocks {len(rows)}  span {(t1 - t0) / 100:.2f} us")
fused = any(r[5] for r in rows)
phases = (("setup/tables", 0, 1), ("elements", 1, 2), ("scan+flush+ticket", 2, 3), ("select+stage2", 3, 4), ("total", 0, 4))
if fused:   # fused finalize: column 4 = selection received, 5 = finalize done
    phases = (("setup/tables", 0, 1), ("elements", 1, 2), ("scan+flush+ticket", 2, 3),
              ("ticket->selection", 3, 4), ("finalize", 4, 5), ("total", 0, 5))
    t1 = max(r[5] for r in rows)
    print(f"  fused finalize: span to last finalize {(t1 - t0) / 100:.2f} us")
for name, j0, j1 in phases:
    d = [(r[j1] - r[j0]) / 100 for r in rows]
    print(f"  {name:13s} avg {sum(d)/len(d):7.2f}  max {max(d):7.2f} us")
starts = sorted((r[0] - t0) / 100 for r in rows)
print("  start offsets: median %.2f  90%% %.2f  max %.2f us" % (starts[len(starts) // 2], starts[int(0.9 * len(starts))], starts[-1]))
cus = {}
for r in rows:
    cus.setdefault(r[5], []).append(r)
print(f"  CUs used {len(cus)}; blocks per CU max {max(len(v) for v in cus.values())}")

pb = (ctypes.c_ulonglong * (5 * 256))()
gp = lib.admmq_debug_prep_trace(pb, 256) if hasattr(lib, "admmq_debug_prep_trace") else 0
pr = [[pb[5 * b + j] for j in range(5)] for b in range(gp)]
pr = [r for r in pr if r[0] and r[3] >= r[0]]
if pr:
    print(f"prep2 blocks {len(pr)}")
    for name, j0, j1 in (("fill", 0, 1), ("sort", 1, 2), ("positions", 2, 3), ("total", 0, 3)):
        d = [(r[j1] - r[j0]) / 100 for r in pr]
        print(f"  {name:10s} avg {sum(d)/len(d):7.2f}  max {max(d):7.2f} us")
