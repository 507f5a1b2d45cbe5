#!/usr/bin/env python3
"""Phase breakdown of the persistent thin-factor loop (k_thin_loop), diagnostics.

Runs the bench workload's thin factors (mode 2 of the resnet18 3x3 convs, I = 9) through
one all-thin admm_iteration_batched call with a TRACE=1 build (ADMMQ_LIB), then reads
every workgroup's summed phase ticks (s_memrealtime, 10 ns) and prints the mean and the
maximum over workgroups of each phase per iteration, overall and for the largest team."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq import _lib, synthetic  # noqa: E402
from admmq.admm import admm_iteration_batched  # noqa: E402

PHASES = ["stage P", "solve", "X+max", "bar1+mx", "thresholds", "s1 inserts", "s1 sums+flush", "bar2", "bins load",
          "suffix+S", "stage2", "finalize", "bar3", "slot reset", "stop test"]
NPH = 16
ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet18")
ap.add_argument("--iters", type=int, default=400)
ap.add_argument("--wide", action="store_true", help="64-column workgroups wherever allowed")
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
shapes = [(s.shape[2], s.rank()) for s in synthetic.MODELS[a.model]() if len(s.shape) == 3]
probs = []
for I, R in shapes:
    B = torch.randn(R, 2 * R, generator=g) / (2 * R) ** 0.5
    G = (B @ B.T + 0.5 * torch.eye(R)).to(dev)
    probs.append((torch.randn(I, R, generator=g).to(dev) * 0.1, torch.zeros(I, R, device=dev),
                  torch.randn(I, R, generator=g).to(dev), G))
with _lib.thin_loop("wide" if a.wide else True):
    admm_iteration_batched(probs, a.iters, 0.0, 4, "tensor_mseminmax_symmetric", check_spd=False)
torch.cuda.synchronize()
lib = _lib.load()
n = 1024
buf = (ctypes.c_ulonglong * (NPH * n))()
got = lib.admmq_debug_thin_loop_trace(buf, n)
lds = [(R + 31) // 32 * 32 for (_, R) in shapes]
order = sorted(range(len(shapes)), key=lambda i: -lds[i])   # the planner's team order (longest rows first)
team = []
for i in order:
    team += [i] * (lds[i] // 32)
nwg = len(team)
rows = [[buf[NPH * b + k] for k in range(NPH)] for b in range(min(nwg, got))]
its = max(r[NPH - 1] for r in rows)
print(f"{nwg} workgroups, {its} iterations")
big = [b for b in range(nwg) if lds[team[b]] == max(lds)]
for name, sel in (("all", range(nwg)), (f"largest teams (ld {max(lds)})", big)):
    print(name)
    tot = 0.0
    for k, ph in enumerate(PHASES):
        v = [rows[b][k] * 0.01 / max(rows[b][NPH - 1], 1) for b in sel]
        tot += sum(v) / len(v)
        print(f"  {ph:14s} mean {sum(v) / len(v):7.2f} us  max {max(v):7.2f} us")
    print(f"  {'sum':14s} mean {tot:7.2f} us per iteration")
