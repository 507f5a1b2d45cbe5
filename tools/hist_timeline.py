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
ap.add_argument("--shapes", default="", help="I:R,I:R,... instead of the resnet18 factors of --mode")
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
probs = []
shapes = ([tuple(int(v) for v in x.split(":")) for x in a.shapes.split(",")] if a.shapes else
          [(s.shape[a.mode], s.rank()) for s in synthetic.resnet18_layers()])
for I, R in shapes:
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
    print(f"  {name:13s} avg {sum(d)/len(d):7.2f}  max {max(d):7.2f}  min {min(d):7.2f} us")
starts = sorted((r[0] - t0) / 100 for r in rows)
print("  start offsets: median %.2f  90%% %.2f  max %.2f us" % (starts[len(starts) // 2], starts[int(0.9 * len(starts))], starts[-1]))
if fused and hasattr(lib, "admmq_debug_fin_trace"):
    fb = (ctypes.c_ulonglong * (5 * n))()
    lib.admmq_debug_fin_trace(fb, n)
    fr = [([fb[5 * b + j] for j in range(5)], rows[b]) for b in range(len(rows))]
    fr = [(f, r) for f, r in fr if f[0] >= r[4] and f[3] >= f[0]]
    if fr:
        print(f"  finalize sub-phases over {len(fr)} blocks:")
        # stamps 2 / 3 (row-max barrier, split stores) exist only in the split solve form;
        # elsewhere column 2 holds a stale value of an earlier launch, so the phases between
        # stamp 1 and the end are reported as one
        split = all(f[1] <= f[2] <= f[3] for f, _ in fr)
        sub = [("start->rho", None, 0), ("rho->loads done", 0, 4), ("elements+stores", 4, 1)]
        sub += ([("rowmax barrier", 1, 2), ("split stores", 2, 3), ("residuals+end", 3, None)] if split
                else [("residuals+end", 1, None)])
        for name, a0, a1 in sub:
            d = [((f[a1] if a1 is not None else r[5]) - (f[a0] if a0 is not None else r[4])) / 100 for f, r in fr]
            print(f"    {name:16s} avg {sum(d)/len(d):6.2f}  max {max(d):6.2f} us")
sfn = getattr(lib, "admmq_debug_setup_trace", None)
if sfn is not None:
    sb = (ctypes.c_ulonglong * (5 * n))()
    sg = sfn(sb, n)
    sr = [[sb[5 * b + k] for k in range(5)] for b in range(sg) if sb[5 * b] and sb[5 * b + 4] >= sb[5 * b]]
    if sr:
        print(f"  setup sub-phases over {len(sr)} blocks (kernel start -> setup start avg "
              f"{sum((s[0] - r[0]) / 100 for s, r in zip(sr, rows)) / len(sr):.2f} us):")
        for k, nm in enumerate(["thresholds+scatter", "ties", "check+L+cells", "(fallback)"]):
            d = [(r[k + 1] - r[k]) / 100 for r in sr]
            print(f"    {nm:18s} avg {sum(d) / len(d):6.2f}  max {max(d):6.2f} us")
# the CU of each block: (XCC_ID << 32) | HW_ID from admmq_debug_hist_cu (column 5 of the
# fused kernel's trace is a time stamp, not a CU id); key (XCC, SE, SH, CU) as gemm_timeline.py
cfn = getattr(lib, "admmq_debug_hist_cu", None)
if cfn is not None:
    cb = (ctypes.c_ulonglong * n)()
    cfn(cb, n)
    cus = {}
    for b in range(len(rows)):
        hid = cb[b]
        hw = hid & 0xFFFFFFFF
        cus.setdefault(((hid >> 32) & 0xFF, (hw >> 13) & 0x7, (hw >> 12) & 1, (hw >> 8) & 0xF), []).append(b)
    per = sorted(len(v) for v in cus.values())
    print(f"  CUs used {len(cus)}; blocks per CU max {per[-1]}; CUs with 1 / 2 / >2 blocks: "
          f"{per.count(1)} / {per.count(2)} / {sum(1 for x in per if x > 2)}")

pb = (ctypes.c_ulonglong * (5 * 256))()
gp = lib.admmq_debug_prep_trace(pb, 256) if hasattr(lib, "admmq_debug_prep_trace") else 0
pr = [[pb[5 * b + j] for j in range(5)] for b in range(gp)]
pr = [r for r in pr if r[0] and r[3] >= r[0]]
if pr:
    print(f"prep2 blocks {len(pr)}")
    for name, j0, j1 in (("fill", 0, 1), ("sort", 1, 2), ("positions", 2, 3), ("total", 0, 3)):
        d = [(r[j1] - r[j0]) / 100 for r in pr]
        print(f"  {name:10s} avg {sum(d)/len(d):7.2f}  max {max(d):7.2f} us")
