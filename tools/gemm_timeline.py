#!/usr/bin/env python3
"""Per-workgroup timeline of one grouped-GEMM launch (diagnostics).

Runs the resnet18 mode-`--mode` factor problems of the bench workload through
admm_iteration_batched for a few iterations, then reads the last GEMM launch's
per-block {start, end, XCC, HW_ID} trace and prints the kernel span, per-CU busy
time and how blocks were placed."""
import argparse
import collections
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
ap.add_argument("--ksplit-form", type=int, default=1)
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
_lib.check(_lib.load().admmq_debug_set_ksplit_form(a.ksplit_form), "ksplit_form")
admm_iteration_batched(probs, a.iters, 0.0, 4, "tensor_mseminmax_symmetric", check_spd=False)
torch.cuda.synchronize()
lib = _lib.load()
lib.admmq_debug_gemm_trace.restype = ctypes.c_int32
n = 8192
buf = (ctypes.c_ulonglong * (4 * n))()
got = lib.admmq_debug_gemm_trace(buf, n)
recs = []
clk = []
for b in range(got):
    t0, t1, hid = buf[4 * b], buf[4 * b + 1], buf[4 * b + 2]
    if t1 > t0:
        clk.append(buf[4 * b + 3] / ((t1 - t0) / 100.0) / 1e3)   # shader cycles per us -> GHz
    if t0 == 0 or t1 < t0:   # grid padding (empty tiles leave no record)
        continue
    wg = (hid >> 48) & 0x7FFF
    nk = (hid >> 40) & 0xFF
    xcc = (hid >> 32) & 0xFF
    hw = hid & 0xFFFFFFFF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    recs.append((b, t0, t1, xcc, se, sh, cu, wg, nk))
# K-split phases (k_gemm_f32b, TRACE builds): K-loop end and combine end per workgroup
buf2 = (ctypes.c_ulonglong * (2 * n))()
lib.admmq_debug_gemm_trace2.restype = ctypes.c_int32
if lib.admmq_debug_gemm_trace2(buf2, n) > 0:
    ph = collections.defaultdict(list)
    for (b, s0, s1, *_r) in recs:
        tk, tc = buf2[2 * b], buf2[2 * b + 1]
        if tk >= s0 and tc >= tk and s1 >= tc and tk:
            done = "last/whole" if not (buf[4 * b + 2] >> 63) else "non-last piece"
            ph[done].append(((tk - s0) / 100, (tc - tk) / 100, (s1 - tc) / 100))
    for k, v in ph.items():
        m = [sum(x[i] for x in v) / len(v) for i in range(3)]
        print(f"{k}: n {len(v)}  K-loop {m[0]:.2f}  combine {m[1]:.2f}  epilogue {m[2]:.2f} us (means)")
t0 = min(r[1] for r in recs)
t1 = max(r[2] for r in recs)
print(f"tiles {len(recs)}  span {(t1 - t0) / 100:.2f} us (100 MHz ticks)")
clk.sort()
print(f"in-kernel shader clock (s_memtime / s_memrealtime) GHz: min {clk[0]:.3f} median {clk[len(clk) // 2]:.3f} max {clk[-1]:.3f}")
dur = [(r[2] - r[1]) / 100 for r in recs]
print(f"tile duration us: min {min(dur):.2f} avg {sum(dur)/len(dur):.2f} max {max(dur):.2f}")
print("first 8 tiles dur:", [round(x, 1) for x in dur[:8]], " last 8:", [round(x, 1) for x in dur[-8:]])
per_wg = collections.defaultdict(list)
for r in recs:
    per_wg[r[7]].append(r)
ends = sorted(((max(x[2] for x in v) - t0) / 100, k, len(v)) for k, v in per_wg.items())
print(f"workgroups {len(per_wg)}; latest-finishing (us, wg, ntiles):", [(round(e, 1), k, n) for e, k, n in ends[-6:]])
for e, k, n in ends[-3:]:
    v = sorted(per_wg[k], key=lambda x: x[1])
    print("  wg", k, "tiles:", [(x[0], round((x[1] - t0) / 100, 1), round((x[2] - x[1]) / 100, 1)) for x in v])
per_cu = collections.defaultdict(set)
for r in recs:
    per_cu[(r[3], r[4], r[5], r[6])].add(r[7])
cnt = collections.Counter(len(v) for v in per_cu.values())
print("workgroups per CU histogram:", dict(sorted(cnt.items())), "CUs", len(per_cu))
# placement check for the CU-balanced tile order: do workgroups b and b + 256 share a CU?
where = {r[7]: (r[3], r[4], r[5], r[6]) for r in recs}
pairs = [(b, b + 256) for b in range(max(where) + 1) if b + 256 in where and b in where]
same = sum(1 for a, b in pairs if where[a] == where[b])
print(f"placement: workgroups b and b+256 on the same CU for {same}/{len(pairs)} pairs; "
      f"same XCD for {sum(1 for a, b in pairs if where[a][0] == where[b][0])}/{len(pairs)}")

# per-CU view: K-steps carried, first start, last end (the launch is as long as the last CU)
cus = collections.defaultdict(list)
for r in recs:
    cus[(r[3], r[4], r[5], r[6])].append(r)
rows = []
for k, v in cus.items():
    ks = sum(x[8] for x in v)
    rows.append(((max(x[2] for x in v) - t0) / 100, (min(x[1] for x in v) - t0) / 100, ks, len(v)))
rows.sort()
import statistics
print(f"CUs {len(rows)}; K-steps per CU: max {max(r[2] for r in rows)} mean {statistics.mean(r[2] for r in rows):.1f}")
print("CU end times (us) percentiles 0/10/50/90/100:",
      [round(rows[int(q * (len(rows) - 1))][0], 1) for q in (0, 0.1, 0.5, 0.9, 1.0)])
print("CU first-start (us) max:", round(max(r[1] for r in rows), 2))
# us per K-step of a CU = end / K-steps (all tiles of a CU start at ~0)
rate = sorted(r[0] / r[2] for r in rows if r[2])
print("us per K-step per CU (64x64x32 units) percentiles 0/50/100:", [round(rate[int(q * (len(rate) - 1))], 3) for q in (0, .5, 1)])
by_load = collections.defaultdict(list)
for r in rows:
    by_load[r[2]].append(r[0])
print("end time by CU load (K-steps: mean end us, n):", {k: (round(statistics.mean(v), 1), len(v)) for k, v in sorted(by_load.items())})
tile_rate = collections.defaultdict(list)
for r in recs:
    tile_rate[r[8]].append((r[2] - r[1]) / 100)
print("tile duration by K-steps (mean us, n):", {k: (round(statistics.mean(v), 1), len(v)) for k, v in sorted(tile_rate.items())})

# per-CU tail: the CU's last K-loop end (k_gemm_f32b TRACE builds) against its last tile end,
# i.e. how long a CU runs after its MFMA work is over (epilogues, stores, atomics)
if lib.admmq_debug_gemm_trace2(buf2, n) > 0:
    tails, lastk = [], []
    for k, v in cus.items():
        tks = [buf2[2 * x[0]] for x in v if buf2[2 * x[0]] >= x[1]]
        if not tks:
            continue
        tk = max(tks)
        tails.append((max(x[2] for x in v) - tk) / 100)
        lastk.append((tk - t0) / 100)
    tails.sort()
    lastk.sort()
    print("CU tail after its last K-loop end (us) percentiles 0/10/50/90/100:",
          [round(tails[int(q * (len(tails) - 1))], 2) for q in (0, 0.1, 0.5, 0.9, 1.0)])
    print("CU last K-loop end (us) percentiles 0/10/50/90/100:",
          [round(lastk[int(q * (len(lastk) - 1))], 1) for q in (0, 0.1, 0.5, 0.9, 1.0)])

# SIMDs each workgroup's four waves ran on (k_gemm_f32b TRACE builds): a CU's 1..3 resident
# tiles put their waves on distinct SIMDs, or do some share one?
sfn = getattr(lib, "admmq_debug_gemm_simd", None)
if sfn is not None:
    nmax = 8192
    sb = (ctypes.c_uint * nmax)()
    if sfn(sb, nmax) > 0:
        nsimd = collections.Counter(bin(sb[r[0]]).count("1") for r in recs)
        print("distinct SIMDs per workgroup (4 waves):", dict(sorted(nsimd.items())))
        lone = [bin(sb[v[0][0]]).count("1") for v in cus.values() if len(v) == 1]
        if lone:
            print("  workgroups alone on their CU:", dict(sorted(collections.Counter(lone).items())))
