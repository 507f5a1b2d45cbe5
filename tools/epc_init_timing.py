#!/usr/bin/env python3
"""Time of the CP-ALS / EPC initialiser on the device (diagnostics for DESIGN §2.9 / §6):

  * per mode step at the resnet ranks above the one-workgroup limit (183 ... 1141): the
    CP-ALS solve (admmq.panel.spd_solve64, blocked) and the EPC update (the blocked step,
    cold and warm-started), with the number of error-equation evaluations per step;
  * init_factors('parafac-epc')'s call (source/admm.py:40-44: 50 ALS + 50 EPC iterations per
    round, up to 50 rounds) on resnet18 layer4.0.conv2 (512, 512, 9), R = 1141, with its mode
    step count;
  * all 16 resnet18 3x3 convs: one call of init_factors_many (one stream per layer) against
    the sum of the per-layer calls.

Writes one JSON object to stdout (profiles/r06_epc_init_timing.json). `--model-only`: only the
whole-model part (e.g. under GPU_MAX_HW_QUEUES=16, set before the process starts);
`--steps-only`: only the per-step part."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq import _lib, panel, synthetic, parafac_epc as pe  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
out = {"steps": [], "layer4": None, "model": None, "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
model_only = "--model-only" in sys.argv
steps_only = "--steps-only" in sys.argv


def evals(reset=False):
    v = ctypes.c_ulonglong(0)
    lib.admmq_debug_s64_evals(ctypes.byref(v), 1 if reset else 0)
    return v.value


def sync_time(fn, reps):
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    return (time.time() - t0) / reps * 1e3, r


for R, m in (() if model_only else ((183, 128), (278, 128), (566, 256), (1141, 512), (1141, 9))):
    g = torch.Generator().manual_seed(R)
    B = torch.randn(R, R + 8, generator=g, dtype=torch.float64)
    G = (B @ B.T / (R + 8) + 1e-3 * torch.eye(R, dtype=torch.float64)).to(dev)
    F = torch.randn(m, R, generator=g, dtype=torch.float64).to(dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    panel.spd_solve64(G, F, info=info)
    als_ms, X = sync_time(lambda: panel.spd_solve64(G, F, info=info), 10)
    ls = float(torch.sum(F * X))
    normY2, delta2 = ls * 1.5, ls * 0.5 * 2.5
    mu = torch.zeros((), dtype=torch.float64, device=dev)
    panel.epc_step64(G, F, normY2, delta2, mu, info=info)   # warm-up
    mu.zero_()
    evals(True)
    cold_ms, _ = sync_time(lambda: panel.epc_step64(G, F, normY2, delta2, mu.zero_(), info=info), 3)
    cold_ev = evals(True) / 3
    warm_ms, _ = sync_time(lambda: panel.epc_step64(G, F, normY2, delta2, mu, info=info), 5)
    warm_ev = evals(True) / 5
    rec = {"R": R, "m": m, "als_solve_ms": round(als_ms, 3), "epc_cold_ms": round(cold_ms, 3),
           "epc_cold_evals": cold_ev, "epc_warm_ms": round(warm_ms, 3), "epc_warm_evals": warm_ev, "info": int(info)}
    out["steps"].append(rec)
    print(rec, file=sys.stderr, flush=True)


count = {"gram_mttkrp": 0}
orig = pe.gram_mttkrp_f64


def counted(*a, **k):
    count["gram_mttkrp"] += 1
    return orig(*a, **k)


if steps_only:
    print(json.dumps(out))
    sys.exit(0)
pe.gram_mttkrp_f64 = counted
idx, spec = synthetic.find_layer("resnet18", "layer4.0.conv2")
W = torch.from_numpy(synthetic.layer_weight(spec, idx)).to(dev).double()
R = spec.rank()
if not model_only:
    evals(True)
    torch.cuda.synchronize()
    t0 = time.time()
    lam, Us = pe.parafac_epc(W, R, als_maxiter=50, epc_maxiter=50)
    torch.cuda.synchronize()
    t = time.time() - t0
    steps = count["gram_mttkrp"]
    Wc = W.cpu()
    err = float((Wc - pe._reconstruct(lam.cpu(), [u.cpu() for u in Us])).norm() / Wc.norm())
    out["layer4"] = {"layer": "layer4.0.conv2", "R": R, "seconds": round(t, 3), "mode_steps": steps,
                     "ms_per_mode_step": round(t / max(steps, 1) * 1e3, 3), "epc_evals": evals(True), "rel_err": err}
    print(out["layer4"], file=sys.stderr, flush=True)
pe.gram_mttkrp_f64 = orig

specs = synthetic.resnet18_layers()
Ws = [torch.from_numpy(synthetic.layer_weight(s, i)).to(dev).double() for i, s in enumerate(specs)]
ranks = [s.rank() for s in specs]
per = []
torch.cuda.synchronize()
for Wl, Rl in zip(Ws, ranks) if not model_only else ():
    t0 = time.time()
    pe.parafac_epc(Wl, Rl, als_maxiter=50, epc_maxiter=50)
    torch.cuda.synchronize()
    per.append(round(time.time() - t0, 3))
    print(f"layer R={Rl}: {per[-1]} s", file=sys.stderr, flush=True)
t0 = time.time()
res = pe.parafac_epc_many(Ws, ranks, als_maxiter=50, epc_maxiter=50)
torch.cuda.synchronize()
t_many = time.time() - t0
out["model"] = {"model": "resnet18 16 3x3 convs", "per_layer_s": per, "sequential_s": round(sum(per), 3),
                "concurrent_s": round(t_many, 3), "speedup": round(sum(per) / t_many, 2) if per else None}
print(json.dumps(out))
