#!/usr/bin/env python3
"""Where init_factors('parafac-epc') spends its time on the GPU (diagnostics): the
reference call (source/admm.py:40-44: als_maxiter=50, epc_maxiter=50, 50 EPC rounds) on
resnet18 layer1.0.conv1 (R = 134), with the number of CP-ALS iterations, EPC rounds and
EPC mode steps, and the time of one R x R eigendecomposition / solve on the device."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq import synthetic, parafac_epc as pe  # noqa: E402

idx, spec = synthetic.find_layer("resnet18", "layer1.0.conv1")
W = torch.from_numpy(synthetic.layer_weight(spec, idx)).cuda().double()
R = spec.rank()
calls = {"gram_mttkrp": 0, "eigh": 0, "solve": 0, "cp_anc": 0}
orig_gm, orig_eigh, orig_solve, orig_anc = pe.gram_mttkrp_f64, torch.linalg.eigh, torch.linalg.solve, pe.cp_anc


def gm(*a, **k):
    calls["gram_mttkrp"] += 1
    return orig_gm(*a, **k)


def eigh(*a, **k):
    calls["eigh"] += 1
    return orig_eigh(*a, **k)


def solve(*a, **k):
    calls["solve"] += 1
    return orig_solve(*a, **k)


def anc(*a, **k):
    calls["cp_anc"] += 1
    return orig_anc(*a, **k)


pe.gram_mttkrp_f64, torch.linalg.eigh, torch.linalg.solve, pe.cp_anc = gm, eigh, solve, anc
pe.parafac_epc(W, R, als_maxiter=2, epc_maxiter=2, epc_rounds=1)   # warm-up (kernels, library handles)
for k in calls:
    calls[k] = 0
torch.cuda.synchronize()
t0 = time.time()
lam, Us = pe.parafac_epc(W, R, als_maxiter=50, epc_maxiter=50)
torch.cuda.synchronize()
t = time.time() - t0
print(f"parafac_epc layer1.0.conv1 R={R}: {t:.2f} s; calls {calls}")
G = torch.randn(R, 2 * R, device="cuda", dtype=torch.float64)
G = G @ G.T
F = torch.randn(64, R, device="cuda", dtype=torch.float64)
for name, fn in (("eigh", lambda: orig_eigh(G)), ("solve", lambda: orig_solve(G, F.T)),
                 ("gram_mttkrp", lambda: orig_gm(W, [u.contiguous() for u in Us], 0))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    print(f"  {name}: {(time.time() - t0) / 50 * 1e3:.3f} ms per call")
t0 = time.time()
w, fs = pe.parafac(W, R, tol=1e-5, n_iter_max=50, normalize_factors=True)
torch.cuda.synchronize()
print(f"  parafac alone (50 its): {time.time() - t0:.2f} s")
