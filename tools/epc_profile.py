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
import ctypes  # noqa: E402
from admmq import _lib as _l  # noqa: E402
_ev = ctypes.c_ulonglong(0)
_l.load().admmq_debug_epc_evals(ctypes.byref(_ev), 1)
torch.cuda.synchronize()
t0 = time.time()
lam, Us = pe.parafac_epc(W, R, als_maxiter=50, epc_maxiter=50)
torch.cuda.synchronize()
t = time.time() - t0
_l.load().admmq_debug_epc_evals(ctypes.byref(_ev), 1)
print(f"parafac_epc layer1.0.conv1 R={R}: {t:.2f} s; calls {calls}; EPC error-equation evaluations {_ev.value}")
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

# the EPC step alone: error-equation evaluations per call and device time per call, on the G / F of
# one mode of the factors just computed (warm start = the previous call's mu)
import ctypes  # noqa: E402
from admmq import _lib, panel  # noqa: E402
from admmq.als import gram_mttkrp_f64  # noqa: E402
lib = _lib.load()
Y = W.permute(*sorted(range(3), key=lambda m: W.shape[m])).contiguous()
fs = [u.contiguous() for u in Us]
fs = [fs[m] for m in sorted(range(3), key=lambda m: W.shape[m])]
F, G = orig_gm(Y, fs, 1)
normY2 = float(torch.sum(Y * Y))
s = torch.linalg.eigvalsh(G)
for label, d2 in (("mu ~ 0 (flat)", None), ("mu ~ s", 1.0)):
    X0 = panel.spd_solve64(G, F)
    e0 = normY2 - float(torch.sum(F * X0))
    delta2 = e0 * 1.0001 if d2 is None else e0 + 0.5 * (normY2 - e0)
    mu = torch.zeros((), dtype=torch.float64, device="cuda")
    cnt = ctypes.c_ulonglong(0)
    lib.admmq_debug_epc_evals(ctypes.byref(cnt), 1)
    panel.epc_step64(G, F, normY2, delta2, mu)   # cold
    torch.cuda.synchronize()
    lib.admmq_debug_epc_evals(ctypes.byref(cnt), 1)
    cold = cnt.value
    t0 = time.time()
    for _ in range(20):
        panel.epc_step64(G, F, normY2, delta2, mu)   # warm (at the root)
    torch.cuda.synchronize()
    dt = (time.time() - t0) / 20
    lib.admmq_debug_epc_evals(ctypes.byref(cnt), 1)
    print(f"  epc_step64 {label}: mu {float(mu):.3e} (s {float(s.min()):.3e} .. {float(s.max()):.3e}); "
          f"evals cold {cold}, warm {cnt.value / 20:.1f}; {dt * 1e3:.3f} ms per warm call")
t0 = time.time()
for _ in range(50):
    panel.spd_solve64(G, F)
torch.cuda.synchronize()
print(f"  spd_solve64: {(time.time() - t0) / 50 * 1e3:.3f} ms per call")
