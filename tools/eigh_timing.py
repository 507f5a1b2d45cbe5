#!/usr/bin/env python3
"""Device time of the library path the EPC step keeps above R = 136 (admmq.parafac_epc
._epc_update: torch.linalg.eigh + the device mu search + two products) against the
one-workgroup tridiagonal step at R <= 136 (diagnostics for DESIGN §8)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq.parafac_epc import _epc_update  # noqa: E402

for R, m in ((134, 64), (183, 128), (566, 256), (1141, 512)):
    g = torch.Generator().manual_seed(R)
    B = torch.randn(R, R + 8, generator=g, dtype=torch.float64)
    G = (B @ B.T / (R + 8) + 1e-3 * torch.eye(R, dtype=torch.float64)).cuda()
    F = torch.randn(m, R, generator=g, dtype=torch.float64).cuda()
    ls = float(torch.sum(F * torch.linalg.solve(G, F.T).T))
    normY2, delta2 = ls * 1.5, ls * 0.5 * 2.5
    mu = torch.zeros((), dtype=torch.float64, device="cuda")
    for _ in range(2):
        _epc_update(G, F, normY2, delta2, mu)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(5):
        _epc_update(G, F, normY2, delta2, mu)
    torch.cuda.synchronize()
    print(f"EPC mode step R {R:5d} m {m:4d}: {(time.time() - t0) / 5 * 1e3:8.2f} ms per step "
          f"({'one-workgroup tridiagonal' if R <= 136 else 'torch eigh + device mu'})")
