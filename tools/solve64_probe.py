#!/usr/bin/env python3
"""A few blocked EPC steps at R = 1141 (m = 512) for a kernel trace (rocprofv3 --kernel-trace
--stats -- python3 tools/solve64_probe.py): where one evaluation of the error equation spends
its time (csrc/solve64.hip)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq import panel  # noqa: E402

R, m = int(sys.argv[1]) if len(sys.argv) > 1 else 1141, 512
g = torch.Generator().manual_seed(R)
B = torch.randn(R, R + 8, generator=g, dtype=torch.float64)
G = (B @ B.T / (R + 8) + 1e-3 * torch.eye(R, dtype=torch.float64)).cuda()
F = torch.randn(m, R, generator=g, dtype=torch.float64).cuda()
info = torch.zeros(1, dtype=torch.int32, device="cuda")
X = panel.spd_solve64(G, F, info=info)
ls = float(torch.sum(F * X))
mu = torch.zeros((), dtype=torch.float64, device="cuda")
for _ in range(3):
    panel.epc_step64(G, F, ls * 1.5, ls * 1.25, mu.zero_(), info=info)
torch.cuda.synchronize()
print("ok", int(info), float(mu))
