#!/usr/bin/env python3
"""Device time of the one-workgroup fp64 solves (csrc/epc_kernels.hip) by size (diagnostics):
admmq_spd_solve64 for n in {32, 64, 96, 134} and m in {1, 64}, HIP-event timed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq import _lib  # noqa: E402

lib = _lib.load()
for n in (32, 64, 96, 134):
    for m in (1, 64):
        g = torch.Generator().manual_seed(n + m)
        B = torch.randn(n, 2 * n, generator=g, dtype=torch.float64)
        G = (B @ B.T / (2 * n) + 0.1 * torch.eye(n, dtype=torch.float64)).cuda()
        F = torch.randn(m, n, generator=g, dtype=torch.float64).cuda()
        X = torch.empty_like(F)
        st = _lib.stream_handle(F.device)
        for _ in range(3):
            lib.admmq_spd_solve64(_lib.ptr(G), _lib.ptr(F), m, n, _lib.ptr(X), None, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lib.admmq_spd_solve64(_lib.ptr(G), _lib.ptr(F), m, n, _lib.ptr(X), None, st)
        e1.record()
        torch.cuda.synchronize()
        print(f"spd_solve64 n {n:4d} m {m:3d}: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per call")

# phase stamps (TRACE build: ADMMQ_LIB=tools/tracelib/libadmmq.so)
import ctypes  # noqa: E402
fn = getattr(lib, "admmq_debug_spd_trace", None)
if fn is not None and os.environ.get("ADMMQ_LIB", "").endswith("tracelib/libadmmq.so"):
    for n in (64, 134):
        g = torch.Generator().manual_seed(n)
        B = torch.randn(n, 2 * n, generator=g, dtype=torch.float64)
        G = (B @ B.T / (2 * n) + 0.1 * torch.eye(n, dtype=torch.float64)).cuda()
        F = torch.randn(64, n, generator=g, dtype=torch.float64).cuda()
        X = torch.empty_like(F)
        lib.admmq_spd_solve64(_lib.ptr(G), _lib.ptr(F), 64, n, _lib.ptr(X), None, _lib.stream_handle(F.device))
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 16)()
        fn(buf)
        t = [buf[k] for k in range(16)]
        print(f"  inverse phases: pivot block + copy {t[8] / 100:.1f} us, row block B' {t[9] / 100:.1f} us, "
              f"rank-8 update {t[10] / 100:.1f} us (sums over the {(n + 7) // 8} block steps)")
        ghz = (t[7] - t[4]) / ((t[3] - t[0]) * 10.0)   # shader clocks per ns
        print(f"trace n {n}: load G {(t[1] - t[0]) / 100:.1f} us, inverse {(t[2] - t[1]) / 100:.1f} us, "
              f"products {(t[3] - t[2]) / 100:.1f} us; shader clock {ghz:.2f} GHz")
