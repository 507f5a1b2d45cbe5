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

# the EPC step (k_epc_step64: tridiagonalisation + Z = F Q + the mu search + X), n = 134, m = 64
fe = getattr(lib, "admmq_debug_epc_trace", None)
n, m = 134, 64
g = torch.Generator().manual_seed(5)
B = torch.randn(n, n + 8, generator=g, dtype=torch.float64)
G = (B @ B.T / (n + 8) + 1e-3 * torch.eye(n, dtype=torch.float64)).cuda()
F = torch.randn(m, n, generator=g, dtype=torch.float64).cuda()
X, W = torch.empty_like(F), torch.empty_like(F)
ls = float(torch.sum(F * torch.linalg.solve(G, F.T).T))
normY2, delta2 = ls * 1.5, ls * 0.5 * 2.5
mu = torch.zeros((), dtype=torch.float64, device="cuda")
st = _lib.stream_handle(F.device)
call = lambda: lib.admmq_epc_step64(_lib.ptr(G), _lib.ptr(F), m, n, normY2, delta2, _lib.ptr(mu), _lib.ptr(X),  # noqa: E731
                                    _lib.ptr(W), None, st)
for warm in (False, True):
    for _ in range(3):
        if not warm:
            mu.zero_()
        call()
    ev = (ctypes.c_ulonglong * 1)()
    lib.admmq_debug_epc_evals(ev, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        if not warm:
            mu.zero_()
        call()
    e1.record()
    torch.cuda.synchronize()
    lib.admmq_debug_epc_evals(ev, 1)
    print(f"epc_step64 n {n} m {m} {'warm' if warm else 'cold'}: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per call, "
          f"{ev[0] / 20:.1f} evaluations")
    if fe is not None and os.environ.get("ADMMQ_LIB", "").endswith("tracelib/libadmmq.so"):
        buf = (ctypes.c_ulonglong * 16)()
        fe(buf)
        t = [buf[k] for k in range(16)]
        print(f"  trace: load G {(t[1] - t[0]) / 100:.1f} us, tridiagonal {(t[2] - t[1]) / 100:.1f} us, "
              f"Z = F Q {(t[3] - t[2]) / 100:.1f} us, search {(t[4] - t[3]) / 100:.1f} us, X {(t[5] - t[4]) / 100:.1f} us")
        print(f"  tridiagonal phases (sums over the steps): barrier 1 wait {t[8] / 100:.1f} us, matvec {t[9] / 100:.1f} us, "
              f"barrier 2 wait {t[10] / 100:.1f} us, update {t[11] / 100:.1f} us, next reflector {t[12] / 100:.1f} us")
        print(f"  search phases (sums): LDL coefficients {t[13] / 100:.1f} us, row sums {t[14] / 100:.1f} us, "
              f"block sum {t[15] / 100:.1f} us")
