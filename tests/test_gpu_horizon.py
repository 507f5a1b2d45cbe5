"""The benchmarked horizon (BASELINE configs C2 / C3): max_iter_admm = 1000 (999 inner
iterations per mode call, scripts/factorize.py:218-221) with eps = 0, the schedule
bench.py times. Shorter-horizon parity (one step bit-level, 30 steps at the largest R,
the 20 x 20 ALS band) is in test_gpu_parity.py; here the contract is what survives 999
chaotic iterations. The reference is not reproducible against itself at this horizon
(SURVEY.md §0, F8): F11 (tests/golden/gen_f11_horizon.py) re-ran the reference's own
admm_iteration on C2 from the same start at torch CPU thread counts {1, 2, 4, 8} (F4's
method: the thread count moves the summation order) and, at each, with its cholesky_solve
moved by <= 1 ulp (F8's proxy) - 24 runs - and its objective ||F - H G|| / ||F|| spreads over
~2 % (mode 0: 0.1581 ... 0.1610), so the contract is that band (widened by half its width,
the F10 rule), not a 1e-3 match to any one run:

  * C2 (resnet18 layer1.0.conv1, every mode from the same seed-42 start, F and G from the
    oracle): the reference's iteration count, every result on a 4-bit grid (<= 16 levels),
    and the 999-iteration result's objective and grid step inside the reference's F11 band;
    the CPU oracle's run of the same call (an independent float32 restatement) inside it
    too (mode 2: the reference's one-thread runs reach 0.11946, where the oracle lands);
  * C2 as one ALS sweep (the three modes in sequence, the reference loop): the sweep's
    reconstruction errors (rec_error, quant_rec_error) inside the reference's F11 sweep band;
  * C3 (all 16 resnet18 3x3 convs batched, the bench's step): property checks on every
    (layer, mode) - 999 iterations each, finite factors on <= 16 levels, finite losses
    below the random start's, no fused-path fault repaired.
"""
import json
import os

import numpy as np
import pytest

from conftest import gpu_available
from oracle import admm_oracle as ao

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

MSE = "tensor_mseminmax_symmetric"
MAX_ITER = 1000   # the bench's max_iter_admm: 999 inner iterations
F11 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "f11_horizon.json")


def _band(vals):
    """[min, max] of the reference's runs widened by half the width on each side (F10's rule)."""
    lo, hi = min(vals), max(vals)
    w = 0.5 * (hi - lo)
    return lo - w, hi + w


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    return torch, torch.device("cuda:0")


def _t(torch, dev, a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def _c2_start():
    import torch
    from admmq import synthetic
    idx, spec = synthetic.find_layer("resnet18", "layer1.0.conv1")
    W = synthetic.layer_weight(spec, idx)
    R = spec.rank()
    g = torch.Generator().manual_seed(42)
    fs = [torch.randn(n, R, generator=g).numpy() for n in W.shape]
    return W, R, fs


def _levels(h):
    lv = np.unique(h)
    assert np.all(np.isfinite(lv))
    assert len(lv) <= 16, len(lv)   # 4 bits
    return float(np.min(np.diff(lv))) if len(lv) > 1 else 0.0


def _objective(F, G, h):
    F64 = F.astype(np.float64)
    return float(np.linalg.norm(F64 - h.astype(np.float64) @ G.astype(np.float64)) / np.linalg.norm(F64))


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_c2_mode_call_at_bench_horizon(torch_dev, mode):
    torch, dev = torch_dev
    from admmq import admm_iteration_batched
    ref = json.load(open(F11))["modes"][str(mode)]
    W, R, fs = _c2_start()
    G, F = ao.gram_mttkrp(W, fs, mode)
    H0 = fs[mode]
    p = (_t(torch, dev, H0), torch.zeros(H0.shape, device=dev), _t(torch, dev, F), _t(torch, dev, G))
    (H,), info = admm_iteration_batched([p], MAX_ITER, 0.0, 4, MSE, return_info=True)
    H, U = H.cpu().numpy(), p[1].cpu().numpy()
    assert int(info[0, 0]) == MAX_ITER - 1   # eps = 0: the reference runs every iteration
    assert int(info[0, 2]) == 0 and int(info[0, 3]) == 0   # no SPD error, no internal fault
    assert np.all(np.isfinite(U))
    og, sg = _objective(F, G, H), _levels(H)
    Ho, _, oinfo = ao.admm_iteration(H0, np.zeros_like(H0), F, G, MAX_ITER, 0.0, 4, MSE, return_info=True)
    assert oinfo["iters"] == MAX_ITER - 1
    oo, so = _objective(F, G, Ho), _levels(Ho)
    lo, hi = _band(ref["objective"])
    slo, shi = _band(ref["grid_step"])
    print(f"C2 mode {mode}, {MAX_ITER - 1} its: objective gpu {og:.6e}, oracle {oo:.6e}, "
          f"reference runs {min(ref['objective']):.6e} .. {max(ref['objective']):.6e}; grid step gpu {sg:.4e}, "
          f"oracle {so:.4e}, reference {min(ref['grid_step']):.4e} .. {max(ref['grid_step']):.4e}")
    meta = json.load(open(F11))
    assert meta["threads"] == [1, 2, 4, 8] and len(ref["objective"]) == len(meta["runs"]) == 24
    assert lo <= og <= hi, (og, lo, hi)
    assert slo <= sg <= shi, (sg, slo, shi)
    assert lo <= oo <= hi and slo <= so <= shi, (oo, so, lo, hi, slo, shi)   # the oracle is inside too


def test_c2_sweep_at_bench_horizon(torch_dev):
    torch, dev = torch_dev
    from admmq.factorize import LayerRun, als_sweep
    ref = json.load(open(F11))["sweep"]
    W, R, fs = _c2_start()
    run = LayerRun("layer1.0.conv1", _t(torch, dev, W), R, [_t(torch, dev, f) for f in fs])
    iters = als_sweep([run], MAX_ITER, 0.0, 4, MSE)
    assert iters[id(run)] == 3 * (MAX_ITER - 1)
    for f, q in zip(run.factors, run.quantized):
        _levels(f.cpu().numpy())
        _levels(q.cpu().numpy())
    print(f"C2 sweep: rec_error gpu {run.loss[-1]:.6f}, reference {min(ref['rec_error']):.6f} .. "
          f"{max(ref['rec_error']):.6f}; quant_rec_error gpu {run.lossq[-1]:.6f}, reference "
          f"{min(ref['quant_rec_error']):.6f} .. {max(ref['quant_rec_error']):.6f}")
    lo, hi = _band(ref["rec_error"])
    assert lo <= run.loss[-1] <= hi, (run.loss[-1], lo, hi)
    lo, hi = _band(ref["quant_rec_error"])
    assert lo <= run.lossq[-1] <= hi, (run.lossq[-1], lo, hi)


def test_c3_batch_at_bench_horizon(torch_dev):
    torch, dev = torch_dev
    import bench
    from admmq import _lib
    from admmq.factorize import LayerRun, als_sweep
    work, _, _ = bench.build_workload("resnet18", 0, 1, "layers", dev)
    runs = [LayerRun(s.name, W, R, [f.clone() for f in init]) for (s, W, R, init) in work]
    start = [float(np.linalg.norm(W.double().cpu().numpy() - np.einsum("ir,jr,kr->ijk", *[f.double().cpu().numpy()
                                                                                       for f in init])) /
                   np.linalg.norm(W.double().cpu().numpy())) for (_, W, _, init) in work]
    _lib.fault_repairs(reset=True)
    iters = als_sweep(runs, MAX_ITER, 0.0, 4, MSE)
    assert _lib.fault_repairs() == 0
    for r, e0 in zip(runs, start):
        assert iters[id(r)] == 3 * (MAX_ITER - 1), r.name
        for f, q, u in zip(r.factors, r.quantized, r.duals):
            _levels(f.cpu().numpy())
            _levels(q.cpu().numpy())
            assert bool(torch.isfinite(u).all()), r.name
        assert np.isfinite(r.loss[-1]) and np.isfinite(r.lossq[-1]), r.name
        assert r.loss[-1] < e0, (r.name, r.loss[-1], e0)
    print("C3 losses:", [round(r.loss[-1], 4) for r in runs])
