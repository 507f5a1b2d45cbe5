#!/usr/bin/env python3
"""F11: the reference's own spread at the benchmarked horizon (survey container only).

Run:  python3 -B tests/golden/gen_f11_horizon.py [--reference /root/reference] [--trials 5] [--threads 1,2,4,8]

bench.py times max_iter_admm = 1000 (999 inner iterations, eps = 0; scripts/factorize.py:
218-221). At that horizon the reference is chaotic at the 1-ulp level: two
solvers within 1 ulp of each other end on different quantization branches, so only the
band the reference itself spans is reproducible. This script runs the reference's
``admm_iteration`` (source/admm.py:51-67) and ``quantize_tensor`` on BASELINE config C2
(resnet18 layer1.0.conv1, synthetic weight, seed-42 random start, U = 0, F / G from the
oracle's Gram / MTTKRP - the inputs tests/test_gpu_horizon.py feeds the device):

  * per mode, 1000 iterations from the start as given and with the result of its
    ``torch.cholesky_solve`` moved by <= 1 ulp per element in every iteration (F8's
    proxy; no reference file is touched): the objective ||F - H G|| / ||F|| (float64)
    and the 4-bit grid step of every run;
  * one ALS sweep (the three modes in sequence, scripts/factorize.py:207-266) the same
    way: the sweep's rec_error and quant_rec_error;
  * all of it at every torch CPU thread count of ``--threads`` (F4's method): the
    reference's matmul / cholesky_solve summation order follows the thread count, a spread
    the 1-ulp proxy alone does not explore. ``runs`` records each run's thread count and
    trial (0 = unperturbed).

Writes data only: tests/golden/f11_horizon.json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
from gen_f8_branches import _TorchProxy  # noqa: E402
from gen_golden import import_reference  # noqa: E402
from oracle import admm_oracle as ao  # noqa: E402

MSE = "tensor_mseminmax_symmetric"
MAX_ITER = 1000


def c2_start():
    from admmq import synthetic
    idx, spec = synthetic.find_layer("resnet18", "layer1.0.conv1")
    W = synthetic.layer_weight(spec, idx)
    R = spec.rank()
    g = torch.Generator().manual_seed(42)
    return W, R, [torch.randn(n, R, generator=g).numpy() for n in W.shape]


def objective(F, G, h):
    F64 = F.astype(np.float64)
    return float(np.linalg.norm(F64 - h.astype(np.float64) @ G.astype(np.float64)) / np.linalg.norm(F64))


def grid_step(h):
    lv = np.unique(h)
    return float(np.min(np.diff(lv))) if len(lv) > 1 else 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--trials", type=int, default=5)
    ap.add_argument("--threads", default="1,2,4,8")
    a = ap.parse_args()
    threads = [int(t) for t in a.threads.split(",")]
    ref_admm, ref_quant = import_reference(a.reference)
    W, R, fs0 = c2_start()
    out = {"config": "C2 resnet18 layer1.0.conv1 R=134, seed-42 random start, U=0, 4-bit mse-minmax, eps=0",
           "max_iter_admm": MAX_ITER, "trials_perturbed": a.trials, "torch": torch.__version__, "threads": threads,
           "runs": [[nt, t] for nt in threads for t in range(a.trials + 1)],
           "modes": {}, "sweep": {"rec_error": [], "quant_rec_error": []}}

    def run(H0, F, G, rng):
        ref_admm.torch = _TorchProxy(rng)
        try:
            H, _ = ref_admm.admm_iteration(torch.from_numpy(H0.copy()), torch.zeros(H0.shape), torch.from_numpy(F),
                                           torch.from_numpy(G), MAX_ITER, 0.0, 4, MSE)
        finally:
            ref_admm.torch = torch
        return H.numpy().astype(np.float32)

    for mode in range(3):
        G, F = ao.gram_mttkrp(W, fs0, mode)
        objs, steps = [], []
        for nt, t in out["runs"]:
            torch.set_num_threads(nt)
            t0 = time.time()
            h = run(fs0[mode], F, G, None if t == 0 else np.random.default_rng(5000 + 10 * mode + t + 1000 * nt))
            objs.append(objective(F, G, h))
            steps.append(grid_step(h))
            print(f"mode {mode} threads {nt} trial {t}: objective {objs[-1]:.6e} step {steps[-1]:.4e} "
                  f"({time.time() - t0:.1f} s)", flush=True)
        out["modes"][str(mode)] = {"objective": objs, "grid_step": steps}
    for nt, t in out["runs"]:
        torch.set_num_threads(nt)
        rng = None if t == 0 else np.random.default_rng(7000 + t + 1000 * nt)
        fs = [f.copy() for f in fs0]
        qf = [None] * 3
        for m in range(3):
            G, F = ao.gram_mttkrp(W, fs, m)
            fs[m] = run(fs[m], F, G, rng)
            qf[m] = ref_quant.quantize_tensor(torch.from_numpy(fs[m]), 4, MSE).numpy()
        Wt = torch.from_numpy(W)
        rec = [torch.from_numpy(np.ascontiguousarray(f)) for f in fs]
        recq = [torch.from_numpy(np.ascontiguousarray(f)) for f in qf]
        out["sweep"]["rec_error"].append(float(ref_admm.squared_relative_diff(Wt, torch.einsum("ir,jr,kr->ijk", *rec))))
        out["sweep"]["quant_rec_error"].append(
            float(ref_admm.squared_relative_diff(Wt, torch.einsum("ir,jr,kr->ijk", *recq))))
        print(f"sweep threads {nt} trial {t}: rec {out['sweep']['rec_error'][-1]:.6f} quant {out['sweep']['quant_rec_error'][-1]:.6f}",
              flush=True)
    with open(os.path.join(HERE, "f11_horizon.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
