#!/usr/bin/env python3
"""F8: the reference's own branches at the 5-step ADMM horizon (survey container only).

Run:  python3 -B tests/golden/gen_f8_branches.py [--reference /root/reference] [--trials 32]

SURVEY §0 measured the reference's ADMM as chaotic at the 1-ulp level. F2 stores ONE
trajectory per (mode, scheme): the one the reference's own float32 rounding happened
to pick. This script re-runs the reference's ``admm_iteration`` (source/admm.py:51-67)
from the F2 start (H0, U = 0, F, G), ``max_iter`` = 6, with the result of its
``torch.cholesky_solve`` (:56) moved by at most 1 ulp per element in every iteration
(each element independently nudged up, down or kept, seeded; the module's ``torch``
name is pointed at a proxy for the run, no reference file is touched) - i.e. the
reference as any solver within 1 ulp of its own would run it - and clusters the
final H by its quantization scale (relative 1e-5). Every distinct branch
the reference reaches is stored with its frequency, so a GPU test can require "the
HIP result is ON a reference branch" at that horizon instead of "equal to the one
sample F2 happened to store". The unperturbed run must reproduce F2's it6 H exactly
(checked). Writes data only: tests/golden/f8_branches.npz + .json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import golden_cases as gc  # noqa: E402
from gen_golden import import_reference  # noqa: E402

EPS = 1e-8


def cases():
    out = [(0, qs) for qs in gc.F2_SCHEMES if qs != "tensor_minmax"]
    out += [(1, "tensor_mseminmax_symmetric"), (2, "tensor_mseminmax_symmetric")]
    return out


def perturb(F, rng):
    """Each element moved by at most 1 ulp: up, down or kept (equal odds)."""
    d = rng.integers(-1, 2, size=F.shape)
    up = np.nextafter(F, np.float32(np.inf))
    dn = np.nextafter(F, np.float32(-np.inf))
    return np.where(d > 0, up, np.where(d < 0, dn, F)).astype(np.float32)


class _TorchProxy:
    """``torch`` with cholesky_solve's result perturbed by <= 1 ulp per element."""

    def __init__(self, rng):
        self.rng = rng

    def __getattr__(self, name):
        return getattr(torch, name)

    def cholesky_solve(self, *a, **k):
        x = torch.cholesky_solve(*a, **k)
        return torch.from_numpy(perturb(x.numpy(), self.rng)) if self.rng is not None else x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--trials", type=int, default=32)
    a = ap.parse_args()
    torch.set_num_threads(8)   # F2 was generated at 8 threads
    ref_admm, _ = import_reference(a.reference)
    z = np.load(os.path.join(HERE, "f2_admm.npz"))
    arrays, meta = {}, []
    for mode, qs in cases():
        G, F, H0 = z[f"l1_m{mode}_G"], z[f"l1_m{mode}_F"], z["l1_" + "ABC"[mode]]
        rng = np.random.default_rng(1000 + 10 * mode + gc.F2_SCHEMES.index(qs))
        branches = []   # [scale, H, count]
        for t in range(a.trials + 1):
            ref_admm.torch = _TorchProxy(None if t == 0 else rng)
            try:
                H, _ = ref_admm.admm_iteration(torch.from_numpy(H0.copy()), torch.zeros(H0.shape), torch.from_numpy(F),
                                               torch.from_numpy(G), max_iter=6, eps=EPS, bits=4, qscheme=qs)
            finally:
                ref_admm.torch = torch
            H = H.numpy()
            if t == 0:
                assert np.array_equal(H, z[f"l1_m{mode}_{qs}_it6_H"]), "reference does not reproduce F2 it6"
            _, s = gc.grid_levels(H)
            for b in branches:
                if abs(float(s) - b[0]) / b[0] < 1e-5:
                    b[2] += 1
                    break
            else:
                branches.append([float(s), H, 1])
        branches.sort(key=lambda b: -b[2])
        key = f"m{mode}_{qs}"
        for j, b in enumerate(branches[:4]):
            arrays[f"{key}_b{j}_H"] = b[1]
        meta.append({"key": key, "mode": mode, "qscheme": qs, "trials": a.trials + 1,
                     "branches": [{"scale": b[0], "count": b[2]} for b in branches[:4]],
                     "n_branches": len(branches)})
        print(key, [(round(b[0], 7), b[2]) for b in branches])
    np.savez_compressed(os.path.join(HERE, "f8_branches.npz"), **arrays)
    with open(os.path.join(HERE, "f8_branches.json"), "w") as f:
        json.dump({"torch": torch.__version__, "threads": 8, "perturbation": "cholesky_solve result +-1 ulp per element, every iteration",
                   "cases": meta}, f, indent=1)


if __name__ == "__main__":
    main()
