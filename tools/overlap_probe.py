#!/usr/bin/env python3
"""Probe: does the 9-row spatial mode (mode 2: thin solve + one-CU-per-job search) of one
layer set overlap with the big mode (mode 0) of another when the two ADMM runs are on
separate HIP streams? Times mode 0 alone, mode 2 alone and both concurrently (C3 shapes,
eps = 0). usage: python tools/overlap_probe.py [iters]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))

import torch  # noqa: E402

from admmq import synthetic  # noqa: E402
from admmq.admm import admm_iteration_batched  # noqa: E402
from admmq.als import gram_mttkrp_batched  # noqa: E402

MSE = "tensor_mseminmax_symmetric"


def problems(mode, dev):
    specs = synthetic.MODELS["resnet18"]()
    ws, fs = [], []
    for i, s in enumerate(specs):
        W = torch.from_numpy(synthetic.layer_weight(s, i, 0)).to(dev)
        g = torch.Generator().manual_seed(42)
        fs.append([torch.randn(n, s.rank(), generator=g).to(dev) for n in s.shape])
        ws.append(W)
    GF = gram_mttkrp_batched(list(zip(ws, fs)), mode)
    return [(f[mode].clone(), torch.zeros_like(f[mode]), F, G) for f, (G, F) in zip(fs, GF)]


def run(probs, iters):
    ps = [(h.clone(), u.clone(), F, G) for (h, u, F, G) in probs]
    return admm_iteration_batched(ps, iters, 0.0, 4, MSE, check_spd=False)


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda:0")
    p0, p2 = problems(0, dev), problems(2, dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    run(p0, 3), run(p2, 3)   # warm-up

    def both():
        with torch.cuda.stream(s1):
            run(p0, iters)
        with torch.cuda.stream(s2):
            run(p2, iters)

    for rep in range(2):
        a = timed(lambda: run(p0, iters))
        b = timed(lambda: run(p2, iters))
        c = timed(both)
        print(f"rep {rep}: mode0 {a:.1f} ms  mode2 {b:.1f} ms  serial {a + b:.1f} ms  two streams {c:.1f} ms "
              f"(saved {100 * (a + b - c) / (a + b):.1f} %)", flush=True)


if __name__ == "__main__":
    main()
