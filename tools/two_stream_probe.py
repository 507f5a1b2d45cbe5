#!/usr/bin/env python3
"""Probe: one batched admm_iteration over all resnet18 factors of a mode on one stream,
against the same factors split into k LPT-balanced groups, each group's batched call
on its own HIP stream (issued back to back by the host, running concurrently)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "admm-quantization_amd")]
import torch  # noqa: E402
from admmq import synthetic  # noqa: E402
from admmq.admm import admm_iteration_batched  # noqa: E402
from admmq.als import gram_mttkrp_batched  # noqa: E402

MSE = "tensor_mseminmax_symmetric"
dev = torch.device("cuda:0")
specs = synthetic.MODELS["resnet18"]()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 201
fused = (sys.argv[2] != "nofused") if len(sys.argv) > 2 else True
from admmq import _lib  # noqa: E402
_lib.load().admmq_debug_set_fused_finalize(1 if fused else 0)
print(f"fused finalize: {fused}; fp32 solve: {_lib.load().admmq_get_solve_mode() == 0}", flush=True)
for mode in range(3):
    layers = []
    for i, s in enumerate(specs):
        W = torch.from_numpy(synthetic.layer_weight(s, i)).to(dev)
        g = torch.Generator().manual_seed(42)
        fs = [torch.randn(n, s.rank(), generator=g).to(dev) for n in s.shape]
        layers.append((W, fs))
    GF = gram_mttkrp_batched(layers, mode)
    probs = [(fs[mode], torch.zeros_like(fs[mode]), F, G) for (W, fs), (G, F) in zip(layers, GF)]
    cost = [2.0 * p[0].shape[0] * p[0].shape[1] ** 2 + 1600.0 * p[0].numel() for p in probs]

    def run(groups):
        streams = [torch.cuda.Stream() for _ in groups]
        infos = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for st, grp in zip(streams, groups):
            with torch.cuda.stream(st):
                _, info = admm_iteration_batched([(probs[i][0], torch.zeros_like(probs[i][1]), probs[i][2], probs[i][3])
                                                  for i in grp], iters, 0.0, 4, MSE, check_spd=False, return_info=True,
                                                 check_fault=False)
                infos.append(info)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        faults = sum(int(i[:, 3].sum()) for i in infos)
        if faults:
            print(f"  ({faults} problems hit the fused-finalize timeout)", flush=True)
        return dt

    for k in (1, 2, 3):
        loads = [0.0] * k
        groups = [[] for _ in range(k)]
        for i in sorted(range(len(probs)), key=lambda j: -cost[j]):
            b = min(range(k), key=lambda j: loads[j])
            groups[b].append(i)
            loads[b] += cost[i]
        run(groups)
        ts = sorted(run(groups) for _ in range(3))
        print(f"mode {mode} groups {k}: {1e3 * ts[1]:.2f} ms for {iters - 1} iterations "
              f"({1e6 * ts[1] / (iters - 1):.1f} us/iter)", flush=True)
