#!/usr/bin/env python3
"""F7: near-tie fixtures - quantizer inputs captured from the reference's own ADMM.

Run (survey/build container only; imports /root/reference read-only):
    python3 -B tests/golden/gen_f7.py [--reference /root/reference] [--stats-steps 1,2,...]

Why: the MSE-minmax search picks the argmin of 200 float32 means
(source/quantization.py:136-141). On ADMM iterates X = H_T - U the best and
second-best candidates can be ~1e-7 apart, so the argmin depends on how the mean
is rounded. The kernels and oracle use an order-independent rule for that mean
(oracle/quant_oracle.py); F7 measures how often that rule picks a different
candidate than the reference on *real* iterates, and pins the HIP path to the
reference on the committed inputs.

How: `source.admm.admm_iteration` is run unchanged on resnet18 synthetic layers
(first ALS sweep from the seed-42 random init, eps = 0), with its module-level
`quantize_tensor` wrapped so that the inputs of chosen inner iterations are
recorded together with the reference's own output. For each captured input the
reference's 200 float32 means are recomputed with the same torch operations as
source/quantization.py:123-141 (checked: the argmin reproduces the reference's
output bit-for-bit).

Outputs (data only):
  f7_neartie.npz   committed inputs X (layer1.0.conv1 / layer2.0.conv1 all modes,
                   layer4.0.conv2 mode 2; steps 5, 50, 500) with the reference's
                   argmin index, float32 means and output digest
  f7_stats.json    agreement of each argmin rule with the reference over every
                   (layer, mode, step) captured (16 layers x 3 modes x stats steps)
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
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from admmq import synthetic  # noqa: E402
import golden_cases as gc  # noqa: E402
from gen_golden import import_reference, mttkrp_ref  # noqa: E402
from oracle import quant_oracle_c as qc  # noqa: E402

MSE = "tensor_mseminmax_symmetric"
FIXTURE = [("layer1.0.conv1", (0, 1, 2)), ("layer2.0.conv1", (0, 1, 2)), ("layer4.0.conv2", (2,))]
FIXTURE_STEPS = (5, 50, 500)


def ref_means(x: torch.Tensor, bits=4, n=200):
    """The reference's per-candidate float32 means and argmin, with the torch
    operations of source/quantization.py:123-141 (the loop body restated so the
    internal `mses` can be read)."""
    q = 2 ** (bits - 1)
    den = 2 * q - 1
    mx = torch.max(torch.abs(x.min()), torch.abs(x.max()))
    grid = torch.linspace(0.2 * mx.item(), 1.2 * mx.item(), n)
    mses = torch.zeros(n)
    dims = list(torch.arange(len(x.shape)))
    for i in range(n):
        scale = 2 * grid[i] / den
        xfp = torch.clamp(torch.round(x / scale), -q, q - 1) * scale
        mses[i] = ((x - xfp) ** 2).mean(dim=dims)
    idx = int(mses.argmin())
    scale = 2 * grid[idx] / den
    return mses.numpy(), idx, (torch.clamp(torch.round(x / scale), -q, q - 1) * scale)


def capture(ref_admm, H0, F, G, steps, max_iter):
    """Run the reference's admm_iteration (eps = 0) recording the quantizer input and
    output of the inner iterations in `steps` (1-based)."""
    rec = {}
    orig = ref_admm.quantize_tensor
    count = [0]

    def hook(tensor, *a, **kw):
        count[0] += 1
        y = orig(tensor, *a, **kw)
        if count[0] in steps:
            rec[count[0]] = (tensor.clone(), y.clone())
        return y

    ref_admm.quantize_tensor = hook
    try:
        ref_admm.admm_iteration(H0.clone(), torch.zeros_like(H0), F, G, max_iter, 0.0, 4, MSE)
    finally:
        ref_admm.quantize_tensor = orig
    return rec


def layer_problems(ref_admm, name):
    li, spec = synthetic.find_layer("resnet18", name)
    W = torch.from_numpy(synthetic.layer_weight(spec, li))
    fs = ref_admm.init_factors(W, rank=spec.rank(2.0), init="random", device="cpu", seed=42)
    return W, fs


def analyse(x: np.ndarray, means, ridx):
    sse, grid, mx, K = qc.sse_table(x, 4)
    srt = np.sort(np.asarray(means, np.float32))
    # how close the reference's best two candidates are, in ulps of its best mean
    out = {"gap_ulps": float(srt[1] - srt[0]) / float(np.spacing(srt[0]))}
    for rule in (0, 1):
        out[f"rule{rule}"] = qc.argmin(sse, rule, K, x.size)
    # the reference's float32 gap between its choice and the rule-0 choice, in ulps
    a = out["rule0"]
    if a != ridx:
        gap = abs(float(means[a]) - float(means[ridx]))
        out["ulps"] = gap / float(np.spacing(np.float32(means[ridx])))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--stats-steps", default="1,2,3,5,8,13,21,34,55,89,144,233")
    ap.add_argument("--no-stats", action="store_true")
    a = ap.parse_args()
    torch.set_num_threads(8)
    ref_admm, _ = import_reference(a.reference)

    # ---- committed fixtures
    arrays = {}
    meta = []
    for name, modes in FIXTURE:
        W, fs = layer_problems(ref_admm, name)
        for m in modes:
            G, F = mttkrp_ref(W, *fs, m)
            rec = capture(ref_admm, fs[m], F, G, set(FIXTURE_STEPS), max(FIXTURE_STEPS) + 1)
            for st in FIXTURE_STEPS:
                x, y = rec[st]
                means, idx, yr = ref_means(x)
                assert gc.canonical_sha(yr.numpy()) == gc.canonical_sha(y.numpy()), "restated mses disagree"
                key = f"{name}_m{m}_s{st}"
                arrays[key + "_X"] = x.numpy()
                arrays[key + "_means"] = means
                meta.append({"key": key, "layer": name, "mode": m, "step": st, "shape": list(x.shape),
                             "ref_index": idx, "ref_sha": gc.canonical_sha(y.numpy()), **analyse(x.numpy(), means, idx)})
                print(meta[-1], flush=True)
    np.savez_compressed(os.path.join(HERE, "f7_neartie.npz"), **arrays)
    with open(os.path.join(HERE, "f7_neartie.json"), "w") as f:
        json.dump(meta, f, indent=1)

    if a.no_stats:
        return
    # ---- agreement statistics over every layer and mode of resnet18
    steps = sorted(int(s) for s in a.stats_steps.split(","))
    stats = {"steps": steps, "cases": [], "torch": torch.__version__, "threads": torch.get_num_threads()}
    t0 = time.time()
    for spec in synthetic.resnet18_layers():
        W, fs = layer_problems(ref_admm, spec.name)
        for m in range(3):
            G, F = mttkrp_ref(W, *fs, m)
            rec = capture(ref_admm, fs[m], F, G, set(steps), max(steps) + 1)
            for st in steps:
                x, y = rec[st]
                means, idx, yr = ref_means(x)
                assert gc.canonical_sha(yr.numpy()) == gc.canonical_sha(y.numpy())
                r = {"layer": spec.name, "mode": m, "step": st, "ref_index": idx, **analyse(x.numpy(), means, idx)}
                stats["cases"].append(r)
            print(spec.name, m, f"{time.time() - t0:.0f}s", flush=True)
    n = len(stats["cases"])
    for rule in (0, 1):
        d = sum(1 for c in stats["cases"] if c[f"rule{rule}"] != c["ref_index"])
        stats[f"rule{rule}_disagree"] = d
        print(f"rule {rule}: {d} of {n} argmins differ from the reference")
    stats["n"] = n
    gaps = sorted(c["gap_ulps"] for c in stats["cases"])
    stats["gap_ulps_min"], stats["gap_ulps_median"] = gaps[0], gaps[len(gaps) // 2]
    stats["cases_within_16_ulps"] = sum(1 for g in gaps if g <= 16)
    print("best-vs-second gap (ulps): min", gaps[0], "median", gaps[len(gaps) // 2])
    with open(os.path.join(HERE, "f7_stats.json"), "w") as f:
        json.dump(stats, f, indent=1)


if __name__ == "__main__":
    main()
