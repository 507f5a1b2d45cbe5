"""GPU parity against the REFERENCE's own outputs (not only the oracle).

* F2 (tests/golden/f2_admm.npz): source/admm.py:51-67 run by the reference itself on
  resnet18 layer1.0.conv1 (all 3 modes; mode 0 with all four schemes) and on a 2-way
  problem, for max_iter 2, 3 and 6 (1, 2 and 5 inner steps). The HIP path starts from
  the same (H, U=0, F, G) and is compared step horizon by step horizon:
    it2 (P2): the same quantization candidate (scale within 1e-6), and integer levels
              equal except elements whose pre-round value is within 1e-4 of a
              half-integer (counted; explained flips only);
    it3 (P3): the same candidate; at most 0.1 % of the levels differ, and with no
              step-1 flip every difference is a near-half rounding of step 2 (the
              reference itself is chaotic at the 1-ulp level); with no level
              difference, H within 1e-4 rel-Frob;
    it6:      the result lies ON one of the reference's own branches (F8,
              tests/golden/gen_f8_branches.py: the reference re-run with its
              cholesky_solve moved by <= 1 ulp per element reaches, e.g. for
              tensor_symmetric mode 0, two trajectories with scales 10.8 % apart):
              scale within 1e-5 of a branch's and at most 0.5 % of the levels
              differing from that branch's H. F2 stores one sample of them.
  tensor_minmax has no uniform grid (source/quantization.py:48-66): H within 1e-5.
* F7 (tests/golden/f7_neartie.*): quantizer inputs captured from the reference's own
  ADMM at steps 5, 50, 500 (tests/golden/gen_f7.py). The HIP quantizer output must
  equal the reference's output digest, or - a near tie of the reference's float32
  means - be counted and bounded to 2 ulps of the reference's own mean.
"""
import json
import os

import numpy as np
import pytest

import golden_cases as gc
from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
MSE = "tensor_mseminmax_symmetric"


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    return torch, torch.device("cuda:0")


def _t(torch, dev, a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _f2_cases():
    out = []
    for mode in range(3):
        for qs in (gc.F2_SCHEMES if mode == 0 else [MSE]):
            out.append((mode, qs))
    return out


def _run(torch, dev, H0, F, G, max_iter, qs, solve="split"):
    from admmq import admm_iteration_batched
    from admmq._lib import solve_mode
    U = torch.zeros(H0.shape, device=dev)
    with solve_mode(solve):
        (H,), dbg = admm_iteration_batched([(_t(torch, dev, H0), U, _t(torch, dev, F), _t(torch, dev, G))], max_iter,
                                           1e-8, 4, qs, debug_outputs=True)
    return H.cpu().numpy(), U.cpu().numpy(), dbg[0][1].cpu().numpy()


@pytest.mark.parametrize("solve", ["split", "fp32"])
@pytest.mark.parametrize("mode,qscheme", _f2_cases())
def test_f2_reference_horizons(torch_dev, mode, qscheme, solve):
    torch, dev = torch_dev
    z = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    G, F, H0 = z[f"l1_m{mode}_G"], z[f"l1_m{mode}_F"], z["l1_" + "ABC"[mode]]
    report = {}
    flipped_at_1 = None
    for mi in (2, 3, 6):
        H, U, X = _run(torch, dev, H0, F, G, mi, qscheme, solve)
        rH, rU = z[f"l1_m{mode}_{qscheme}_it{mi}_H"], z[f"l1_m{mode}_{qscheme}_it{mi}_U"]
        if qscheme == "tensor_minmax":
            assert _rel(H, rH) < 1e-5, (mi, _rel(H, rH))
            continue
        k, s = gc.grid_levels(H)
        kr, sr = gc.grid_levels(rH)
        assert k is not None and kr is not None, "quantized output is not on a uniform grid"
        srel = abs(float(s) - float(sr)) / float(sr)
        n_bad, n_unexplained = gc.level_mismatch(H, rH, X)
        report[mi] = dict(scale_rel=srel, mismatches=n_bad, unexplained=n_unexplained, H_rel=_rel(H, rH))
        if mi == 2:
            assert srel < 1e-6, report
            assert n_unexplained == 0, report
            flipped_at_1 = n_bad > 0
        elif mi == 3:
            assert srel < 1e-6 and n_bad <= 1e-3 * H.size, report
            if not flipped_at_1:   # every step-2 difference is a near-half rounding of step 2
                assert n_unexplained == 0, report
            if n_bad == 0:
                assert _rel(H, rH) < 1e-4, report
        else:
            bH, frac = _reference_branch(mode, qscheme, s)
            assert bH is not None, (report, "it6 scale on no reference branch", float(s))
            n_bad, _ = gc.level_mismatch(H, bH, X)
            report[mi].update(branch_frequency=frac, branch_mismatches=n_bad)
            assert n_bad <= 5e-3 * H.size, report
    print(mode, qscheme, solve, report)


def _reference_branch(mode, qscheme, scale):
    """(H, frequency) of the F8 reference branch whose scale is within 1e-5 of `scale`."""
    with open(os.path.join(GOLDEN, "f8_branches.json")) as f:
        meta = {c["key"]: c for c in json.load(f)["cases"]}
    c = meta[f"m{mode}_{qscheme}"]
    z = np.load(os.path.join(GOLDEN, "f8_branches.npz"))
    for j, b in enumerate(c["branches"]):
        if abs(float(scale) - b["scale"]) / b["scale"] < 1e-5:
            return z[f"{c['key']}_b{j}_H"], b["count"] / c["trials"]
    return None, 0.0


def test_f2_two_way_reference(torch_dev):
    torch, dev = torch_dev
    z = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    G, F, H0 = z["w2_G"], z["w2_F"], z["w2_A"]
    for mi in (2, 3, 6):
        H, U, X = _run(torch, dev, H0, F, G, mi, MSE)
        rH = z[f"w2_it{mi}_H"]
        n_bad, n_unexplained = gc.level_mismatch(H, rH, X)
        assert n_unexplained == 0 and n_bad == 0, (mi, n_bad)
        assert _rel(H, rH) < 1e-4


def test_f7_neartie_reference(torch_dev):
    """The HIP quantizer on the reference's own ADMM iterates (F7): every one of the 21
    outputs equals the reference's (DESIGN §2.3 claims 21/21; a difference would have to be
    a float32 tie of the reference's means, reported with its ulp distance)."""
    torch, dev = torch_dev
    from admmq import quantize_batched
    with open(os.path.join(GOLDEN, "f7_neartie.json")) as f:
        meta = json.load(f)
    z = np.load(os.path.join(GOLDEN, "f7_neartie.npz"))
    xs = [_t(torch, dev, z[m["key"] + "_X"]) for m in meta]
    ys = quantize_batched(xs, 4, MSE)
    differ = []
    for m, y in zip(meta, ys):
        y = y.cpu().numpy()
        if gc.canonical_sha(y) == m["ref_sha"]:
            continue
        means = z[m["key"] + "_means"]
        k, s = gc.grid_levels(y)
        # which candidate the GPU chose: the grid entry whose scale it used
        x = z[m["key"] + "_X"]
        from oracle import quant_oracle as qo
        mx = np.float32(max(abs(x.min()), abs(x.max())))
        grid = qo.candidate_grid(mx, 200)
        scales = ((np.float32(2) * grid).astype(np.float32) / np.float32(15)).astype(np.float32)
        c = int(np.nonzero(scales == s)[0][0])
        ulps = abs(float(means[c]) - float(means[m["ref_index"]])) / float(np.spacing(means[m["ref_index"]]))
        differ.append((m["key"], c, m["ref_index"], ulps))
    print(f"F7: {len(meta) - len(differ)} of {len(meta)} equal to the reference; near ties: {differ}")
    assert len(meta) == 21
    assert differ == [], differ


@pytest.mark.parametrize("name", ["l1", "w2"])
def test_svd_init_reference(torch_dev, name):
    """init_factors('svd') (source/admm.py:29-35) vs the reference's own factors (F2):
    singular vectors up to sign, the random completion columns bit-exact."""
    torch, dev = torch_dev
    from admmq import init_factors
    z = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    T = z["l1_W"] if name == "l1" else z["w2_W"]
    R = 134 if name == "l1" else 13
    fs = init_factors(_t(torch, dev, T), rank=R, init="svd", device=dev, seed=42)
    for m, f in enumerate(fs):
        ref = z[f"{name}_svd_m{m}"]
        got = f.cpu().numpy()
        assert got.shape == ref.shape
        ns = min(T.shape[m], R)
        for j in range(ns):
            sgn = np.sign(np.dot(got[:, j], ref[:, j])) or 1.0
            assert _rel(sgn * got[:, j], ref[:, j]) < 2e-3, (m, j)
        assert np.array_equal(got[:, ns:], ref[:, ns:]), m
