"""CPU tests of host logic: layer tables, ranks, the ALS driver's Gram/MTTKRP
formulation, and the oracle's ALS restatement vs the reference fixtures."""
import json
import os

import numpy as np
import pytest
import torch

from admmq import synthetic
from admmq.factorize import reconstruct
from oracle import torch_port
from oracle import admm_oracle as ao

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_resnet18_ranks_match_reference_table():
    # source/rank_map.py:317-340 (rate 2, resnet18)
    ref = {"layer1.0.conv1": 134, "layer1.0.conv2": 134, "layer1.1.conv1": 134, "layer1.1.conv2": 134,
           "layer2.0.conv1": 183, "layer2.0.conv2": 278, "layer2.1.conv1": 278, "layer2.1.conv2": 278,
           "layer3.0.conv1": 375, "layer3.0.conv2": 566, "layer3.1.conv1": 566, "layer3.1.conv2": 566,
           "layer4.0.conv1": 759, "layer4.0.conv2": 1141, "layer4.1.conv1": 1141, "layer4.1.conv2": 1141}
    layers = synthetic.resnet18_layers()
    assert [l.name for l in layers] == list(ref)
    assert {l.name: l.rank(2.0) for l in layers} == ref


def test_resnet50_ranks_match_reference_table():
    # source/rank_map.py:266-315 (rate 2, resnet50), spot checks incl. 1x1 (2-way) layers
    ref = {"layer1.0.conv1": 16, "layer1.0.conv2": 134, "layer1.0.conv3": 25, "layer1.1.conv1": 25,
           "layer2.0.conv1": 42, "layer2.0.conv3": 51, "layer3.0.conv1": 85, "layer3.0.conv3": 102,
           "layer4.0.conv1": 170, "layer4.0.conv2": 1141, "layer4.2.conv3": 204}
    got = {l.name: l.rank(2.0) for l in synthetic.resnet50_layers()}
    assert len(got) == 48
    for k, v in ref.items():
        assert got[k] == v, k


def test_torch_port_gram_mttkrp_matches_oracle():
    """The CPU baseline's per-mode setup (reference expressions) vs the numpy oracle."""
    rng = np.random.default_rng(0)
    W = torch.from_numpy(rng.standard_normal((6, 5, 4)).astype(np.float32))
    fs = [torch.from_numpy(rng.standard_normal((n, 3)).astype(np.float32)) for n in W.shape]
    specs = ["abc,cr,br->ar", "abc,cr,ar->br", "abc,br,ar->cr"]
    args = [(fs[2], fs[1]), (fs[2], fs[0]), (fs[1], fs[0])]
    for m in range(3):
        G, F = torch_port.gram_mttkrp(W, fs, m)
        torch.testing.assert_close(F, torch.einsum(specs[m], W, *args[m]), rtol=1e-5, atol=1e-5)
        Gn, Fn = ao.gram_mttkrp(W.numpy(), [f.numpy() for f in fs], m)
        np.testing.assert_allclose(G.numpy(), Gn, rtol=1e-6)
    W2 = torch.from_numpy(rng.standard_normal((6, 5)).astype(np.float32))
    G, F = torch_port.gram_mttkrp(W2, fs[:2], 1)
    torch.testing.assert_close(F, W2.T @ fs[0])
    assert reconstruct(fs[:2]).shape == (6, 5)


def test_oracle_admm_vs_reference_fixtures():
    """Oracle few-step ADMM tracks the reference's own outputs (F2): the solve to 1e-5 after
    one step (implied H_T = H - U1), and the dual to 1e-4 over 1-5 steps on modes where no
    MSE candidate flip occurred."""
    z = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    for mode in range(3):
        G, F, H0 = z[f"l1_m{mode}_G"], z[f"l1_m{mode}_F"], z["l1_" + "ABC"[mode]]
        _, _, info = ao.admm_iteration(H0, np.zeros_like(H0), F, G, 2, 1e-8, 4, "tensor_mseminmax_symmetric",
                                       return_info=True)
        ref_HT = z[f"l1_m{mode}_tensor_mseminmax_symmetric_it2_H"] - z[f"l1_m{mode}_tensor_mseminmax_symmetric_it2_U"]
        assert np.linalg.norm(info["HT"] - ref_HT) / np.linalg.norm(ref_HT) < 1e-5
    for qs in ("tensor_minmax", "tensor_symmetric", "tensor_affine"):
        G, F, H0 = z["l1_m0_G"], z["l1_m0_F"], z["l1_A"]
        for it in (2, 3, 6):
            H, U = ao.admm_iteration(H0, np.zeros_like(H0), F, G, it, 1e-8, 4, qs)
            ref = z[f"l1_m0_{qs}_it{it}_U"]
            assert np.linalg.norm(U - ref) / np.linalg.norm(ref) < 1e-4


def test_oracle_als_short_vs_reference():
    z = np.load(os.path.join(GOLDEN, "f3_als.npz"))
    f2 = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    _, _, loss, lossq = ao.als(f2["l1_W"], [f2["l1_A"], f2["l1_B"], f2["l1_C"]], 2, 3)
    np.testing.assert_allclose(loss, z["l1_loss"], rtol=1e-4)
    np.testing.assert_allclose(lossq, z["l1_lossq"], rtol=1e-4)
    _, _, loss, lossq = ao.als(f2["w2_W"], [f2["w2_A"], f2["w2_B"]], 3, 4)
    np.testing.assert_allclose(loss, z["w2_loss"], rtol=1e-4)


@pytest.mark.slow
def test_oracle_long_horizon_band():
    with open(os.path.join(GOLDEN, "f4_band.json")) as f:
        band = json.load(f)
    f2 = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    _, _, loss, lossq = ao.als(f2["l1_W"], [f2["l1_A"], f2["l1_B"], f2["l1_C"]], 20, 20)
    rec = [v["loss"][-1] for v in band.values()]
    assert min(rec) * 0.98 <= loss[-1] <= max(rec) * 1.02


def test_torch_port_vs_reference_fixtures():
    """The bench's CPU baseline port follows the reference to float32 rounding (F2)."""
    from oracle import torch_port
    z = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    for mode in (0, 2):
        G, F, H0 = (torch.from_numpy(z[k]) for k in (f"l1_m{mode}_G", f"l1_m{mode}_F", "l1_" + "ABC"[mode]))
        H, U = torch_port.admm_iteration(H0, torch.zeros_like(H0), F, G, 2, 1e-8, 4)
        ref = z[f"l1_m{mode}_tensor_mseminmax_symmetric_it2_U"]
        assert np.linalg.norm(U.numpy() - ref) / np.linalg.norm(ref) < 1e-5


def test_sweep_metrics_jsonl(tmp_path):
    """SURVEY §5 metrics: one JSON object per (sweep, layer) with the reference's wandb keys
    (scripts/factorize.py:249-253) plus the sweep's wall time and factor-iterations."""
    from admmq.factorize import JsonlWriter, LayerRun, parse_args, sweep_records
    runs = [LayerRun("a", torch.zeros(4, 3, 9), 2, [torch.zeros(4, 2), torch.zeros(3, 2), torch.zeros(9, 2)]),
            LayerRun("b", torch.zeros(5, 6), 3, [torch.zeros(5, 3), torch.zeros(6, 3)])]
    runs[0].loss, runs[0].lossq = [0.5, 0.4], [0.6, 0.45]
    runs[1].loss, runs[1].lossq = [0.3], [0.35]
    runs[1].active = False
    iters = {id(runs[0]): 3 * 999, id(runs[1]): 2 * 17}
    recs = sweep_records(runs, 1, iters, 2.0)
    w = JsonlWriter(str(tmp_path / "sub" / "m.jsonl"))
    for r in recs:
        w(r)
    w.close()
    back = [json.loads(x) for x in (tmp_path / "sub" / "m.jsonl").read_text().splitlines()]
    assert back == recs
    assert [r["layer"] for r in back] == ["a", "b"] and all(r["sweep"] == 1 for r in back)
    assert back[0]["rec_error"] == 0.4 and back[0]["quant_rec_error"] == 0.45 and back[0]["factor_iterations"] == 2997
    assert back[1]["active"] is False and back[1]["factor_iterations"] == 34
    assert back[0]["factor_iterations_per_s"] == pytest.approx((2997 + 34) / 2.0)
    a = parse_args(["--model-name", "resnet18", "--method", "admm", "--layer", "layer1.0.conv1", "--rank", "8",
                    "--bits", "4", "--seed", "0", "--qscheme", "tensor_minmax_symmetric", "--with-wandb"])
    assert a.with_wandb and a.metrics_jsonl is None
