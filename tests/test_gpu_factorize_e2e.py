"""O1 end to end: ``python -m admmq.factorize`` (the reference CLI, scripts/factorize.py:38-102)
writes the files scripts/calibrate.py:169-184 loads, and they build the factorized layer.

The run goes through admmq.factorize.main in this process (one GPU process for the whole
test session). Checked: the output tree
``{bits}bit_{qscheme}/factors_{method}_seed{seed}/{layer}_{method}_{init}_rank_{R}_mode_{n}.pt``
(+ ``_losshist.pt`` / ``_lossquanthist.pt``) with the reference's names
(scripts/factorize.py:164-166, 315-318, 345-347), float32 CPU tensors of shape (I_n, R),
loss histories as Python float lists, the saved factors equal to the driver's result, and
the calibrate-side load + admmq.export.build_cp_layer / build_cp2conv_layer reproducing the
CP reconstruction as a convolution (source/models.py:24-74).
"""
import json
import os

import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


def _calibrate_load(root, bits, qscheme, method, seed, layer, init, rank, three_way):
    """scripts/calibrate.py:169-184 (file names and dtype assertion), weights_only loads."""
    name = os.path.join(root, f"{bits}bit_{qscheme}", f"factors_{method}_seed{seed}", f"{layer}_{method}_{init}_rank_{rank}_")
    A = torch.load(name + "mode_0.pt", weights_only=True)
    assert A.dtype == torch.float
    B = torch.load(name + "mode_1.pt", weights_only=True)
    C = torch.load(name + "mode_2.pt", weights_only=True) if three_way else None
    return A, B, C


@pytest.mark.parametrize("model,layer,three_way", [("resnet18", "layer1.0.conv1", True),
                                                   ("resnet50", "layer1.0.conv1", False)])
def test_factorize_cli_outputs(tmp_path, model, layer, three_way):
    from admmq import factorize, synthetic
    from admmq.export import build_cp_layer, build_cp2conv_layer
    argv = ["--model-name", model, "--method", "admm", "--layer", layer, "--reduction-rate", "2.0", "--bits", "4",
            "--seed", "42", "--qscheme", "tensor_mseminmax_symmetric", "--max_iter_als", "3", "--max_iter_admm", "20",
            "--outdir-root", str(tmp_path), "--metrics-jsonl", str(tmp_path / "metrics.jsonl")]
    factors, factors_q = factorize.main(argv)
    idx, spec = synthetic.find_layer(model, layer)
    W = torch.from_numpy(synthetic.layer_weight(spec, idx))
    if W.dim() == 4:
        W = W.reshape(W.shape[0], W.shape[1]) if W.shape[2:] == (1, 1) else W.reshape(W.shape[0], W.shape[1], -1)
    R = int(W.numel() / sum(W.shape) / 2.0)
    out = tmp_path / "4bit_tensor_mseminmax_symmetric" / "factors_admm_seed42"
    prefix = f"{layer}_admm_random_rank_{R}"
    names = sorted(p.name for p in out.iterdir())
    expect = sorted([f"{prefix}_mode_{m}.pt" for m in range(W.dim())] +
                    [f"{prefix}_losshist.pt", f"{prefix}_lossquanthist.pt"])
    assert names == expect
    A, B, C = _calibrate_load(str(tmp_path), 4, "tensor_mseminmax_symmetric", "admm", 42, layer, "random", R, three_way)
    for m, (f, ref) in enumerate(zip([A, B] + ([C] if three_way else []), factors)):
        assert f.device.type == "cpu" and f.dtype == torch.float32 and tuple(f.shape) == (W.shape[m], R)
        assert torch.equal(f, ref.cpu())
    lh = torch.load(out / f"{prefix}_losshist.pt", weights_only=True)
    lq = torch.load(out / f"{prefix}_lossquanthist.pt", weights_only=True)
    assert isinstance(lh, list) and all(isinstance(v, float) for v in lh) and 1 <= len(lh) <= 3
    assert len(lq) == len(lh) and all(0.0 < v < 1.5 for v in lh + lq)
    # SURVEY §5 metrics: one JSONL record per sweep, the errors equal the saved histories
    recs = [json.loads(x) for x in (tmp_path / "metrics.jsonl").read_text().splitlines()]
    assert [r["sweep"] for r in recs] == list(range(len(lh)))
    assert [r["rec_error"] for r in recs] == lh and [r["quant_rec_error"] for r in recs] == lq
    assert all(r["layer"] == layer and 0 < r["factor_iterations"] <= 20 * W.dim() and r["sweep_s"] > 0 for r in recs)
    # the calibrate side: the CP layer built from the files equals the CP reconstruction
    cout, cin = W.shape[0], W.shape[1]
    if three_way:
        layer_mod = build_cp_layer(R, [A, B, C], None, cin, cout, (3, 3), (1, 1), (1, 1), 1)
        rec = torch.einsum("ir,jr,kr->ijk", A, B, C).reshape(cout, cin, 3, 3)
    else:
        layer_mod = build_cp2conv_layer(R, [A, B], None, cin, cout, (0, 0), (1, 1))
        rec = (A @ B.T).reshape(cout, cin, 1, 1)
    x = torch.randn(2, cin, 8, 8, generator=torch.Generator().manual_seed(0))
    y = layer_mod(x)
    y_ref = torch.nn.functional.conv2d(x, rec, None, 1, 1 if three_way else 0)
    assert torch.allclose(y, y_ref, rtol=1e-4, atol=1e-4)
