"""The C restatement of the quantizer oracle (oracle/quant_oracle_c.c) against the numpy
oracle and the reference's own outputs (F1 KATs, F7 near-tie ADMM iterates). CPU only."""
import json
import os

import numpy as np
import pytest

import golden_cases as gc
from oracle import quant_oracle as qo
from oracle import quant_oracle_c as qc

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
MSE = "tensor_mseminmax_symmetric"


@pytest.mark.parametrize("shape,bits,na", [((9, 134), 4, 200), ((64, 134), 2, 200), ((37, 53), 3, 1000),
                                           ((128, 278), 8, 50), ((1, 5), 4, 7), ((3,), 4, 200), ((2, 3, 5), 4, 200)])
def test_c_table_equals_numpy(shape, bits, na):
    rng = np.random.default_rng(abs(hash((shape, bits, na))) % 2 ** 32)
    x = (rng.standard_normal(shape) * 0.2).astype(np.float32)
    a, grid, mx, K = qc.sse_table(x, bits, na)
    b, grid2, mx2 = qo.mse_sse_table(x, bits, na)
    assert np.array_equal(a, b)
    assert np.array_equal(grid.view(np.uint32), grid2.view(np.uint32))
    assert K == qo.fixed_point_exponent(mx2, int(np.prod(shape[:-1] or (1,))) * ((shape[-1] + 3) // 4))


def test_c_quantizer_on_reference_kats():
    """Every MSE-minmax KAT of F1 (rule 0), bit-exact with the reference digest."""
    with open(os.path.join(GOLDEN, "f1_quant.json")) as f:
        meta = json.load(f)
    n = 0
    for case in meta:
        if case["qscheme"] != MSE or case["error"] is not None:
            continue
        x = gc.f1_input(case)
        if not np.isfinite(x).all() or np.abs(x).max() == 0:
            continue   # degenerate ranges: the C quantizer's NaN output is not the KAT's subject
        na = case.get("num_attempts") or 200
        y, _ = qc.quantize_mse(x, case["bits"], na, rule=0)
        assert gc.canonical_sha(y) == case["sha"], case["id"]
        n += 1
    assert n >= 60


def test_f7_rules_match_reference_argmin():
    """Both argmin rules pick the reference's candidate on its own ADMM iterates (the
    committed F7 inputs), and the statistics over all resnet18 layers/modes agree."""
    with open(os.path.join(GOLDEN, "f7_neartie.json")) as f:
        meta = json.load(f)
    z = np.load(os.path.join(GOLDEN, "f7_neartie.npz"))
    for m in meta:
        x = z[m["key"] + "_X"]
        sse, grid, mx, K = qc.sse_table(x, 4)
        for rule in (0, 1):
            assert qc.argmin(sse, rule, K, x.size) == m["ref_index"], (m["key"], rule)
        y, idx = qc.quantize_mse(x, 4, rule=0)
        assert gc.canonical_sha(y) == m["ref_sha"], m["key"]
        # the reference's own float32 means, recomputed by it, pick the same index
        assert int(np.argmin(z[m["key"] + "_means"])) == m["ref_index"]
    with open(os.path.join(GOLDEN, "f7_stats.json")) as f:
        st = json.load(f)
    assert st["n"] >= 500 and st["rule0_disagree"] == 0


def test_rule1_means_round_like_float32():
    sse = np.array([1 << 40, (1 << 40) + 1, 3 << 38], np.uint64)
    m = qc.rule1_means(sse, 50, 1000)
    assert m.dtype == np.float32 and m[0] == m[1]        # a 1-unit difference vanishes in float32
    assert qc.argmin(sse, 1, 50, 1000) == 2 and qc.argmin(sse, 0, 50, 1000) == 2
