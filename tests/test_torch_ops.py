"""torch.ops.admmq.* (csrc/torch_ops.cpp over the C-ABI of include/admmq.h).

CPU: the op library loads, declares the six schemas, propagates shapes on the Meta
device (fake tensors / tracing) and rejects CPU tensors in the dispatcher (there is no
CPU kernel). GPU: every op returns exactly what the C-ABI called through ctypes
returns, and the Python drop-ins route through the ops.
"""
import numpy as np
import pytest
import torch

from conftest import gpu_available

SCHEMAS = {
    "admm_iteration_batched": "admmq::admm_iteration_batched(Tensor[] H, Tensor(a!)[] U, Tensor[] F, Tensor[] G, "
                              "int max_iter, float eps, int bits, int qscheme, int num_attempts=200, "
                              "bool check_spd=True, bool debug=False, int solve=-1, bool check_fault=True) -> (Tensor[] H_out, Tensor info, Tensor[] HT, "
                              "Tensor[] X)",
    "quantize_batched": "admmq::quantize_batched(Tensor[] x, int bits, int qscheme, int num_attempts=200, "
                        "float? tmin=None, float? tmax=None) -> Tensor[]",
    "quantize_channel": "admmq::quantize_channel(Tensor x, int bits, int qscheme, int dim) -> Tensor",
    "cp_gram_mttkrp": "admmq::cp_gram_mttkrp(Tensor[] W, Tensor[] factors, int mode) -> (Tensor[] G, Tensor[] F)",
    "cp_rel_error": "admmq::cp_rel_error(Tensor[] W, Tensor[] factors) -> Tensor",
    "fault_repairs": "admmq::fault_repairs(bool reset=False) -> int",
}


@pytest.fixture(scope="module")
def ops():
    from admmq import _lib
    return _lib.ops()


def test_schemas(ops):
    for name, schema in SCHEMAS.items():
        assert str(getattr(ops, name).default._schema) == schema


def test_meta_shapes(ops):
    m = torch.device("meta")
    H = [torch.empty(64, 134, device=m), torch.empty(9, 1141, device=m)]
    G = [torch.empty(134, 134, device=m), torch.empty(1141, 1141, device=m)]
    outs, info, hts, xs = ops.admm_iteration_batched(H, [torch.empty_like(h) for h in H], [torch.empty_like(h) for h in H],
                                                     G, 10, 1e-8, 4, 0, 200, False, True)
    assert [o.shape for o in outs] == [h.shape for h in H] and info.shape == (2, 5) and info.dtype == torch.int32
    assert [t.shape for t in hts] == [h.shape for h in H] and len(xs) == 2
    ys = ops.quantize_batched([torch.empty(3, 5, device=m)], 4, 0)
    assert ys[0].shape == (3, 5)
    W = [torch.empty(64, 32, 9, device=m), torch.empty(40, 30, device=m)]
    fs = [torch.empty(64, 7, device=m), torch.empty(32, 7, device=m), torch.empty(9, 7, device=m),
          torch.empty(40, 5, device=m), torch.empty(30, 5, device=m)]
    Gs, Fs = ops.cp_gram_mttkrp(W, fs, 1)
    assert [g.shape for g in Gs] == [(7, 7), (5, 5)] and [f.shape for f in Fs] == [(32, 7), (30, 5)]
    assert ops.cp_rel_error(W, fs).shape == (2,)


def test_fault_repair_counter(ops):
    """The op's process-wide count of calls repaired after an internal fault (no GPU
    needed): a non-negative int, reset to 0 by reset=True."""
    from admmq import _lib
    assert ops.fault_repairs(False) >= 0
    _lib.fault_repairs(reset=True)
    assert ops.fault_repairs(False) == 0 and _lib.fault_repairs() == 0
    _lib.note_repair()
    assert _lib.fault_repairs(reset=True) == 1 and _lib.fault_repairs() == 0


def test_cpu_tensors_rejected(ops):
    with pytest.raises(NotImplementedError):
        ops.quantize_batched([torch.zeros(4, 4)], 4, 0)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_ops_equal_cabi(ops):
    """Bit-identical results through torch.ops.admmq and through the C-ABI (ctypes)."""
    import os
    from admmq import _lib, admm as A, quantization as Q, als
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    probs = []
    for I, R in ((64, 134), (9, 566), (512, 300)):
        B = torch.randn(R, 2 * R, generator=g) / (2 * R) ** 0.5
        probs.append((torch.randn(I, R, generator=g).to(dev) * 0.1, torch.zeros(I, R, device=dev),
                      torch.randn(I, R, generator=g).to(dev), (B @ B.T + 0.5 * torch.eye(R)).to(dev)))
    U1 = [p[1].clone() for p in probs]
    U2 = [p[1].clone() for p in probs]
    H1, info1 = A.admm_iteration_batched([(p[0], u, p[2], p[3]) for p, u in zip(probs, U1)], 8, 0.0, 4,
                                         "tensor_mseminmax_symmetric", return_info=True)
    H2, info2 = A._admm_iteration_batched_cabi([(p[0], u, p[2], p[3]) for p, u in zip(probs, U2)], 8, 0.0, 4, 0, 200,
                                               True, False, True)
    for a, b in zip(H1 + U1, H2 + U2):
        assert torch.equal(a, b)
    assert torch.equal(info1, info2)
    xs = [torch.randn(33, 77, generator=g).to(dev), torch.randn(9, 1141, generator=g).to(dev)]
    for qs in ("tensor_mseminmax_symmetric", "tensor_minmax", "tensor_symmetric", "tensor_affine"):
        y1 = Q.quantize_batched(xs, 4, qs)
        os.environ["ADMMQ_LIB"] = _lib.LIB_PATH   # same library, ctypes route
        try:
            y2 = Q.quantize_batched(xs, 4, qs)
        finally:
            del os.environ["ADMMQ_LIB"]
        for a, b in zip(y1, y2):
            assert torch.equal(a, b), qs
    W = torch.randn(64, 32, 9, generator=g).to(dev)
    fs = [torch.randn(n, 20, generator=g).to(dev) for n in W.shape]
    (G1, F1), = als.gram_mttkrp_batched([(W, fs)], 2)
    e1 = als.rel_error_batched([(W, fs)])
    os.environ["ADMMQ_LIB"] = _lib.LIB_PATH
    try:
        (G2, F2), = als.gram_mttkrp_batched([(W, fs)], 2)
        e2 = als.rel_error_batched([(W, fs)])
    finally:
        del os.environ["ADMMQ_LIB"]
    assert torch.equal(G1, G2) and torch.equal(F1, F2) and e1 == e2


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_ops_errors_and_compile(ops):
    """Reference error behaviour through the ops (non-SPD -> LinAlgError), U mutated in
    place, and the op traced by torch.compile (graph break-free with the Meta kernels)."""
    from admmq import admm_iteration
    dev = torch.device("cuda:0")
    H = torch.randn(16, 8, device=dev)
    U = torch.zeros(16, 8, device=dev)
    G = -torch.eye(8, device=dev)
    with pytest.raises(torch.linalg.LinAlgError):
        admm_iteration(H, U, torch.randn(16, 8, device=dev), G * 3.0 + torch.ones(8, 8, device=dev), 5, 1e-8, 4,
                       "tensor_mseminmax_symmetric")
    G = torch.eye(8, device=dev) * 2.0
    Hn, Uo = admm_iteration(H, U, torch.randn(16, 8, device=dev), G, 5, 1e-8, 4, "tensor_mseminmax_symmetric")
    assert Uo is U and not torch.equal(U, torch.zeros_like(U))

    def f(x):
        return ops.quantize_batched([x * 2.0], 4, 0)[0] + 1.0

    x = torch.randn(64, 134, device=dev)
    y = torch.compile(f, fullgraph=True)(x)
    assert torch.equal(y, f(x))
