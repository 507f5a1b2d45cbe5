"""GPU checks of the rank projection's panel kernels (csrc/panel_kernels.hip, C-ABI
admmq_panel_xtq / _xy / _outer; the products of scripts/factorize_lowrank.py:80-82's
truncation as admmq.lowrank.KrylovProjector forms them):

  * X^T Q and X Y against float64 torch GEMMs of the widened X: 1e-13 relative per column
    (both are exact products summed in float64; only the summation order differs);
  * ragged shapes (rows / columns not multiples of 4, 16 or 64; k above one 32-column
    block, k below 16), a strided X, the scalar-load form;
  * the same bits on every call (fixed summation order, no data atomics), also when the
    workspace is shared by the two kernels;
  * A B^T rounded once to float32: within one float32 rounding of float64 torch;
  * argument errors.
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


@pytest.fixture(scope="module")
def env():
    import torch
    return torch, torch.device("cuda:0")


def _colrel(a, b):
    """max over columns of ||a - b|| / ||b||"""
    num = (a - b).norm(dim=0)
    den = b.norm(dim=0).clamp_min(1e-300)
    return float((num / den).max())


SHAPES = [(4096, 4096, 32), (1000, 777, 40), (129, 4100, 8), (333, 257, 200), (64, 64, 16), (5, 3, 1)]


@pytest.mark.parametrize("m,n,k", SHAPES)
def test_xtq_matches_fp64(env, m, n, k):
    torch, dev = env
    from admmq import panel
    g = torch.Generator(device="cpu").manual_seed(m * 7 + n + k)
    X = torch.randn(m, n, generator=g).to(dev)
    Q = torch.randn(m, k, generator=g, dtype=torch.float64).to(dev)
    Y = panel.xtq(X, Q)
    ref = X.double().T @ Q
    assert Y.shape == (n, k)
    assert _colrel(Y, ref) < 1e-13
    assert torch.equal(Y, panel.xtq(X, Q))   # same bits every call


@pytest.mark.parametrize("m,n,k", SHAPES)
def test_xy_matches_fp64(env, m, n, k):
    torch, dev = env
    from admmq import panel
    g = torch.Generator(device="cpu").manual_seed(m + 3 * n + k)
    X = torch.randn(m, n, generator=g).to(dev)
    Y = torch.randn(n, k, generator=g, dtype=torch.float64).to(dev)
    Z = panel.xy(X, Y)
    ref = X.double() @ Y
    assert Z.shape == (m, k)
    assert _colrel(Z, ref) < 1e-13
    assert torch.equal(Z, panel.xy(X, Y))


def test_strided_x_and_xxtq_chain(env):
    """A row-strided view of X (ldx > n, the scalar-load form when n % 4 != 0) and the
    X (X^T Q) chain of one Krylov block on one shared workspace."""
    torch, dev = env
    from admmq import panel
    g = torch.Generator(device="cpu").manual_seed(5)
    big = torch.randn(700, 1030, generator=g).to(dev)
    for X in (big[:, :1024], big[:, 3:1022]):
        Q = torch.randn(700, 32, generator=g, dtype=torch.float64).to(dev)
        Z = panel.xy(X, panel.xtq(X, Q))
        Xd = X.double()
        assert _colrel(Z, Xd @ (Xd.T @ Q)) < 1e-12


def test_tile_count_grows_on_one_workspace(env):
    """Calls whose tile counts grow (k = 32, then the Rayleigh-Ritz panel of 8 blocks, then
    back) on one workspace: every tile's arrival counter keeps its address (the counters sit
    at the workspace's end), so a later, larger call never reads a partial as a counter."""
    torch, dev = env
    from admmq import panel
    g = torch.Generator(device="cpu").manual_seed(9)
    X = torch.randn(2048, 2048, generator=g).to(dev)
    Xd = X.double()
    lib = __import__("admmq")._lib.load()
    ws = torch.zeros(lib.admmq_panel_workspace_size(2048, 2048, 256), dtype=torch.uint8, device=dev)
    key = panel._key(X.device)   # (device, current stream): the workspace these calls use
    panel._WS[key] = ws          # one workspace for every call below
    for k in (32, 256, 64, 256, 32, 160):
        Q = torch.randn(2048, k, generator=g, dtype=torch.float64).to(dev)
        assert _colrel(panel.xtq(X, Q), Xd.T @ Q) < 1e-13
        assert _colrel(panel.xy(X, Q), Xd @ Q) < 1e-13
    assert panel._WS[key] is ws


@pytest.mark.parametrize("m,n,r", [(4096, 4096, 8), (1000, 777, 32), (17, 5, 3)])
def test_outer_rounds_once(env, m, n, r):
    torch, dev = env
    from admmq import panel
    g = torch.Generator(device="cpu").manual_seed(m + n + r)
    A = torch.randn(m, r, generator=g, dtype=torch.float64).to(dev)
    B = torch.randn(n, r, generator=g, dtype=torch.float64).to(dev)
    O = panel.outer(A, B)
    ref = A @ B.T
    assert O.dtype == torch.float32 and O.shape == (m, n)
    # one float32 rounding of a float64 sum (torch's order may differ in the last fp64 bits)
    err = (O.double() - ref).abs()
    bound = 2.0 ** -24 * ref.abs() + 1e-13 * (A.abs() @ B.abs().T)
    assert bool((err <= bound).all())


@pytest.mark.parametrize("m,p,q", [(4096, 32, 32), (4096, 256, 32), (4096, 256, 256), (1000, 40, 17), (5, 3, 2),
                                   (70000, 8, 8)])
def test_gram_matches_fp64(env, m, p, q):
    """A^T B of tall float64 panels (the Krylov block's Gram and cross products)."""
    torch, dev = env
    from admmq import panel
    g = torch.Generator(device="cpu").manual_seed(m + p + q)
    A = torch.randn(m, p, generator=g, dtype=torch.float64).to(dev)
    B = torch.randn(m, q, generator=g, dtype=torch.float64).to(dev)
    C = panel.gram(A, B)
    assert C.shape == (p, q)
    assert _colrel(C, A.T @ B) < 1e-13
    assert torch.equal(C, panel.gram(A, B))
    Ct = panel.gram(A.T.contiguous().T, B)   # a column-major A (copied to rows)
    assert torch.equal(C, Ct)


def test_panel_argument_errors(env):
    torch, dev = env
    from admmq import panel
    X = torch.zeros(8, 8, device=dev)
    with pytest.raises(ValueError):
        panel.xtq(X, torch.zeros(7, 4, dtype=torch.float64, device=dev))
    with pytest.raises(ValueError):
        panel.xy(X.double(), torch.zeros(8, 4, dtype=torch.float64, device=dev))
    with pytest.raises(Exception):
        panel.outer(torch.zeros(4, 40, dtype=torch.float64, device=dev), torch.zeros(4, 40, dtype=torch.float64, device=dev))


def test_two_streams_own_workspaces(env):
    """Panel calls queued on two streams at once (advisor r04: one shared workspace let
    their partial slots and monotonic arrival counters race) each get their own (device,
    stream) workspace: every product equals the single-stream result bit for bit, and a
    later call on the default stream is still correct (counters stayed in step)."""
    torch, dev = env
    from admmq import panel
    g = torch.Generator().manual_seed(11)
    X = torch.randn(2048, 1536, generator=g).to(dev)
    Qs = [torch.randn(2048, 32, generator=g, dtype=torch.float64).to(dev) for _ in range(2)]
    Ys = [torch.randn(1536, 32, generator=g, dtype=torch.float64).to(dev) for _ in range(2)]
    ref_t = [panel.xtq(X, Q) for Q in Qs]
    ref_y = [panel.xy(X, Y) for Y in Ys]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    outs = [[], []]
    for rep in range(8):
        for j, s in enumerate(streams):
            with torch.cuda.stream(s):
                outs[j].append((panel.xtq(X, Qs[j]), panel.xy(X, Ys[j])))
    torch.cuda.synchronize()
    for j in range(2):
        for t, y in outs[j]:
            assert torch.equal(t, ref_t[j]) and torch.equal(y, ref_y[j])
    keys = {k for k in panel._WS if k[0] == dev}
    assert len(keys) >= 3   # the default stream and the two side streams
    assert torch.equal(panel.xtq(X, Qs[0]), ref_t[0])
