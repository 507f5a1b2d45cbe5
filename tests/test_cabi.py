"""CPU tests of the C-ABI library: it loads without a GPU, exports every symbol that
include/admmq.h declares, and its host-side planner answers (no compute calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "admmq.h")


@pytest.fixture(scope="module")
def lib():
    from admmq import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libadmmq.so is not built: run __graft_entry__.build()")
    return _lib.load()


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(admmq_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("admmq_admm_prepare", "admmq_admm_run", "admmq_quantize_batched", "admmq_mse_sse_table"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert missing == []


def test_struct_layouts_match_header():
    from admmq import _lib
    assert ctypes.sizeof(_lib.AdmmProblem) == 7 * 8 + 2 * 4
    assert ctypes.sizeof(_lib.QTensor) == 2 * 8 + 2 * 8 + 2 * 4 + 2 * 4


def test_version_and_error_text(lib):
    assert lib.admmq_version() >= 100
    assert isinstance(lib.admmq_last_error(), bytes)


def test_workspace_planner(lib):
    from admmq import _lib
    p = _lib.AdmmProblem(0, 0, 0, 0, 0, 0, 0, 64, 134)
    arr = _lib.problems_array([p])
    one = lib.admmq_admm_workspace_size(arr, 1, 200)
    # Fp,H,U,P,X,HT (64 x 144 f32) + M (192^2 f32) + A64,L64 (192^2 f64) + D64 + tables
    assert one >= 6 * 64 * 144 * 4 + 192 * 192 * 4 + 2 * 192 * 192 * 8
    big = _lib.AdmmProblem(0, 0, 0, 0, 0, 0, 0, 512, 1141)
    two = lib.admmq_admm_workspace_size(_lib.problems_array([p, big]), 2, 200)
    assert two > one
    assert lib.admmq_admm_workspace_size(arr, 0, 200) == 0          # no problems -> error (0)
    bad = _lib.AdmmProblem(0, 0, 0, 0, 0, 0, 0, 0, 5)
    assert lib.admmq_admm_workspace_size(_lib.problems_array([bad]), 1, 200) == 0
    assert b"positive" in lib.admmq_last_error()


def test_workspace_size_matches_carve(lib):
    """Sizing (null base) and the real carve (non-null base) must agree for every
    mix of thin (I <= 16: split-K VALU solve), 32-row and tall factors."""
    from admmq import _lib
    shapes = [(9, 134), (9, 1141), (3, 40), (16, 700), (17, 300), (32, 64), (64, 134), (512, 1141)]
    sets = [[s] for s in shapes] + [shapes, shapes[::-1], [(9, 134), (512, 1141)]]
    for st in sets:
        arr = _lib.problems_array([_lib.AdmmProblem(0, 0, 0, 0, 0, 0, 0, i, r) for i, r in st])
        n = lib.admmq_admm_workspace_size(arr, len(st), 200)
        assert n > 0
        assert lib.admmq_debug_admm_plan_bytes(arr, len(st), 200, ctypes.c_void_p(1 << 20)) == n, st


def test_quantize_planner(lib):
    from admmq import _lib
    t = _lib.QTensor(0, 0, 9, 134, 0.0, 0.0, 0, 0)
    n = lib.admmq_quantize_workspace_size(_lib.qtensor_array([t]), 1, 200)
    assert n >= 9 * 136 * 4 + 200 * 8
    assert lib.admmq_quantize_workspace_size(_lib.qtensor_array([t]), 1, 0) == 0


def test_product_path_refuses_cpu_tensors():
    import torch
    from admmq import quantize_tensor, admm_iteration
    x = torch.randn(4, 5)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        quantize_tensor(x, 4, "tensor_mseminmax_symmetric")
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        admm_iteration(x, torch.zeros_like(x), x, torch.eye(5), 3, 1e-8, 4, "tensor_mseminmax_symmetric")
    with pytest.raises(TypeError):
        quantize_tensor(x, 4, "channel_affine")
    with pytest.raises(NotImplementedError):
        quantize_tensor(x, 4, "tensor_log")


def test_cp_layer_struct_and_planner(lib):
    """admmq_cp_layer layout and the ALS-contraction workspace planner (no compute)."""
    from admmq import _lib
    assert ctypes.sizeof(_lib.CpLayer) == 8 + 3 * 8 + 8 + 8 + 3 * 4 + 4 + 4 + 4   # + tail pad to 8

    def layer(dims, R):
        L = _lib.CpLayer()
        L.W = 0x1000
        for d in range(3):
            L.factors[d] = 0x2000 * (d + 1) if d < len(dims) else None
            L.dims[d] = dims[d] if d < len(dims) else 0
        L.ndim, L.R = len(dims), R
        return L

    arr = (_lib.CpLayer * 2)(layer((512, 512, 9), 1141), layer((2048, 512), 204))
    for mode in range(2):
        n = lib.admmq_cp_workspace_size(arr, 2, mode)
        assert n > 0
    # mode 2 of the 3x3 conv: K = 512*512 split into chunks -> partial planes (9 x 1141 each)
    one = (_lib.CpLayer * 1)(layer((512, 512, 9), 1141))
    assert lib.admmq_cp_workspace_size(one, 1, 2) > 2 * 9 * 1141 * 4
    bad = (_lib.CpLayer * 1)(layer((4, 5, 6), 3))
    bad[0].ndim = 4
    assert lib.admmq_cp_workspace_size(bad, 1, 0) == 0


def test_als_contractions_refuse_cpu_tensors():
    import torch
    from admmq.als import gram_mttkrp, rel_error
    W = torch.randn(4, 5, 6)
    fs = [torch.randn(n, 3) for n in W.shape]
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        gram_mttkrp(W, fs, 0)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        rel_error(W, fs)


def test_ksplit_pieces_by_shape(lib):
    """K-split pieces of the fp32 solve tiles (api.hip ksplit_pieces) depend on (I, R)
    only: the resnet18 layer4 conv modes (512, 1141) take 3 pieces of 12 K-steps, the
    (512, 759) ones 2, the mid layers 2-4, factors whose tiles fill the chip (C5, resnet50
    (2048, 204)), 32-row and thin factors, and short K ranges none."""
    expect = {(512, 1141): 3, (512, 759): 2, (256, 759): 4, (256, 566): 3, (256, 375): 2, (128, 375): 2,
              (128, 278): 1, (64, 134): 1, (4096, 1024): 1, (11008, 1492): 1, (2048, 204): 1, (32, 1141): 1,
              (9, 1141): 1, (1024, 1141): 1}
    for (I, R), n in expect.items():
        assert lib.admmq_debug_ksplit_pieces(I, R) == n, (I, R, lib.admmq_debug_ksplit_pieces(I, R))
    assert lib.admmq_debug_ksplit_pieces(0, 5) == 0


def test_panel_entry_points_check_arguments(lib):
    """The rank projection's panel products (admmq_panel_*, admmq_gram64): workspace sizes
    and argument / workspace checks answered on the host before any launch."""
    P = ctypes.c_void_p
    one = P(16)   # a non-null dummy address: every call below is refused before a launch
    assert lib.admmq_panel_workspace_size(4096, 4096, 32) >= 64 * 4 * 64 * 32 * 8
    assert lib.admmq_panel_workspace_size(0, 4096, 32) == 0
    big = lib.admmq_panel_workspace_size(4096, 4096, 256)
    assert big > lib.admmq_panel_workspace_size(4096, 4096, 32)
    ERR_ARG, ERR_WS = -1, -3
    assert lib.admmq_panel_xtq(None, 8, 8, 8, one, 4, one, one, 1 << 20, None) == ERR_ARG
    assert lib.admmq_panel_xtq(one, 8, 8, 7, one, 4, one, one, 1 << 20, None) == ERR_ARG      # ldx < n
    assert lib.admmq_panel_xy(one, 8, 8, 8, one, 4, one, one, 16, None) == ERR_WS            # workspace too small
    assert lib.admmq_panel_xy(one, 8, 8, 8, one, 4, one, None, 1 << 20, None) == ERR_WS
    assert lib.admmq_panel_outer(one, one, 8, 8, 33, one, 8, None) == ERR_ARG                # rank above 32
    assert lib.admmq_panel_outer(one, one, 8, 8, 4, one, 7, None) == ERR_ARG                 # ldo < n
    assert lib.admmq_gram64_workspace_size(4096, 32, 32) >= 16 * 16 * 64 * 8
    assert lib.admmq_gram64(one, 3, one, 4, 8, 4, 4, one, one, 1 << 20, None) == ERR_ARG     # lda < p
    assert lib.admmq_gram64(one, 4, one, 4, 8, 4, 4, one, one, 8, None) == ERR_WS
    assert b"workspace" in lib.admmq_last_error()


def test_epc_solves_refuse_bad_arguments(lib):
    """The one-workgroup R x R solves and the column normalisation of the EPC initialiser
    check their arguments on the host before any launch (include/admmq.h: 1 <= n <= 136,
    non-NULL buffers); the Python wrappers refuse CPU or non-float64 tensors and n > 136,
    and parafac_epc refuses a CPU tensor (no CPU path)."""
    import torch
    from admmq import panel
    from admmq.parafac_epc import parafac_epc
    p = ctypes.c_void_p(0x1000)
    assert lib.admmq_spd_solve64(p, p, 4, 137, p, None, None) != 0          # n above the LDS limit
    assert lib.admmq_spd_solve64(None, p, 4, 8, p, None, None) != 0         # no G
    assert lib.admmq_epc_step64(p, p, 4, 137, 1.0, 0.5, p, p, p, None, None) != 0
    assert lib.admmq_epc_step64(p, p, 4, 8, 1.0, 0.5, p, p, None, None, None) != 0   # no workspace
    assert lib.admmq_cp_colnorm64(None, 4, None, 0, 8, p, None, None) != 0
    assert lib.admmq_cp_colnorm64(p, 4, p, 3, 8, p, None, None) != 0        # B without its output
    G = torch.eye(4, dtype=torch.float64)
    F = torch.randn(3, 4, dtype=torch.float64)
    with pytest.raises(ValueError):
        panel.colnorm64(F)                                                 # a CPU tensor
    with pytest.raises(ValueError):
        panel.spd_solve64(G.float(), F)                                    # float32
    with pytest.raises(RuntimeError, match="ROCm GPU"):                  # a CPU tensor (n > 136: the blocked step)
        panel.epc_step64(torch.eye(137, dtype=torch.float64), torch.randn(2, 137, dtype=torch.float64), 1.0, 0.5,
                         torch.zeros((), dtype=torch.float64))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        panel.spd_solve64(torch.eye(200, dtype=torch.float64), torch.randn(2, 200, dtype=torch.float64))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        parafac_epc(torch.randn(4, 5, 6, dtype=torch.float64), 3)


def test_blocked_solves_check_arguments(lib):
    """The blocked R x R solves (csrc/solve64.hip: any n) size their workspace from (m, n) alone
    and refuse bad arguments or a short workspace on the host, before any launch."""
    p = ctypes.c_void_p(0x1000)
    ERR_ARG, ERR_WS = -1, -3
    assert lib.admmq_solve64_workspace_size(0, 5) == 0
    assert lib.admmq_solve64_workspace_size(4, 0) == 0
    big = lib.admmq_solve64_workspace_size(512, 1141)
    assert big >= 2 * 1152 * 1152 * 8 + 2 * 512 * 1141 * 8                # A, L^-1 and the two m x n products
    assert big == lib.admmq_solve64_workspace_size(512, 1141)               # a function of (m, n) only
    assert lib.admmq_solve64_workspace_size(9, 1141) < big
    assert lib.admmq_spd_solve64_ws(None, p, 4, 200, 0.0, p, None, p, 1 << 30, None) == ERR_ARG
    assert lib.admmq_spd_solve64_ws(p, p, 4, 200, -1.0, p, None, p, 1 << 30, None) == ERR_ARG   # negative shift
    assert lib.admmq_spd_solve64_ws(p, p, 4, 200, 0.0, p, None, p, 8, None) == ERR_WS
    assert lib.admmq_epc_begin64(p, p, 4, 200, 1.0, 0.5, None, p, p, 1 << 30, None) == ERR_ARG   # no mu
    assert lib.admmq_epc_begin64(p, p, 4, 200, 1.0, 0.5, p, p, p, 8, None) == ERR_WS
    assert lib.admmq_epc_rounds64(p, p, 4, 200, p, -1, None, p, 1 << 30, None) == ERR_ARG
    assert lib.admmq_epc_rounds64(p, p, 4, 200, p, 1, None, p, 8, None) == ERR_WS
    assert lib.admmq_epc_end64(0, 200, p, None, p, 1 << 30, None) == ERR_ARG
    assert lib.admmq_epc_end64(4, 200, p, None, p, 8, None) == ERR_WS
