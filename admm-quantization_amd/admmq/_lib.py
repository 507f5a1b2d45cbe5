"""ctypes binding of libadmmq.so (the C-ABI of include/admmq.h).

The product path has no CPU fallback: if the HIP library is missing or a tensor
is not on a ROCm device, calls raise. Device memory, the current HIP stream and
the workspace allocation come from PyTorch-ROCm (plumbing only).
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# ADMMQ_LIB: another build of the same library (diagnostics only, e.g. the TRACE=1
# build libadmmq_trace.so read by tools/*_timeline.py)
LIB_PATH = os.environ.get("ADMMQ_LIB") or os.path.join(_HERE, "libadmmq.so")

SCHEMES = {
    "tensor_mseminmax_symmetric": 0,
    "tensor_minmax": 1,
    "tensor_symmetric": 2,
    "tensor_affine": 3,
}
CHANNEL_SCHEMES = {"channel_symmetric": 4, "channel_affine": 5}


class AdmmProblem(ctypes.Structure):
    _fields_ = [("F", ctypes.c_void_p), ("G", ctypes.c_void_p), ("H0", ctypes.c_void_p),
                ("H_out", ctypes.c_void_p), ("U", ctypes.c_void_p), ("HT_out", ctypes.c_void_p),
                ("X_out", ctypes.c_void_p), ("I", ctypes.c_int32), ("R", ctypes.c_int32)]


class AdmmOptions(ctypes.Structure):
    """admmq_admm_options (include/admmq.h): per-call solve form and fused finalize."""
    _fields_ = [("solve_mode", ctypes.c_int32), ("fused_finalize", ctypes.c_int32), ("reserved", ctypes.c_int32 * 6)]


SOLVE_MODES = {"fp32": 0, "split": 1}


def default_options() -> AdmmOptions:
    o = AdmmOptions()
    check(load().admmq_admm_default_options(ctypes.byref(o)), "default_options")
    return o


class QTensor(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("y", ctypes.c_void_p), ("rows", ctypes.c_int64),
                ("cols", ctypes.c_int64), ("tmin", ctypes.c_float), ("tmax", ctypes.c_float),
                ("has_minmax", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class CpLayer(ctypes.Structure):
    _fields_ = [("W", ctypes.c_void_p), ("factors", ctypes.c_void_p * 3), ("G", ctypes.c_void_p),
                ("F", ctypes.c_void_p), ("dims", ctypes.c_int32 * 3), ("ndim", ctypes.c_int32),
                ("R", ctypes.c_int32)]


_lib = None
# ADMMQ_LIB (diagnostics, e.g. a `make TRACE=1` build): its directory also holds the ops library
OPS_PATH = os.path.join(os.path.dirname(LIB_PATH), "libadmmq_torch.so")
_ops = None


def use_ops() -> bool:
    """The drop-ins route through torch.ops.admmq (libadmmq_torch.so over the C-ABI),
    except when ADMMQ_LIB selects another build of the C-ABI library for diagnostics
    (the op library links the default one): then they call the C-ABI through ctypes."""
    return not os.environ.get("ADMMQ_LIB")


def ops():
    """``torch.ops.admmq`` (csrc/torch_ops.cpp): loads libadmmq_torch.so once and raises
    loudly when it was not built - there is no CPU fallback."""
    global _ops
    if _ops is None:
        if not os.path.exists(OPS_PATH):
            raise ImportError(f"admmq: {OPS_PATH} is missing - build it with `make -C admm-quantization_amd/csrc`")
        load()
        torch.ops.load_library(OPS_PATH)
        _ops = torch.ops.admmq
    return _ops


def load() -> ctypes.CDLL:
    """Load libadmmq.so once (raises loudly when it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"admmq: {LIB_PATH} is missing - build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "or `make -C admm-quantization_amd/csrc`; there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    P, S, I32, I64, F32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
    sig = {
        "admmq_admm_workspace_size": (S, [P, I32, I32]),
        "admmq_admm_prepare": (I32, [P, I32, I32, P, S, P]),
        "admmq_admm_run": (I32, [P, I32, I32, F32, I32, I32, I32, P, S, P, P]),
        "admmq_admm_iteration_batched": (I32, [P, I32, I32, F32, I32, I32, I32, P, S, P, P]),
        "admmq_admm_default_options": (I32, [P]),
        "admmq_admm_workspace_size_ex": (S, [P, I32, I32, P]),
        "admmq_admm_prepare_ex": (I32, [P, I32, I32, P, P, S, P]),
        "admmq_admm_run_ex": (I32, [P, I32, I32, F32, I32, I32, I32, P, P, S, P, P]),
        "admmq_debug_set_fin_wait_polls": (I32, [ctypes.c_uint32]),
        "admmq_debug_set_f32_persistent": (I32, [I32, I32]),
        "admmq_debug_set_gemm_ks": (I32, [I32]),
        "admmq_debug_set_gemm_stage": (I32, [I32]),
        "admmq_debug_set_ksplit": (I32, [I32]),
        "admmq_debug_set_ksplit_form": (I32, [I32]),
        "admmq_debug_set_ksplit_balance": (I32, [I32, I32]),
        "admmq_debug_ksplit_balance_count": (ctypes.c_int64, [ctypes.c_void_p, I32]),
        "admmq_debug_ksplit_pieces": (I32, [I32, I32]),
        "admmq_debug_set_even_units": (I32, [I32]),
        "admmq_spd_solve64": (I32, [P, P, I64, I64, P, P, P]),
        "admmq_debug_epc_evals": (I32, [P, I32]),
        "admmq_debug_spd_trace": (I32, [P]),
        "admmq_debug_epc_trace": (I32, [P]),
        "admmq_epc_step64": (I32, [P, P, I64, I64, ctypes.c_double, ctypes.c_double, P, P, P, P, P]),
        "admmq_debug_hist_cu": (I32, [P, I32]),
        "admmq_debug_set_fin_capacity": (I32, [I32]),
        "admmq_debug_set_fin_nv3": (I32, [I32]),
        "admmq_debug_set_thin_loop": (I32, [I32]),
        "admmq_quantize_workspace_size": (S, [P, I32, I32]),
        "admmq_quantize_batched": (I32, [P, I32, I32, I32, I32, P, S, P]),
        "admmq_mse_sse_table": (I32, [P, I64, I64, I32, I32, P, P, S, P]),
        "admmq_quantize_channel_workspace_size": (S, [P, I32, I32]),
        "admmq_quantize_channel": (I32, [P, P, P, I32, I32, I32, I32, P, S, P]),
        "admmq_set_exhaustive_search": (I32, [I32]),
        "admmq_debug_set_sel_widen": (I32, [I32]),
        "admmq_debug_set_wide_min_tiles": (I32, [ctypes.c_int64]),
        "admmq_set_solve_mode": (I32, [I32]),
        "admmq_get_solve_mode": (I32, []),
        "admmq_debug_set_legacy_stage1": (I32, [I32]),
        "admmq_debug_admm_plan_bytes": (S, [P, I32, I32, P]),
        "admmq_debug_check_thresholds": (I32, [ctypes.c_uint32, I32]),
        "admmq_debug_set_fused_finalize": (I32, [I32]),
        "admmq_debug_set_search_units_per_block": (I32, [I32]),
        "admmq_debug_check_cells": (I32, [I32, I32, ctypes.c_uint32, I32, P]),
        "admmq_profile_begin": (I32, [I32, I32]),
        "admmq_profile_end": (I32, [P, P]),
        "admmq_cp_workspace_size": (S, [P, I32, I32]),
        "admmq_cp_gram_mttkrp": (I32, [P, I32, I32, P, S, P]),
        "admmq_cp_rel_error": (I32, [P, I32, P, P, S, P]),
        "admmq_cp64_workspace_size": (S, [P, I32, I32]),
        "admmq_cp64_gram_mttkrp": (I32, [P, I32, I32, P, S, P]),
        "admmq_lowrank_workspace_size": (S, [I64]),
        "admmq_lowrank_reset": (I32, [P, S, P]),
        "admmq_lowrank_pre": (I32, [P, P, P, P, P, P, I64, F32, P, S, P]),
        "admmq_lowrank_post": (I32, [P, P, P, P, I64, F32, P, S, P]),
        "admmq_panel_workspace_size": (S, [I64, I64, I64]),
        "admmq_panel_xtq": (I32, [P, I64, I64, I64, P, I64, P, P, S, P]),
        "admmq_panel_xy": (I32, [P, I64, I64, I64, P, I64, P, P, S, P]),
        "admmq_panel_outer": (I32, [P, P, I64, I64, I64, P, I64, P]),
        "admmq_gram64_workspace_size": (S, [I64, I64, I64]),
        "admmq_gram64": (I32, [P, I64, P, I64, I64, I64, I64, P, P, S, P]),
        "admmq_epc_mu": (I32, [P, P, I64, ctypes.c_double, ctypes.c_double, P, P]),
        "admmq_cp_colnorm64": (I32, [P, I64, P, I64, I64, P, P, P]),
        "admmq_solve64_workspace_size": (S, [I64, I64]),
        "admmq_debug_s64_evals": (I32, [P, I32]),
        "admmq_spd_solve64_ws": (I32, [P, P, I64, I64, ctypes.c_double, P, P, P, S, P]),
        "admmq_epc_begin64": (I32, [P, P, I64, I64, ctypes.c_double, ctypes.c_double, P, P, P, S, P]),
        "admmq_epc_rounds64": (I32, [P, P, I64, I64, P, I32, P, P, S, P]),
        "admmq_epc_end64": (I32, [I64, I64, P, P, P, S, P]),
        "admmq_version": (I32, []),
        "admmq_last_error": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("ADMMQ_LIB") and not hasattr(lib, name):
            continue   # a diagnostic build (ADMMQ_LIB) from before the entry point existed
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().admmq_last_error().decode(errors="replace")
        raise RuntimeError(f"admmq: {what} failed (status {rc}): {msg}")


def require_device(*tensors: torch.Tensor):
    for t in tensors:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"admmq: expected a torch.Tensor, got {type(t).__name__}")
        if t.device.type != "cuda":
            raise RuntimeError("admmq: tensors must live on a ROCm GPU (device 'cuda'); the MI355X path has "
                               "no CPU implementation")
        if t.dtype != torch.float32:
            raise TypeError(f"admmq: float32 tensors required, got {t.dtype}")


def stream_handle(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def workspace(nbytes: int, device: torch.device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def problems_array(items: Sequence[AdmmProblem]):
    arr = (AdmmProblem * len(items))(*items)
    return arr


def qtensor_array(items: Sequence[QTensor]):
    return (QTensor * len(items))(*items)


# Calls repaired on the Python side (the ctypes route, and admmq.factorize's per-sweep
# repair): see fault_repairs
_PY_REPAIRS = [0]


def note_repair(n: int = 1):
    _PY_REPAIRS[0] += n


def fault_repairs(reset: bool = False) -> int:
    """Re-runs made because a fused path reported an internal fault (its bounded wait
    expired: the launch's blocks were not all resident, e.g. another stream's kernels on
    the device), since the last reset, process-wide: the torch op's own repairs
    (``torch.ops.admmq.fault_repairs``) plus the Python routes'. 0 on an undisturbed device."""
    n = _PY_REPAIRS[0]
    if reset:
        _PY_REPAIRS[0] = 0
    if use_ops():
        n += int(ops().fault_repairs(bool(reset)))
    return n


class exhaustive_search:
    """Context manager: evaluate every MSE candidate (the reference's 200 full passes)
    instead of the default two-stage exact search. Results are bit-identical; used
    for A/B timing and as a cross-check in the parity tests."""

    def __init__(self, enable: bool = True):
        self.enable = enable

    def __enter__(self):
        load().admmq_set_exhaustive_search(1 if self.enable else 0)
        return self

    def __exit__(self, *exc):
        load().admmq_set_exhaustive_search(0)
        return False


class sel_widen:
    """Context manager (diagnostics): keep every candidate in the two-stage search's
    selected set, so its multi-candidate paths - the canonical SSEs, and in the fused
    finalize the record published before the ready word, and the thin loop's stage 2 - run
    on every call. The answer is exact either way, so the bits are the same."""

    def __enter__(self):
        check(load().admmq_debug_set_sel_widen(1), "sel_widen")
        return self

    def __exit__(self, *exc):
        check(load().admmq_debug_set_sel_widen(0), "sel_widen")
        return False


class solve_mode:
    """Context manager: the process default of the per-iteration solve's operand form,
    ``"fp32"`` (default: fp32 MFMA, the reference's arithmetic) or ``"split"`` (fp16
    hi/lo planes on f16 MFMA, opt-in). Restores the previous mode on exit."""

    MODES = SOLVE_MODES

    def __init__(self, mode: str):
        if mode not in self.MODES:
            raise ValueError(mode)
        self.mode = mode

    def __enter__(self):
        self.prev = load().admmq_get_solve_mode()
        check(load().admmq_set_solve_mode(self.MODES[self.mode]), "set_solve_mode")
        return self

    def __exit__(self, *exc):
        load().admmq_set_solve_mode(self.prev)
        return False


class fin_nv3:
    """Context manager: let the search take three float4 groups per thread where that keeps
    the finalize in the search launch (default), or at most two (planned at prepare, so the
    manager must enclose the whole call). Same integers. Restores the default on exit."""

    def __init__(self, enable: bool):
        self.enable = enable

    def __enter__(self):
        load().admmq_debug_set_fin_nv3(1 if self.enable else 0)
        return self

    def __exit__(self, *exc):
        load().admmq_debug_set_fin_nv3(1)
        return False


class fused_finalize:
    """Context manager: run the big jobs' finalize step inside the search launch
    (default, where all of its blocks are resident) or as its own launch. Same
    integers; used as a cross-check in the parity tests. Restores the default on exit."""

    def __init__(self, enable: bool):
        self.enable = enable

    def __enter__(self):
        load().admmq_debug_set_fused_finalize(1 if self.enable else 0)
        return self

    def __exit__(self, *exc):
        load().admmq_debug_set_fused_finalize(1)
        return False


class fin_wait_polls:
    """Context manager (diagnostics): polls of the fused finalize's bounded wait for its
    job's selection (1 forces the timeout / internal-fault path). Restores the default."""

    def __init__(self, polls: int):
        self.polls = polls

    def __enter__(self):
        check(load().admmq_debug_set_fin_wait_polls(int(self.polls)), "fin_wait_polls")
        return self

    def __exit__(self, *exc):
        load().admmq_debug_set_fin_wait_polls(0)
        return False


class fin_capacity:
    """Context manager (diagnostics): resident-block budget of the fused finalize (0: the
    device's). A small budget forces its several-units-per-block form."""

    def __init__(self, blocks: int):
        self.blocks = blocks

    def __enter__(self):
        check(load().admmq_debug_set_fin_capacity(int(self.blocks)), "fin_capacity")
        return self

    def __exit__(self, *exc):
        load().admmq_debug_set_fin_capacity(0)
        return False


class thin_loop:
    """Context manager: the persistent loop of the thin factors (k_thin_loop: every
    iteration of a call whose factors all have I <= 16 in one launch; default on) or the
    per-iteration launches; ``"wide"``: on, with 64-column workgroups wherever allowed
    (ld <= 512; normally only when 32-column teams would not fit on the CUs). Restores the
    default on exit."""

    def __init__(self, enable):
        self.enable = enable

    def __enter__(self):
        code = 2 if self.enable == "wide" else (1 if self.enable else 0)
        check(load().admmq_debug_set_thin_loop(code), "thin_loop")
        return self

    def __exit__(self, *exc):
        load().admmq_debug_set_thin_loop(1)
        return False


class search_units_per_block:
    """Context manager: stage-1 units per block of the search launch that runs without the
    fused finalize (0 = the planner's choice). Same integers for any value; used as a
    cross-check in the parity tests. Restores the planner's choice on exit."""

    def __init__(self, reps: int):
        self.reps = reps

    def __enter__(self):
        check(load().admmq_debug_set_search_units_per_block(int(self.reps)), "search_units_per_block")
        return self

    def __exit__(self, *exc):
        load().admmq_debug_set_search_units_per_block(0)
        return False


class stage1_form:
    """Context manager: run stage 1 of the two-stage search in its per-level form
    (``"legacy"``, k_mse_hist) or its merged-threshold form (``"merged"``,
    k_mse_prep2 + k_mse_hist2). Both produce the same integers; used as a
    cross-check in the parity tests. Restores the merged default on exit."""

    def __init__(self, form: str):
        if form not in ("legacy", "merged"):
            raise ValueError(form)
        self.form = form

    def __enter__(self):
        load().admmq_debug_set_legacy_stage1(1 if self.form == "legacy" else 0)
        return self

    def __exit__(self, *exc):
        load().admmq_debug_set_legacy_stage1(0)
        return False
