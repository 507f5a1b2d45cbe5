"""The EPC multiplier search (csrc/epc_search.h: the state machine shared by the one-workgroup
and the blocked device forms of cp_anc's mode update, source/parafac_epc.py:61-74) built for
the host and driven with e(mu) from an eigen-form spectrum: its root against the oracle's
bisection (oracle/epc_oracle.py _solve_mu) for cold and warm starts, mu = 0 when the
least-squares step keeps the error, and a G that cannot be factorised below a shift (the
search must grow past failed factorisations, never repeat one). Parity unpinned against musco
itself (absent offline); this pins the search to the oracle's root."""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

from oracle import epc_oracle as eo

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = tmp_path_factory.mktemp("epc_search") / "libepc_search_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", os.path.join(HERE, "host", "epc_search_host.cc"),
                    "-o", str(out)], check=True)
    lb = ctypes.CDLL(str(out))
    P, D = ctypes.c_void_p, ctypes.c_double
    lb.epc_search_run.argtypes = [P, P, ctypes.c_int, D, D, D, D, D, P, P]
    lb.epc_search_run.restype = ctypes.c_int
    return lb


def _run(lib, c, s, normY2, delta2, warm, fail_below=-1.0):
    c = np.ascontiguousarray(c, dtype=np.float64)
    s = np.ascontiguousarray(s, dtype=np.float64)
    mu = ctypes.c_double(0.0)
    ev = ctypes.c_int(0)
    rc = lib.epc_search_run(c.ctypes.data, s.ctypes.data, len(c), normY2, delta2, warm, float(s.mean()), fail_below,
                            ctypes.byref(mu), ctypes.byref(ev))
    return rc, mu.value, ev.value


@pytest.mark.parametrize("n,seed", [(5, 1), (134, 2), (1141, 3)])
def test_search_root_matches_oracle(lib, n, seed):
    rng = np.random.default_rng(seed)
    s = rng.random(n) * 10.0 + 1e-3
    c = rng.random(n)
    ls = float(np.sum(c / s))
    normY2 = ls * 1.5
    e0 = normY2 - ls
    for delta2 in (e0 * 1.5, e0 * 2.5, e0 * 0.5):
        ref = eo._solve_mu(torch.from_numpy(c), torch.from_numpy(s), normY2, delta2)
        for warm in (0.0, ref * 1.001, ref * 0.9, ref * 3.0, 1e-3):
            rc, mu, ev = _run(lib, c, s, normY2, delta2, warm)
            assert rc == 0, (delta2, warm)
            if ref == 0.0:
                assert mu == 0.0
            else:
                assert abs(mu - ref) <= 1e-9 * ref, (delta2, warm, mu, ref)
            assert ev <= 40


def test_search_grows_past_failed_factorisations(lib):
    """G + mu I cannot be factorised below a shift (an indefinite G): the search reaches the
    root above it in a bounded number of evaluations and never re-evaluates a failed mu."""
    rng = np.random.default_rng(7)
    n = 60
    s = np.concatenate([np.zeros(20), rng.random(n - 20) * 5.0 + 0.1])
    c = np.concatenate([np.zeros(20), rng.random(n - 20)])
    mu_t = 0.05
    normY2 = float(np.sum(c / np.where(s > 0, s, 1.0))) * 3.0
    delta2 = normY2 - float(np.sum(c * (s + 2 * mu_t) / (s + mu_t) ** 2))
    ref = eo._solve_mu(torch.from_numpy(c), torch.from_numpy(s), normY2, delta2)
    for fail_below in (1e-9, 1e-4, 0.01):
        rc, mu, ev = _run(lib, c, s, normY2, delta2, 0.0, fail_below=fail_below)
        assert rc == 0, fail_below
        assert abs(mu - ref) <= 1e-9 * ref, (fail_below, mu, ref)
        assert ev <= 60
