"""The engine's log (csrc/ce_glibc_log.hpp) is glibc's f64 log restated: the
log scipy.special.entr calls inside scipy.stats.entropy (amg_test.py:443, :451,
:479).  Here its host build (ce_log_f64_host, the same source the device
compiles) is compared bit for bit with this image's libm log on every branch
of the algorithm; tests/test_gpu_parity.py repeats the check on the device."""
import ctypes

import numpy as np
import pytest

from oracle import ce_oracle as O


def host_log(x):
    from ce_amd import _lib

    L = _lib.load()
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    rc = L.ce_log_f64_host(x.ctypes.data_as(ctypes.c_void_p), x.size, y.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return y


@pytest.mark.parametrize("seed", [1987, 2021])
def test_restated_log_matches_libm(seed):
    x = O.log_test_arguments(3_000_000, seed)
    assert O.oracle_log_check(x, host_log(x)) == 0


def test_restated_log_entropy_terms():
    """Arguments as entr sees them: p = mean / row sum of Dirichlet / quantised rows."""
    rng = np.random.default_rng(7)
    P = rng.dirichlet(np.ones(4), 500_000)
    P = np.concatenate([P, np.round(P * 8) / 8 + 1e-300, rng.random((1000, 4)) ** 40])
    p = (P / P.sum(1, keepdims=True)).ravel()
    p = p[p > 0]
    assert O.oracle_log_check(p, host_log(p)) == 0


def test_log_special_values():
    x = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, -2.0, 1.0, 5e-324])
    y = host_log(x)
    assert y[0] == -np.inf and y[1] == -np.inf and y[2] == np.inf
    assert np.isnan(y[3]) and np.isnan(y[4]) and np.isnan(y[5])
    assert y[6] == 0.0 and not np.signbit(y[6])
    assert y[7] == np.log(5e-324)


def host_exp(x):
    from ce_amd import _lib

    L = _lib.load()
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    rc = L.ce_exp_f64_host(x.ctypes.data_as(ctypes.c_void_p), x.size, y.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return y


@pytest.mark.parametrize("seed", [1987, 2021])
def test_restated_exp_matches_libm(seed):
    """csrc/ce_glibc_exp.hpp (glibc's exp, the x86-64 FMA variant's evaluation)
    against this image's libm exp on every branch, bit for bit."""
    x = O.exp_test_arguments(3_000_000, seed)
    assert O.oracle_exp_check(x, host_exp(x)) == 0


def test_exp_special_values():
    x = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 710.0, -746.0, -745.0])
    y = host_exp(x)
    assert y[0] == 1.0 and y[1] == 1.0 and y[2] == np.inf and y[3] == 0.0 and np.isnan(y[4])
    assert y[5] == np.inf and y[6] == 0.0 and not np.signbit(y[6]) and y[7] == 5e-324
