"""The float64 elementary functions of the fused simulate kernel (topotrafficrl_amd/csrc/ttrl_math.h),
built for the host from the same header: error in ulps against numpy's extended-precision functions
over the argument ranges the simulator produces, and special values.

The kernel computes every one of these functions with explicit fma / single IEEE operations
(-ffp-contract=off), so the host build returns the device's bits; the GPU parity tests then hold
the whole step to the oracle's tolerances."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = r"""
#include "ttrl_math.h"
extern "C" {
void v_sincos(const double* x, double* s, double* c, long n) { for (long i = 0; i < n; ++i) ttrl_math::sincos_d(x[i], s[i], c[i]); }
void v_atan(const double* x, double* y, long n) { for (long i = 0; i < n; ++i) y[i] = ttrl_math::atan_d(x[i]); }
void v_asin(const double* x, double* y, long n) { for (long i = 0; i < n; ++i) y[i] = ttrl_math::asin_d(x[i]); }
void v_log(const double* x, double* y, long n) { for (long i = 0; i < n; ++i) y[i] = ttrl_math::log_d(x[i]); }
void v_exp(const double* x, double* y, long n) { for (long i = 0; i < n; ++i) y[i] = ttrl_math::exp_d(x[i]); }
void v_pow(const double* x, const double* e, double* y, long n) { for (long i = 0; i < n; ++i) y[i] = ttrl_math::pow_d(x[i], e[i]); }
}
"""
P = ctypes.POINTER(ctypes.c_double)


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("ttrl_math")
    src = d / "shim.cpp"
    src.write_text(SHIM)
    so = d / "shim.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-I",
                    os.path.join(ROOT, "topotrafficrl_amd", "csrc"), "-o", str(so), str(src)], check=True)
    return ctypes.CDLL(str(so))


def _p(a):
    return a.ctypes.data_as(P)


def ulps(got, ref_ld):
    """|got - ref| in units of the float64 spacing at ref (ref in extended precision)."""
    return float(np.max(np.abs(got.astype(np.longdouble) - ref_ld) / np.spacing(np.abs(ref_ld.astype(np.float64)))))


N = 200_000
rng = np.random.default_rng(0)


@pytest.mark.parametrize("lo,hi", [(-1, 1), (-4, 4), (-100, 100), (-1e5, 1e5)])
def test_sincos(lib, lo, hi):
    x = rng.uniform(lo, hi, N)
    s, c = np.empty(N), np.empty(N)
    lib.v_sincos(_p(x), _p(s), _p(c), N)
    xl = x.astype(np.longdouble)
    assert ulps(s, np.sin(xl)) <= 1.6 and ulps(c, np.cos(xl)) <= 1.6


@pytest.mark.parametrize("lo,hi", [(-0.5, 0.5), (-3, 3), (-100, 100), (-1e8, 1e8)])
def test_atan(lib, lo, hi):
    x = rng.uniform(lo, hi, N)
    y = np.empty(N)
    lib.v_atan(_p(x), _p(y), N)
    assert ulps(y, np.arctan(x.astype(np.longdouble))) <= 1.6


@pytest.mark.parametrize("lo,hi", [(-0.5, 0.5), (-1, 1)])
def test_asin(lib, lo, hi):
    x = rng.uniform(lo, hi, N)
    y = np.empty(N)
    lib.v_asin(_p(x), _p(y), N)
    assert ulps(y, np.arcsin(x.astype(np.longdouble))) <= 2.5


def test_log_exp_pow(lib):
    x = np.concatenate([rng.uniform(1e-3, 2, N), np.exp(rng.uniform(-690, 690, N))])
    y = np.empty(len(x))
    lib.v_log(_p(x), _p(y), len(x))
    assert ulps(y, np.log(x.astype(np.longdouble))) <= 1.0
    e = rng.uniform(-700, 700, N)
    y = np.empty(N)
    lib.v_exp(_p(e), _p(y), N)
    assert ulps(y, np.exp(e.astype(np.longdouble))) <= 1.0
    # the range edges: the top binade up to overflow, and the gradual-underflow tail (one rounding
    # to the subnormal grid, whose spacing is 2^-1074)
    e = np.concatenate([rng.uniform(700, 709.78, N // 10), rng.uniform(-745.13, -708, N // 10)])
    y = np.empty(len(e))
    lib.v_exp(_p(e), _p(y), len(e))
    ref = np.exp(e.astype(np.longdouble))
    err = np.abs(y.astype(np.longdouble) - ref) / np.maximum(np.spacing(ref.astype(np.float64)), 2.0 ** -1074)
    assert float(np.max(err)) <= 1.0 and np.isfinite(y).all() and (y > 0).all()
    # the IDM free-road term: (v / v0) ^ DELTA, ratio in [0, 1.5], DELTA in [3.5, 4.5]; exp(y log x)
    # carries the rounding of y log x into the result, ~|y log x| ulps (the kernel's pow before this
    # header was the same composition of ocml's exp and log)
    r, d = rng.uniform(0, 1.5, N), rng.uniform(3.5, 4.5, N)
    y = np.empty(N)
    lib.v_pow(_p(r), _p(d), _p(y), N)
    ref = np.power(r.astype(np.longdouble), d.astype(np.longdouble))
    rel = np.abs(y - ref) / np.maximum(ref, 1e-300)
    bound = (1 + np.abs(d * np.log(np.maximum(r, 1e-300)))) * 2.3e-16
    assert bool(np.all(rel <= bound)) and float(np.max(rel[r > 0.5])) < 2e-15


def test_special_values(lib):
    x = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-310, 1e300])
    for name, ref in (("v_atan", np.arctan), ("v_log", np.log), ("v_exp", np.exp)):
        y = np.empty(len(x))
        getattr(lib, name)(_p(x), _p(y), len(x))
        with np.errstate(all="ignore"):
            want = ref(x)
        close = np.isclose(y, want, rtol=4e-16, atol=0) | (np.isnan(y) & np.isnan(want)) | (y == want)
        assert close.all(), (name, x[~close], y[~close], want[~close])
    x = np.array([0.0, -0.0, 1.0, -1.0, 0.5, -0.5, np.nan])
    y = np.empty(len(x))
    lib.v_asin(_p(x), _p(y), len(x))
    want = np.arcsin(x)
    assert (np.isclose(y, want, rtol=5e-16, atol=0) | (np.isnan(y) & np.isnan(want))).all()
    assert np.signbit(y[1]) and not np.signbit(y[0])  # asin(-0) = -0
    r, d = np.array([0.0, 1.0]), np.array([4.0, 4.0])
    y = np.empty(2)
    lib.v_pow(_p(r), _p(d), _p(y), 2)
    assert y[0] == 0.0 and y[1] == 1.0
