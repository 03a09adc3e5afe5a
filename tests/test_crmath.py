"""include/fm3d_crmath.h -- the correctly rounded sin, cos, atan2 and exp of the LM kernel and of the
oracle's DETMATH mode -- pinned against mpmath at 200 bits, through the oracle's
orc_math_eval (the same header the GPU compiles).  CPU only.

Inputs: the ranges the LM feeds them (angles of a few radians, exponents of the LM's weights),
the reduction's hard cases (multiples of pi/2 rounded to double, the Cody-Waite range's end 2^19),
signed zeros, subnormals and the axes of atan2.  Every result must be mpmath's value rounded to
nearest; the 1-ulp polynomials (fm3d_detmath.h, DET_1ULP; the NCC hypotheses) within one ulp."""
import math

import numpy as np
import pytest

mpmath = pytest.importorskip("mpmath")
mp = mpmath.mp


def _ref(fn, x, y=None):
    with mpmath.workprec(200):
        if fn == "sin":
            return np.array([float(mpmath.sin(mpmath.mpf(v))) for v in x])
        if fn == "cos":
            return np.array([float(mpmath.cos(mpmath.mpf(v))) for v in x])
        if fn == "exp":
            return np.array([float(mpmath.exp(mpmath.mpf(v))) for v in x])
        return np.array([float(mpmath.atan2(mpmath.mpf(a), mpmath.mpf(b))) for a, b in zip(x, y)])


def _mismatch(got, ref):
    """indices where the bits differ (mpmath has no signed zero: a zero matches either zero)"""
    return np.flatnonzero((got.view(np.int64) != ref.view(np.int64)) & ~((got == 0) & (ref == 0)))


def _angles(rng, n):
    k = np.arange(-40, 41)
    hard = np.concatenate([k * (np.pi / 2), np.nextafter(k * (np.pi / 2), np.inf), np.nextafter(k * (np.pi / 2), -np.inf)])
    return np.concatenate([
        rng.uniform(-4, 4, n), rng.uniform(-100, 100, n // 4), rng.uniform(-2.0 ** 19, 2.0 ** 19, n // 8),
        hard, [0.0, -0.0, 5e-324, -5e-324, 1e-300, 2.0 ** -30, 0.5, 1.0, 2.0, np.pi, 2.0 ** 19 - 1],
        np.nextafter(np.float64(2.0 ** 19), 0.0) * np.array([1.0, -1.0])])


@pytest.mark.parametrize("fn", ["sin", "cos"])
def test_sin_cos_correctly_rounded(orc, fn):
    x = _angles(np.random.default_rng(1), 3000)
    got = orc.math_eval(fn, x)
    ref = _ref(fn, x)
    bad = _mismatch(got, ref)
    assert bad.size == 0, [(x[i], got[i], ref[i]) for i in bad[:5]]
    if fn == "sin":  # odd: the sign of zero kept
        assert np.signbit(orc.math_eval(fn, np.array([-0.0]))[0])
    # the 1-ulp polynomials: within one ulp, and they differ from the correctly rounded results
    # somewhere (which is why the LM moved to these)
    one = orc.math_eval(fn, x, mode=orc.DETMATH | orc.DET_1ULP)
    sel = np.abs(x) < 2.0 ** 19
    ulp = np.spacing(np.abs(ref[sel]))
    assert (np.abs(one[sel] - ref[sel]) <= ulp).all()


def test_atan2_correctly_rounded(orc):
    rng = np.random.default_rng(2)
    y = np.concatenate([rng.normal(size=3000), rng.normal(size=500) * 1e-8, [0.0, -0.0, 0.0, -0.0, 1.0, -1.0, 0.0, 5e-324],
                        rng.uniform(-1, 1, 500)])
    x = np.concatenate([rng.normal(size=3000), rng.normal(size=500), [0.0, 0.0, -0.0, -0.0, 0.0, 0.0, 1.0, -1.0],
                        rng.uniform(-1, 1, 500) * 1e6])
    got = orc.math_eval("atan2", y, x)
    ref = _ref("atan2", y, x)
    axes = (x == 0) | (y == 0)  # signed zeros: IEEE's special values (exact in libm), not mpmath's
    ref[axes] = [math.atan2(a, b) for a, b in zip(y[axes], x[axes])]
    bad = _mismatch(got, ref)
    assert bad.size == 0, [(y[i], x[i], got[i], ref[i]) for i in bad[:5]]
    assert math.copysign(1.0, orc.math_eval("atan2", np.array([-0.0]), np.array([1.0]))[0]) == -1.0


def test_exp_correctly_rounded(orc):
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(-40, 40, 3000), rng.uniform(-1e-3, 1e-3, 300), rng.uniform(-700, 700, 300),
                        [0.0, -0.0, 1.0, -1.0, 1e-300, -1e-300, 709.0, -700.0]])
    got = orc.math_eval("exp", x)
    ref = _ref("exp", x)
    bad = _mismatch(got, ref)
    assert bad.size == 0, [(x[i], got[i], ref[i]) for i in bad[:5]]


def test_libm_differs_somewhere(orc):
    """This image's glibc is not what the GPU computes: over random angles its sin or cos differs
    from the correctly rounded value on some inputs (or agrees everywhere -- then the STRICT and
    DETMATH modes coincide for these functions and tools/full_parity.py's attribution says so)."""
    x = np.random.default_rng(4).uniform(-4, 4, 20000)
    d = sum(int((orc.math_eval(f, x, mode=orc.STRICT) != orc.math_eval(f, x)).sum()) for f in ("sin", "cos"))
    print(f"libm sin/cos differ from the correctly rounded value on {d} of {2 * len(x)} inputs")


def test_hypot_correctly_rounded(orc):
    """fm3d_hypot_cr -- the rotation's hypot in OpenCV's JacobiSVDImpl_ (include/fm3d_cvsvd.h, the DLT
    and the polar factor) -- is mpmath's sqrt(x^2 + y^2) rounded to nearest, over random pairs of
    mixed magnitudes (the DLT's p and beta span many decades), equal pairs, zeros, the 2^-60 cut,
    scaled extremes and non-finite values; glibc's hypot here is not correctly rounded everywhere."""
    rng = np.random.default_rng(6)
    n = 6000
    x = rng.normal(size=n) * 10.0 ** rng.uniform(-12, 12, n)
    y = rng.normal(size=n) * 10.0 ** rng.uniform(-12, 12, n)
    hard = np.array([[3.0, 4.0], [1.0, 1.0], [0.0, 0.0], [-0.0, 5.0], [1.0, 2.0 ** -61], [1.0, 2.0 ** -59],
                     [1e300, 1e300], [1e-300, 3e-300], [5e-324, 5e-324], [1.5e308, 1.5e308], [2.0 ** 500, 1.0]])
    x = np.concatenate([x, hard[:, 0]])
    y = np.concatenate([y, hard[:, 1]])
    got = orc.math_eval("hypot", x, y)
    with mpmath.workprec(300):
        ref = np.array([float(mpmath.sqrt(mpmath.mpf(a) ** 2 + mpmath.mpf(b) ** 2)) for a, b in zip(x, y)])
    bad = _mismatch(got, ref)
    assert bad.size == 0, [(x[i], y[i], got[i], ref[i]) for i in bad[:5]]
    inf, nan = float("inf"), float("nan")
    sp = orc.math_eval("hypot", np.array([inf, nan, -inf, nan]), np.array([nan, inf, 1.0, 1.0]))
    assert sp[0] == inf and sp[1] == inf and sp[2] == inf and np.isnan(sp[3])
    libm = orc.math_eval("hypot", x[:n], y[:n], mode=orc.STRICT)
    print(f"libm hypot differs from the correctly rounded value on {int((libm != got[:n]).sum())} of {n} pairs")
