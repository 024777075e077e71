"""Shared assertions for the GPU parity tests (no fixtures, no GPU calls)."""
import numpy as np


def assert_sub_close(sub, exp, tol=1e-5):
    """NaN exactly where the check rejected the pixel,
    elsewhere the f32 parabola within the stated 1e-5 px."""
    assert np.array_equal(np.isnan(sub), np.isnan(exp))
    ok = ~np.isnan(exp)
    assert np.isnan(exp).any() and ok.any()
    assert np.max(np.abs(sub[ok] - exp[ok])) <= tol
