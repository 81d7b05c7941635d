"""The parity gates themselves: a NaN anywhere must fail them (`err > env` is False
for a NaN error, so a NaN tensor used to pass the per-tensor gradient gate)."""
import numpy as np
import pytest
import torch

from golden_util import assert_finite, over_envelope, rel_err


def test_nan_gradient_fails_per_tensor_gate():
    ref = np.linspace(-1.0, 1.0, 64)
    got = ref.copy()
    got[17] = np.nan
    err = rel_err(got, ref)
    assert np.isnan(err)
    assert not (err > 1e-3)                # the old comparison let it through
    assert over_envelope(err, 1e-3)        # the gate's verdict now counts it
    assert over_envelope(np.inf, 1e-3)
    assert not over_envelope(rel_err(ref, ref), 1e-3)
    with pytest.raises(AssertionError):
        assert_finite("grad", got)


def test_assert_finite_whole_tensor():
    t = torch.zeros(4, 5, 6)
    assert_finite("t", t, np.ones(3))
    t[3, 4, 5] = float("inf")
    with pytest.raises(AssertionError):
        assert_finite("t", t)


def test_check_outliers_rejects_nan_entries():
    from test_step_gpu import check_outliers
    check_outliers("ok", [("G_A", "w", 2e-3, 1e-3)], 64)
    with pytest.raises(AssertionError):
        check_outliers("nan", [("G_A", "w", float("nan"), 1e-3)], 64)
