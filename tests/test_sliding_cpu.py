"""Sliding-window inference, host side (reference test.py:38-207, models/test_model.py):
the patch visit order against the oracle's restatement of test.py:111-143, the array helpers,
and `--model test` resolving to TestModel with the reference's options."""
import sys

import numpy as np
import pytest

from oracle.cyclegan_oracle import sliding_window_starts


@pytest.mark.parametrize("shape,patch,s_in,s_lay", [
    ((64, 64, 64), (64, 64, 64), 32, 32),
    ((100, 90, 70), (64, 64, 64), 32, 32),
    ((65, 64, 97), (32, 32, 48), 16, 20),
    ((40, 36, 34), (24, 24, 24), 16, 16),
    ((33, 33, 33), (32, 32, 32), 64, 64),      # stride larger than the remainder
])
def test_patch_order_matches_reference_loop(shape, patch, s_in, s_lay):
    from mragan_hip.sliding_window import patch_starts
    got, grid = patch_starts(shape, patch, s_in, s_lay)
    want = sliding_window_starts(shape, patch, s_in, s_lay)
    assert got == want
    assert len(got) == grid[0] * grid[1] * grid[2]
    # every voxel is covered
    cover = np.zeros(shape, dtype=np.int32)
    for i, j, k in got:
        cover[i:i + patch[0], j:j + patch[1], k:k + patch[2]] += 1
    assert cover.min() >= 1


def test_pad_and_normalize():
    from mragan_hip.sliding_window import normalize_0_255, pad_to_patch
    rng = np.random.default_rng(0)
    x = rng.normal(size=(20, 30, 70)).astype(np.float32)
    n = normalize_0_255(x)
    assert n.dtype == np.float32 and abs(float(n.min())) < 1e-4 and abs(float(n.max()) - 255) < 1e-3
    p = pad_to_patch(n, (32, 32, 64))
    assert p.shape == (32, 32, 70)
    np.testing.assert_array_equal(p[:20, :30, :], n)
    assert not p[20:].any() and not p[:, 30:].any()


def test_model_test_resolves(tmp_path):
    from models import create_model
    from options.test_options import TestOptions
    argv = sys.argv
    try:
        sys.argv = ["test.py", "--checkpoints_dir", str(tmp_path), "--netG", "resnet_6blocks", "--ngf", "8",
                    "--model_suffix", "_A"]
        opt = TestOptions().gather_options()
    finally:
        sys.argv = argv
    opt.isTrain = False
    opt.gpu_ids = 0
    assert opt.model == "test" and opt.dataset_mode == "single"
    model = create_model(opt)
    assert type(model).__name__ == "TestModel"
    assert model.model_names == ["G_A"] and model.netG_A is model.netG
    assert model.visual_names == ["real_A", "fake_B"] and model.loss_names == []
