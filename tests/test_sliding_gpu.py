"""Sliding-window inference on the device (reference test.py:96-186 + TestModel) against the
oracle's restatement of the host loop.

* mragan_patch_gather: bit-exact to numpy's (v − 127.5)/127.5 on the same patches;
* mragan_patch_combine: bit-exact to the reference's fp32 accumulation loop for the same
  predictions (order of the patches, float32 sums from 0, count, + 0.01);
* whole pipeline with a real generator (engine, batched patches) vs the fp64 oracle generator
  run patch by patch: rel ≤ 1e-4 in exact f32 / 1e-3 in bf16x3 (the north-star value gates)."""
import random
import sys

import numpy as np
import pytest
import torch

from oracle.cyclegan_oracle import (generator_forward, resnet_generator_layers, sliding_window_inference,
                                    sliding_window_starts)

pytestmark = pytest.mark.gpu


def test_gather_bit_exact():
    from mragan_hip import ops
    rng = np.random.default_rng(1)
    vol = (rng.random((40, 36, 34)) * 255).astype(np.float32)
    starts = sliding_window_starts(vol.shape, (24, 24, 16), 16, 12)
    st = torch.tensor(starts, dtype=torch.int32, device="cuda")
    out = ops.patch_gather(torch.from_numpy(vol).cuda(), st, (24, 24, 16)).cpu().numpy()
    for p, (i, j, k) in enumerate(starts):
        want = (vol[i:i + 24, j:j + 24, k:k + 16] - 127.5) / 127.5
        np.testing.assert_array_equal(out[p, ..., 0], want)


@pytest.mark.parametrize("shape,patch,s_in,s_lay", [((40, 36, 34), (24, 24, 16), 16, 12),
                                                     ((64, 64, 64), (64, 64, 64), 32, 32),
                                                     ((50, 70, 66), (32, 32, 32), 32, 16)])
def test_combine_bit_exact(shape, patch, s_in, s_lay):
    from mragan_hip import ops
    starts = sliding_window_starts(shape, patch, s_in, s_lay)
    g = torch.Generator().manual_seed(2)
    preds = torch.rand((len(starts),) + patch, generator=g) * 2 - 1
    it = iter(range(len(starts)))
    # the oracle's host loop with a "generator" that replays the stored predictions in order
    want = sliding_window_inference(lambda x: preds[next(it)], np.zeros(shape, np.float32), patch, s_in, s_lay)
    got = ops.patch_combine(preds.cuda(), shape, patch, s_in, s_lay).cpu().numpy()
    np.testing.assert_array_equal(got, want)


def _test_model(tmp_path, precision):
    from models import create_model
    from options.test_options import TestOptions
    argv = sys.argv
    try:
        sys.argv = ["test.py", "--checkpoints_dir", str(tmp_path), "--netG", "resnet_6blocks", "--ngf", "8",
                    "--conv_precision", precision]
        opt = TestOptions().gather_options()
    finally:
        sys.argv = argv
    opt.isTrain, opt.gpu_ids = False, 0
    torch.manual_seed(11)
    random.seed(11)
    return create_model(opt)


def _oracle_state(net):
    return {k: v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu().clone()
            for k, v in net.state_dict().items()}


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_inference_volume_vs_oracle(tmp_path, precision):
    from mragan_hip import ops
    from mragan_hip.sliding_window import inference_volume
    model = _test_model(tmp_path, precision)
    state = _oracle_state(model.netG)               # before: the oracle replays the same calls
    rng = np.random.default_rng(3)
    vol = (rng.random((40, 36, 33)) * 255).astype(np.float32)    # odd z: the edge pad of test.py:101-108
    patch = (24, 24, 24)
    try:
        got = inference_volume(model, vol, patch, 16, 8, patches_per_launch=5)
    finally:
        ops.set_conv_precision("f32")
    params = {k: v for k, v in state.items() if k.endswith(".weight") or k.endswith(".bias")}
    layers = resnet_generator_layers(1, 1, 8, 6)
    want = sliding_window_inference(lambda x: generator_forward(state, params, layers, x.double()), vol, patch, 16, 8)
    assert got.shape == want.shape == vol.shape
    err = float(np.linalg.norm(got.astype(np.float64) - want) / np.linalg.norm(want))
    tol = {"f32": 1e-4, "bf16x3": 1e-3}[precision]
    assert err < tol, err
    # running statistics: one update per patch, in the reference's order (train-mode IN, test.py
    # never calls eval())
    after = model.netG.state_dict()
    for k, v in state.items():
        if "running" in k:
            r = float((after[k].cpu().double() - v).norm() / v.norm())
            assert r < tol, (k, r)


def test_testmodel_forward_matches_generator(tmp_path):
    model = _test_model(tmp_path, "f32")
    x = torch.randn(1, 1, 24, 24, 24)
    model.set_input(x)
    model.test()
    vis = model.get_current_visuals()
    assert tuple(vis["fake_B"].shape) == (1, 1, 24, 24, 24)
    state = {k: v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu()
             for k, v in model.netG.state_dict().items()}
    params = {k: v for k, v in state.items() if k.endswith(".weight") or k.endswith(".bias")}
    want = generator_forward(state, params, resnet_generator_layers(1, 1, 8, 6), x.double())
    err = float((vis["fake_B"].cpu().double() - want).norm() / want.norm())
    assert err < 1e-4, err
