"""Training-loop side of the reference (train.py:35-147), CPU checks:

* the patch sampler's host logic (normalisation, foreground crop, RandCropByPosNegLabeld centres
  with MONAI's draw order) against the oracle's independent restatement of MONAI's algorithm —
  MONAI is an unpinned third-party dependency absent here, so beyond this restatement the sampler
  is "parity unpinned";
* the LambdaLR schedule of get_scheduler (networks3D.py:27-41) over the reference's 600 epochs;
* the loss_log.txt / stdout line format (utils/visualizer.py:20-27);
* the epoch loop's cadence (train.py:78-147): prints, 'latest' saves, per-epoch saves, one
  update_learning_rate per epoch — driven with a stub model and sampler."""
import os
import re
import sys
import types

import numpy as np
import pytest
import torch

from oracle.cyclegan_oracle import monai_crop_foreground, monai_normalize_intensity, monai_pos_neg_crops


def _volume(seed, shape=(30, 26, 22)):
    rng = np.random.default_rng(seed)
    img = rng.normal(2.0, 3.0, size=shape).astype(np.float32)
    img[:3] = -5.0                                   # a non-positive slab: the foreground crop trims it
    lab = (rng.random(shape) < 0.02).astype(np.float32)
    return img, lab


@pytest.mark.parametrize("seed,patch,ns", [(0, (16, 16, 16), 2), (1, (24, 8, 20), 3), (2, (27, 26, 19), 2)])
def test_sampler_host_logic_matches_monai_restatement(seed, patch, ns):
    from mragan_hip.patch_sampler import crop_centers, foreground_box, normalize_intensity
    img, lab = _volume(seed)
    n1 = normalize_intensity(img)
    n2 = monai_normalize_intensity(img)
    np.testing.assert_array_equal(n1, n2)
    (x0, y0, z0), (x1, y1, z1) = foreground_box(n1)
    ci, cl = monai_crop_foreground(n2, lab)
    np.testing.assert_array_equal(n1[x0:x1, y0:y1, z0:z1], ci)
    lab_c = lab[x0:x1, y0:y1, z0:z1]
    fg = np.flatnonzero(lab_c.ravel() != 0)
    for trial in range(5):
        centers = crop_centers(ci.shape, patch, fg, ns, np.random.RandomState(100 + trial))
        want = monai_pos_neg_crops(ci, cl, list(patch), ns, np.random.RandomState(100 + trial))
        assert len(centers) == len(want) == ns
        for c, (wi, wl) in zip(centers, want):
            s = [ci_ - p // 2 for ci_, p in zip(c, patch)]
            sl = tuple(slice(s[i], s[i] + patch[i]) for i in range(3))
            assert all(0 <= s[i] and s[i] + patch[i] <= ci.shape[i] for i in range(3))
            np.testing.assert_array_equal(ci[sl], wi)
            np.testing.assert_array_equal(cl[sl], wl)


def test_lambda_lr_trajectory_600_epochs():
    """networks3D.py:27-41 LambdaLR: lr_e = lr · (1 − max(0, e + 1 + epoch_count − niter) / (niter_decay + 1)),
    stepped once per epoch by update_learning_rate (train.py:147) — the engine's FusedAdam drives the
    same torch scheduler."""
    from models import networks3D
    from models.cycle_gan_model import FusedAdam
    opt = types.SimpleNamespace(lr_policy="lambda", epoch_count=1, niter=500, niter_decay=100)
    net = torch.nn.Linear(2, 2)
    optim = FusedAdam([net], lr=2e-4, betas=(0.5, 0.999))
    sched = networks3D.get_scheduler(optim, opt)
    got = []
    for epoch in range(opt.epoch_count, opt.niter + opt.niter_decay + 1):
        got.append(optim.param_groups[0]["lr"])
        optim._opt_called = True
        sched.step()
    # the lambda sees the scheduler's step count e = 0, 1, …: lr_e = lr·(1 − max(0, e+1+epoch_count−niter)/(niter_decay+1))
    want = [2e-4 * (1.0 - max(0, e + 1 + opt.epoch_count - opt.niter) / float(opt.niter_decay + 1)) for e in range(600)]
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-20)
    assert got[498] == pytest.approx(2e-4) and got[499] == pytest.approx(2e-4 * 100 / 101)
    assert got[-1] == 0.0                      # the reference's schedule reaches 0 in its last epoch


def test_loss_log_format(tmp_path):
    from utils.visualizer import Visualizer
    opt = types.SimpleNamespace(name="exp", checkpoints_dir=str(tmp_path))
    v = Visualizer(opt)
    v.print_current_losses(3, 12, {"D_A": 0.25, "G_A": 1.0, "cycle_A": 3.14159}, 0.1234, 0.0)
    lines = open(os.path.join(tmp_path, "exp", "loss_log.txt")).read().splitlines()
    assert re.match(r"^================ Training Loss \(.+\) ================$", lines[0])
    assert lines[1] == "(epoch: 3, iters: 12, time: 0.123, data: 0.000) D_A: 0.250 G_A: 1.000 cycle_A: 3.142 "


class _StubModel:
    def __init__(self):
        self.calls = []

    def set_input(self, x):
        self.calls.append(("set_input", tuple(x[0].shape)))

    def optimize_parameters(self):
        self.calls.append(("step",))

    def get_current_losses(self):
        return {"D_A": 0.5}

    def save_networks(self, which):
        self.calls.append(("save", which))

    def sync_running_stats(self):
        self.calls.append(("sync",))

    def update_learning_rate(self):
        self.calls.append(("lr",))


def test_epoch_loop_cadence(tmp_path):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mra-gan_amd"))
    import train as T
    opt = types.SimpleNamespace(epoch_count=1, niter=2, niter_decay=1, print_freq=2, save_latest_freq=3,
                                save_epoch_freq=2, batch_size=1, name="loop", checkpoints_dir=str(tmp_path))
    batches = [{"image": torch.zeros(2, 1, 4, 4, 4), "label": torch.zeros(2, 1, 4, 4, 4)}] * 4
    m = _StubModel()
    T.train(opt, batches, model=m, log=lambda *_: None)
    steps = sum(1 for c in m.calls if c[0] == "step")
    assert steps == 3 * 4
    saves = [c[1] for c in m.calls if c[0] == "save"]
    # 'latest' every 3 iterations (12 in all), 'latest' + '2' at the end of epoch 2
    assert saves == ["latest", "latest", "latest", 2, "latest", "latest"]   # steps 3, 6, end of epoch 2, 9, 12
    assert sum(1 for c in m.calls if c[0] == "lr") == 3
    # the data-parallel running-statistics average precedes every save point (one collective each)
    assert [c[0] for c in m.calls if c[0] in ("sync", "save")] == \
        ["sync", "save", "sync", "save", "sync", "save", "save", "sync", "save", "sync", "save"]
    log = open(os.path.join(tmp_path, "loop", "loss_log.txt")).read().splitlines()
    assert len(log) == 1 + 6                         # header + one line every 2 iterations
    assert log[1].startswith("(epoch: 1, iters: 2, time: ")
