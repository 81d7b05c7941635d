"""Device patch sampler and the train.py loop on the GPU (reference train.py:35-147).

* mragan_crop_patches: bit-exact to numpy slicing;
* GpuPatchSampler batches: bit-exact to the oracle's restatement of the MONAI pipeline
  (normalise → foreground crop → RandCropByPosNegLabeld(pos=20, neg=0, num_samples=2)) with the
  same RandomState draws, list_data_collate order;
* train.train() for two epochs on .npy volumes with the real model: loss_log lines, 'latest' and
  per-epoch checkpoints written, LambdaLR stepped once per epoch."""
import os
import random
import sys

import numpy as np
import pytest
import torch

from oracle.cyclegan_oracle import monai_crop_foreground, monai_normalize_intensity, monai_pos_neg_crops

pytestmark = pytest.mark.gpu


def test_crop_bit_exact():
    from mragan_hip import ops
    rng = np.random.default_rng(0)
    vol = rng.normal(size=(31, 29, 27)).astype(np.float32)
    starts = [(0, 0, 0), (15, 13, 11), (7, 3, 9), (15, 0, 11)]
    out = ops.crop_patches(torch.from_numpy(vol).cuda(), torch.tensor(starts, dtype=torch.int32).cuda(),
                           (16, 16, 16)).cpu().numpy()
    for p, (i, j, k) in enumerate(starts):
        np.testing.assert_array_equal(out[p], vol[i:i + 16, j:j + 16, k:k + 16])


def _volumes(n, seed):
    rng = np.random.default_rng(seed)
    vols = []
    for v in range(n):
        shape = (36 + v, 33, 30 + 2 * v)
        img = rng.normal(1.0, 2.0, size=shape).astype(np.float32)
        img[:2] = -3.0
        lab = (rng.random(shape) < 0.03).astype(np.float32)
        vols.append((img, lab))
    return vols


def test_sampler_batches_match_monai_restatement():
    from mragan_hip.patch_sampler import DeviceVolume, GpuPatchSampler
    raw = _volumes(3, 1)
    vols = [DeviceVolume(i, l, torch.device("cuda")) for i, l in raw]
    patch = (24, 24, 20)
    smp = GpuPatchSampler(vols, patch, batch_size=2, num_samples=2, shuffle=False, seed=5)
    rs = np.random.RandomState(5)
    prepped = [monai_crop_foreground(monai_normalize_intensity(i), l) for i, l in raw]
    for b, batch in enumerate(smp):
        idx = list(range(3))[2 * b:2 * b + 2]
        want_i, want_l = [], []
        for v in idx:
            for pi, pl in monai_pos_neg_crops(prepped[v][0], prepped[v][1], list(patch), 2, rs):
                want_i.append(pi)
                want_l.append(pl)
        assert tuple(batch["image"].shape) == (2 * len(idx), 1) + patch
        np.testing.assert_array_equal(batch["image"][:, 0].cpu().numpy(), np.stack(want_i))
        np.testing.assert_array_equal(batch["label"][:, 0].cpu().numpy(), np.stack(want_l))


def test_train_loop_two_epochs(tmp_path):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "mra-gan_amd"))
    import train as T
    from mragan_hip.patch_sampler import GpuPatchSampler
    from options.train_options import TrainOptions
    data = tmp_path / "data"
    os.makedirs(data / "images")
    os.makedirs(data / "labels")
    for v, (img, lab) in enumerate(_volumes(3, 2)):
        np.save(data / "images" / f"{v}.npy", img)
        np.save(data / "labels" / f"{v}.npy", lab)
    argv = sys.argv
    try:
        sys.argv = ["train.py", "--checkpoints_dir", str(tmp_path / "ck"), "--name", "loop", "--data_path", str(data),
                    "--netG", "resnet_6blocks", "--ngf", "8", "--ndf", "8", "--niter", "1", "--niter_decay", "1",
                    "--print_freq", "1", "--save_latest_freq", "2", "--save_epoch_freq", "1", "--batch_size", "2"]
        opt = TrainOptions().gather_options()
    finally:
        sys.argv = argv
    opt.isTrain, opt.gpu_ids = True, 0
    torch.manual_seed(0)
    random.seed(0)
    smp = GpuPatchSampler.from_folder(str(data), (24, 24, 24), torch.device("cuda"), batch_size=2, num_samples=2)
    model = T.train(opt, smp, log=lambda *_: None)
    log = open(tmp_path / "ck" / "loop" / "loss_log.txt").read().splitlines()
    assert len(log) == 1 + 2 * 2                            # 2 epochs × 2 batches (3 volumes, batch 2)
    for net in ("G_A", "G_B", "D_A", "D_B"):
        for which in ("latest", "1", "2"):
            assert os.path.exists(tmp_path / "ck" / "loop" / f"{which}_net_{net}.pth"), (which, net)
    # LambdaLR (networks3D.py:27-41) after two update_learning_rate() calls, niter = niter_decay = 1:
    # lr · (1 − max(0, 2 + 1 + 1 − 1) / 2) = −lr / 2 — the reference's formula, negative past its range
    assert model.optimizers[0].param_groups[0]["lr"] == pytest.approx(-1e-4)
    losses = model.get_current_losses()
    assert all(np.isfinite(v) for v in losses.values())
