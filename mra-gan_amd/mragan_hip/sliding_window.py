"""Sliding-window inference on the HIP engine — the reference's test.py:38-207 (`inference`)
driving TestModel (models/test_model.py:7-48), with the volume resident on the device.

The reference loops over patches on the host: slice a patch out of the numpy volume, scale it
(test.py:150), copy it to the GPU, run G on ONE patch, copy the prediction back, and accumulate
it into a float32 host volume with a float64 cover count (test.py:160-168), then divides
(test.py:173).  Here:

* the normalised volume is uploaded once;
* `mragan_patch_gather` cuts a launch's worth of patches (scaled) into an NDHWC batch;
* the generator runs on up to 8 patches per launch (InstanceNorm is per instance, so a batch of
  k patches computes exactly what k single-patch calls compute; the running statistics get the
  k sequential updates the reference's k calls make);
* every prediction stays on the device and `mragan_patch_combine` overlap-averages them in the
  reference's visit order (bit-identical to the host loop for the same predictions).

Host-side steps the reference does with SimpleITK (reading, Resample, Normalization, Padding,
writing; test.py:42-94, 175-205) stay on the host; `normalize_0_255` and `pad_to_patch` restate
the two that change values (NiftiDataset.py:639-651 and :876-930) for array inputs.
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np
import torch

from . import engine, ops

MAX_PATCHES_PER_LAUNCH = 8      # one running-statistics segment per patch (engine table: ≤ 8)


def patch_starts(shape: Sequence[int], patch: Sequence[int], stride_inplane: int, stride_layer: int):
    """test.py:111-143: patch corners in the reference's visit order (x, then y, then z; the last
    patch of an axis clamped to the end).  Returns (starts [n][3], (inum, jnum, knum))."""
    px, py, pz = patch
    inum = int(math.ceil((shape[0] - px) / float(stride_inplane))) + 1
    jnum = int(math.ceil((shape[1] - py) / float(stride_inplane))) + 1
    knum = int(math.ceil((shape[2] - pz) / float(stride_layer))) + 1
    out = []
    for i in range(inum):
        for j in range(jnum):
            for k in range(knum):
                out.append((min(i * stride_inplane, shape[0] - px), min(j * stride_inplane, shape[1] - py),
                            min(k * stride_layer, shape[2] - pz)))
    return out, (inum, jnum, knum)


def normalize_0_255(image: np.ndarray) -> np.ndarray:
    """NiftiDataset.Normalization (NiftiDataset.py:639-651): z-score (sitk.NormalizeImageFilter)
    then rescale to [0, 255] (RescaleIntensityImageFilter); float32 out."""
    x = np.asarray(image, dtype=np.float64)
    x = (x - x.mean()) / x.std(ddof=1)
    lo, hi = x.min(), x.max()
    x = (x - lo) * (255.0 / (hi - lo)) if hi > lo else np.zeros_like(x)
    return x.astype(np.float32)


def pad_to_patch(image: np.ndarray, patch: Sequence[int]) -> np.ndarray:
    """NiftiDataset.Padding (NiftiDataset.py:876-930): grow every axis shorter than the patch to the
    patch size, same origin and spacing, new voxels 0 (the resampler's default value)."""
    target = [max(s, int(p)) for s, p in zip(image.shape, patch)]
    if list(image.shape) == target:
        return image
    out = np.zeros(target, dtype=image.dtype)
    out[:image.shape[0], :image.shape[1], :image.shape[2]] = image
    return out


@torch.no_grad()
def run_generator_patches(net, x: torch.Tensor) -> torch.Tensor:
    """Generator forward on a batch of k ≤ 8 patches (NDHWC), with the running-statistics
    updates of k sequential single-patch calls (what the reference's loop does)."""
    k = x.shape[0]
    if k > MAX_PATCHES_PER_LAUNCH:
        raise ValueError(f"at most {MAX_PATCHES_PER_LAUNCH} patches per launch")
    from models import networks3D
    networks3D.ensure_flat(net)
    plan = net.plan
    ctx = plan.forward(x)
    keep = engine.apply_running_updates(plan.running_entries([(ctx, i, 1) for i in range(k)]), x.device)
    out = ctx.out
    del keep
    return out


@torch.no_grad()
def inference_volume(model, image_np: np.ndarray, patch: Sequence[int], stride_inplane: int, stride_layer: int,
                     patches_per_launch: int = MAX_PATCHES_PER_LAUNCH) -> np.ndarray:
    """test.py:96-186 on a normalised, resampled and padded volume image_np [x, y, z]: returns the
    overlap-averaged label volume (before the final crop to the pre-padding size, test.py:180)."""
    net = model.netG
    if net.output_nc != 1 or net.input_nc != 1:
        raise NotImplementedError("sliding-window inference handles 1-channel volumes (test.py:152-161)")
    if not 1 <= patches_per_launch <= MAX_PATCHES_PER_LAUNCH:
        raise ValueError(f"patches_per_launch must be in 1..{MAX_PATCHES_PER_LAUNCH}")
    dev = model.device
    image_np = np.asarray(image_np, dtype=np.float32)
    odd = image_np.shape[2] % 2 != 0                                        # test.py:101-108
    if odd:
        image_np = np.pad(image_np, ((0, 0), (0, 0), (0, 1)), 'edge')
    patch = tuple(int(p) for p in patch)
    shape = image_np.shape
    if any(p > s for p, s in zip(patch, shape)):
        raise ValueError(f"patch {patch} larger than the (padded) volume {shape}")
    starts, grid = patch_starts(shape, patch, stride_inplane, stride_layer)
    vol = torch.from_numpy(image_np).to(dev)
    st = torch.tensor(starts, dtype=torch.int32).to(dev)
    pred = torch.empty((len(starts),) + patch, device=dev, dtype=torch.float32)
    for p0 in range(0, len(starts), patches_per_launch):
        p1 = min(p0 + patches_per_launch, len(starts))
        x = ops.patch_gather(vol, st[p0:p1], patch)
        y = run_generator_patches(net, x)
        pred[p0:p1].copy_(y.view((p1 - p0,) + patch))
    label = ops.patch_combine(pred, shape, patch, stride_inplane, stride_layer)
    out = label.cpu().numpy()
    if odd:
        out = out[:, :, :out.shape[2] - 1]
    return out


def inference_array(model, image: np.ndarray, patch: Sequence[int], stride_inplane: int, stride_layer: int,
                    patches_per_launch: int = MAX_PATCHES_PER_LAUNCH) -> np.ndarray:
    """The whole array part of test.py:inference: normalise (0-255), pad to the patch, slide, crop
    back to the input size.  `image` is [x, y, z] (the reference's transposed sitk array)."""
    img = normalize_0_255(image)
    pre = img.shape
    img = pad_to_patch(img, patch)
    label = inference_volume(model, img, patch, stride_inplane, stride_layer, patches_per_launch)
    return label[:pre[0], :pre[1], :pre[2]]
