"""Training patch sampler on the device — replaces the reference's MONAI pipeline (train.py:35-52):

    LoadNiftid → AddChanneld → Orientationd(RAS) → NormalizeIntensityd(image, channel_wise)
    → CropForegroundd(source_key='image') → RandCropByPosNegLabeld(label_key='label',
      spatial_size=patch, pos=20, neg=0, num_samples=2) → ToTensord
    DataLoader(batch_size, shuffle=True, collate_fn=list_data_collate)

MONAI is a third-party dependency the reference does not pin (README.md:9; absent here), so its
published algorithm is restated:
  * the deterministic part (normalisation, foreground crop) is done once per volume on the host,
    as MONAI's PersistentDataset caches it (train.py:49);
  * per step, RandCropByPosNegLabeld draws num_samples centres: with neg = 0 the positive ratio
    is 1, yet MONAI still draws `rand_state.rand()` before `rand_state.randint(len(fg))` for every
    sample; the centre is the unravelled foreground index clamped to the valid range
    [⌊size/2⌋, shape + 1 − size/2) per axis; the crop starts at centre − ⌊size/2⌋
    (monai.transforms.utils.generate_pos_neg_label_crop_centers / SpatialCrop);
  * the crops of a batch are cut out of the device-resident volumes by ONE mragan_crop_patches
    launch per volume and land in the batch tensors the step reads ([B·num_samples, 1, px, py, pz],
    list_data_collate's order: volume-major, sample-minor).

Only .npy volumes [x, y, z] (or SimpleITK / nibabel when installed) are read; Orientationd is the
identity for them (no affine).
"""
from __future__ import annotations

import glob
import os
from typing import List, Sequence

import numpy as np
import torch

from . import ops


def normalize_intensity(img: np.ndarray) -> np.ndarray:
    """NormalizeIntensityd(channel_wise=True, nonzero=False) on one channel: (x − mean) / std
    (population std; std 0 → 1), float32."""
    x = np.asarray(img, dtype=np.float32)
    m, s = float(np.mean(x)), float(np.std(x))
    if s == 0.0:
        s = 1.0
    return ((x - m) / s).astype(np.float32)


def foreground_box(img: np.ndarray):
    """CropForegroundd(source_key='image') with MONAI's default select_fn (x > 0), margin 0:
    the bounding box [start, end) of the positive voxels (the whole volume if there are none)."""
    nz = np.nonzero(img > 0)
    if len(nz[0]) == 0:
        return (0, 0, 0), tuple(img.shape)
    return tuple(int(a.min()) for a in nz), tuple(int(a.max()) + 1 for a in nz)


def crop_centers(shape: Sequence[int], patch: Sequence[int], fg_indices: np.ndarray, num_samples: int,
                 rand_state: np.random.RandomState, pos_ratio: float = 1.0):
    """RandCropByPosNegLabeld's centres (generate_pos_neg_label_crop_centers, neg = 0: no
    background indices), clamped to the valid range; returns a list of (cx, cy, cz)."""
    shape = np.asarray(shape)
    patch = np.asarray(patch)
    if (shape - patch < 0).any():
        raise ValueError("The size of the proposed random crop ROI is larger than the image size.")
    if len(fg_indices) == 0:
        raise ValueError("No sampling location available.")
    valid_start = np.floor_divide(patch, 2)
    valid_end = np.subtract(shape + np.array(1), patch / np.array(2)).astype(np.uint16)
    for i in range(len(valid_start)):
        if valid_start[i] == valid_end[i]:
            valid_end[i] += 1
    out = []
    for _ in range(num_samples):
        rand_state.rand()                       # the pos/neg draw (pos_ratio = 1 → always positive)
        idx = fg_indices[rand_state.randint(len(fg_indices))]
        c = list(np.unravel_index(idx, tuple(shape)))
        for i in range(3):
            if c[i] < valid_start[i]:
                c[i] = valid_start[i]
            if c[i] >= valid_end[i]:
                c[i] = valid_end[i] - 1
        out.append(tuple(int(v) for v in c))
    return out


def load_volume(path: str) -> np.ndarray:
    if path.endswith(".npy"):
        return np.load(path, allow_pickle=False).astype(np.float32)
    try:
        import SimpleITK as sitk
        return np.transpose(sitk.GetArrayFromImage(sitk.ReadImage(path)), (2, 1, 0)).astype(np.float32)
    except ImportError:
        import nibabel as nib
        return np.asarray(nib.load(path).get_fdata(), dtype=np.float32)


class DeviceVolume:
    """One (image, label) pair after the deterministic transforms, resident on the device, with
    its label-foreground index list (map_binary_to_indices: label != 0, flattened C order)."""

    def __init__(self, image: np.ndarray, label: np.ndarray, device):
        img = normalize_intensity(image)
        (x0, y0, z0), (x1, y1, z1) = foreground_box(img)
        img = img[x0:x1, y0:y1, z0:z1]
        lab = np.asarray(label, dtype=np.float32)[x0:x1, y0:y1, z0:z1]
        self.shape = img.shape
        self.fg = np.flatnonzero(lab.ravel() != 0)
        self.image = torch.from_numpy(np.ascontiguousarray(img)).to(device)
        self.label = torch.from_numpy(np.ascontiguousarray(lab)).to(device)


class GpuPatchSampler:
    """DataLoader-equivalent iterator: shuffled volumes, batch_size volumes per batch,
    num_samples crops each; yields dict(image=[B·ns,1,px,py,pz], label=...) device tensors."""

    def __init__(self, volumes: List[DeviceVolume], patch: Sequence[int], batch_size: int = 1, num_samples: int = 2,
                 shuffle: bool = True, seed: int = 0):
        self.volumes = volumes
        self.patch = tuple(int(p) for p in patch)
        self.batch_size = batch_size
        self.num_samples = num_samples
        self.shuffle = shuffle
        self.rand_state = np.random.RandomState(seed)       # MONAI's Randomizable state
        self.order_rng = np.random.RandomState(seed + 1)    # the DataLoader's shuffle

    @classmethod
    def from_folder(cls, data_path: str, patch, device, **kw):
        """<data_path>/images/*.{nii,npy} with <data_path>/labels/* (train.py:31-33)."""
        imgs = sorted(glob.glob(os.path.join(data_path, "images", "*")))
        labs = sorted(glob.glob(os.path.join(data_path, "labels", "*")))
        vols = [DeviceVolume(load_volume(i), load_volume(l), device) for i, l in zip(imgs, labs)]
        return cls(vols, patch, **kw)

    def __len__(self):
        return (len(self.volumes) + self.batch_size - 1) // self.batch_size

    def sample(self, idx: Sequence[int]):
        """The crops of one batch (volumes idx, in order) as device tensors."""
        ns, p = self.num_samples, self.patch
        n = len(idx) * ns
        dev = self.volumes[idx[0]].image.device
        image = torch.empty((n, 1) + p, device=dev, dtype=torch.float32)
        label = torch.empty((n, 1) + p, device=dev, dtype=torch.float32)
        for j, v in enumerate(idx):
            vol = self.volumes[v]
            centers = crop_centers(vol.shape, p, vol.fg, ns, self.rand_state)
            starts = torch.tensor([[c - q // 2 for c, q in zip(ctr, p)] for ctr in centers], dtype=torch.int32).to(dev)
            ops.crop_patches(vol.image, starts, p, out=image[j * ns:(j + 1) * ns].view((ns,) + p))
            ops.crop_patches(vol.label, starts, p, out=label[j * ns:(j + 1) * ns].view((ns,) + p))
        return {"image": image, "label": label}

    def __iter__(self):
        order = self.order_rng.permutation(len(self.volumes)) if self.shuffle else np.arange(len(self.volumes))
        for b in range(0, len(order), self.batch_size):           # no drop_last (train.py:52)
            yield self.sample([int(i) for i in order[b:b + self.batch_size]])
