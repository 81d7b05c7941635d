#!/usr/bin/env python3
"""Phase breakdown of the 1-channel bf16x3 convolution from its in-kernel s_memtime stamps
(MRAGAN_STAMPS=1; diagnostic build path only).  Prints median cycles per phase per block:
raw-halo load, X8 expansion, MFMA loop, epilogue; and the block start spread."""
import os
import sys

os.environ["MRAGAN_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mra-gan_amd"))
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mragan_hip import ops  # noqa: E402
from mragan_hip._lib import lib  # noqa: E402

ops.set_conv_precision("bf16x3")
S, N, ngf = 64, int(sys.argv[1]) if len(sys.argv) > 1 else 2, 32
x = torch.randn(N, S + 6, S + 6, S + 6, 1, device="cuda")
w = torch.randn(343 * ngf, device="cuda") * 0.01
for _ in range(3):
    ops.conv3d(x, w, ngf, 7, 1, 0, (S, S, S))
torch.cuda.synchronize()
nblk = N * (S // 2) * (S // 8) * (S // 32)
nblk = min(nblk, 8192)
buf = (C.c_ulonglong * (nblk * 5))()
assert lib().mragan_debug_stamps(buf, nblk * 5) == 0
st = np.array(buf, dtype=np.float64).reshape(nblk, 5)
d = np.diff(st, axis=1)
print(f"blocks {nblk}; median cycles per phase: raw {np.median(d[:,0]):.0f}  x8 {np.median(d[:,1]):.0f}  "
      f"mfma {np.median(d[:,2]):.0f}  epilogue {np.median(d[:,3]):.0f}  total {np.median(st[:,4]-st[:,0]):.0f}")
print(f"p90: raw {np.percentile(d[:,0],90):.0f} x8 {np.percentile(d[:,1],90):.0f} mfma {np.percentile(d[:,2],90):.0f} "
      f"epi {np.percentile(d[:,3],90):.0f}; kernel span {st[:,4].max()-st[:,0].min():.0f}")
