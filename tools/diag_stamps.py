#!/usr/bin/env python3
"""Phase breakdown of the 1-channel bf16x3 convolution (conv_thin1_ring.hip) from its in-kernel
s_memtime stamps (MRAGAN_STAMPS=1; diagnostic path only): median cycles per work item of the
7-plane prologue and of the depth steps, and the kernel span."""
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

S, N, ngf = 64, int(sys.argv[1]) if len(sys.argv) > 1 else 2, 32
which = sys.argv[2] if len(sys.argv) > 2 else "fwd"
ops.set_conv_precision(sys.argv[3] if len(sys.argv) > 3 else "bf16x3")
x = torch.randn(N, S + 6, S + 6, S + 6, 1, device="cuda")
w = torch.randn(343 * ngf, device="cuda") * 0.01
dh = torch.randn(N, S, S, S, ngf, device="cuda")
gw = torch.empty(343 * ngf, device="cuda")
for _ in range(3):
    if which == "fwd":
        ops.conv3d(x, w, ngf, 7, 1, 0, (S, S, S))
    else:            # the stem weight gradient
        ops.conv3d_wgrad(dh, x, 7, 1, 0, gw, False)
torch.cuda.synchronize()
nitems = 4096
buf = (C.c_ulonglong * (nitems * 3))()
assert lib().mragan_debug_stamps(buf, nitems * 3) == 0
st = np.array(buf, dtype=np.float64).reshape(nitems, 3)
st = st[st[:, 2] > st[:, 0]]
d = np.diff(st, axis=1)
print(f"items {len(st)}; median cycles: prologue {np.median(d[:,0]):.0f}  steps {np.median(d[:,1]):.0f}  "
      f"total {np.median(st[:,2]-st[:,0]):.0f}; p90 steps {np.percentile(d[:,1],90):.0f}; "
      f"span {st[:,2].max()-st[:,0].min():.0f}")
