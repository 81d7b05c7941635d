#!/usr/bin/env python3
"""Phase breakdown of the K-split brick (conv_brick_ks.hip) from its in-kernel s_memtime stamps
(MRAGAN_STAMPS=1, diagnostic path only): per wave, median cycles of table setup, halo prologue,
main loop, K reduction and epilogue, plus the launch span, for the res-block forward and data
gradient at the bench shapes (N = 4 and 2, 64^3 patch: 16^3 x 128 channels)."""
import ctypes as C
import os
import sys

os.environ["MRAGAN_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mra-gan_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mragan_hip import ops  # noqa: E402
from mragan_hip._lib import lib  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
ops.set_conv_precision(prec)
dt = ops.op16_dtype()
c4, s4 = 128, 16
w = torch.randn(27 * c4 * c4, device="cuda") * 0.01
ws_f = torch.empty_like(w)
ws_b = torch.empty_like(w)
base = 4 if prec == "fp16" else 2
ops.pack_weight(w, c4, c4, 27, base, ws_f)
ops.pack_weight(w, c4, c4, 27, base + 1, ws_b)
for N in (4, 2):
    x = torch.randn(N, s4 + 2, s4 + 2, s4 + 2, c4, device="cuda").to(dt)
    dy = torch.randn(N, s4, s4, s4, c4, device="cuda").to(dt)
    part = ops.in_partials_buffer(N, (s4, s4, s4), c4, "cuda")
    cases = {"fwd": lambda: ops.conv3d_op16(x, w, c4, 3, 1, 0, (s4, s4, s4), ws_f, part),
             "dgrad": lambda: ops.conv3d_op16(dy, w, c4, 3, 1, 0, (s4 + 2,) * 3, ws_b, transposed=True)}
    for name, fn in cases.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        nb = 1024
        buf = (C.c_ulonglong * (nb * 32))()
        assert lib().mragan_debug_stamps(buf, -nb * 32) == 0
        st = np.array(buf, dtype=np.float64).reshape(nb, 4, 8)[:, :, :7]
        st = st[st[:, 0, 6] > st[:, 0, 0]]
        st = st[np.abs(st[:, 0, 0] - st[0, 0, 0]) < 20000]     # this launch's blocks only (stale slots of earlier, larger grids dropped)
        d = np.diff(st, axis=2).reshape(-1, 6)
        names = ["issue", "tables", "prologue", "main", "reduce", "epilogue"]
        med = "  ".join(f"{n} {np.median(d[:, i]):7.0f}" for i, n in enumerate(names))
        tot = st[:, :, 6] - st[:, :, 0]
        starts = st[:, 0, 0]
        print(f"N{N} {name:5s} blocks {len(st)}: median cycles {med}  | wave total {np.median(tot):.0f} "
              f"(p90 {np.percentile(tot, 90):.0f}); span {st[:, :, 6].max() - starts.min():.0f}, "
              f"start spread {starts.max() - starts.min():.0f}; main p10/p90 {np.percentile(d[:, 3], 10):.0f}/"
              f"{np.percentile(d[:, 3], 90):.0f}")
