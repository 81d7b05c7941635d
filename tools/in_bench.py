#!/usr/bin/env python3
"""Per-shape timing of the InstanceNorm forward / backward entries (tools/ A/B helper: run it under
different MRAGAN_IN_SMALL settings, one process each — the switch is read once per process).

    python3 tools/in_bench.py [--reps 200]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mra-gan_amd"))
import torch  # noqa: E402

from mragan_hip import ops  # noqa: E402

# (N, S, C, ypad / dypad): the UNet 64³ levels, the PatchGAN tail, a ResnetBlock norm
SHAPES = [(1, 2, 256, 0), (2, 4, 256, 0), (1, 4, 256, 0), (2, 8, 128, 0), (1, 8, 128, 0), (2, 7, 256, 0),
          (4, 7, 256, 0), (2, 16, 64, 0), (1, 16, 64, 0), (2, 16, 128, 1), (4, 16, 128, 1)]


def timed(fn, reps):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    tag = os.environ.get("MRAGAN_IN_SMALL", "default")
    for N, S, C, pad in SHAPES:
        x = torch.randn(N, S, S, S, C, device="cuda")
        tf = timed(lambda: ops.instnorm_fwd(x, act="relu", ypad=pad), args.reps)
        _, mean, rstd = ops.instnorm_fwd(x, act="relu")
        dy = torch.randn(N, S + 2 * pad, S + 2 * pad, S + 2 * pad, C, device="cuda")
        tb = timed(lambda: ops.instnorm_bwd(x, mean, rstd, dy, pad, None, act="relu"), args.reps)
        print(f"IN_SMALL={tag} N{N} S{S} C{C} pad{pad}: fwd {tf:7.2f} us  bwd {tb:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
