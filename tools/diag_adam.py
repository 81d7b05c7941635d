#!/usr/bin/env python3
"""Diagnostic (GPU box): post-step parameters of the HIP step vs the fp64 oracle."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mra-gan_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from golden_util import CASE_KW, inputs, is_pre_in_bias, load  # noqa: E402
from oracle.cyclegan_oracle import CycleGANOracle  # noqa: E402
from test_step_gpu import build_model  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "step_r9_s32_b1"
    z, meta = load(name)
    A, B = inputs(meta, 0)
    model = build_model(meta, "/tmp/diag_ck")
    p0 = {n: {k: p.detach().cpu().double().clone() for k, p in getattr(model, "net" + n).named_parameters()}
          for n in ("G_A", "G_B", "D_A", "D_B")}
    model.set_input([A, B])
    model.optimize_parameters()
    torch.cuda.synchronize()
    torch.manual_seed(meta["seed"])
    orc = CycleGANOracle(dtype=torch.float64, pool_rng=random.Random(meta["seed"]), **CASE_KW[name])
    orc.optimize_parameters(A, B)
    for n in ("G_A", "G_B", "D_A", "D_B"):
        for k, p in getattr(model, "net" + n).named_parameters():
            if is_pre_in_bias(n, k):
                continue
            ours = p.detach().cpu().double()
            ref = orc.params[n][k]
            d = (ours - ref).abs()
            g = p.grad.detach().cpu().double()
            gr = orc.grads[n][k]
            flips = int(((g > 0) != (gr > 0)).sum())
            step_ours = (ours - p0[n][k]).abs()
            step_ref = (ref - p0[n][k]).abs()
            print(f"{n}:{k:28s} n={d.numel():8d} frac|d|>1e-6={float((d > 1e-6).double().mean()):.4f} "
                  f"max|d|={float(d.max()):.2e} sign-flips={flips} "
                  f"mean|step| ours={float(step_ours.mean()):.3e} ref={float(step_ref.mean()):.3e} "
                  f"|g|med={float(gr.abs().median()):.2e}")


if __name__ == "__main__":
    main()
