#!/usr/bin/env python3
"""Diagnostic (GPU box): per-parameter gradient error of the HIP step and of the fp32 CPU
oracle, both against the fp64 oracle, for one golden case.  Usage:
    python tools/diag_grads.py step_r9_s32_b1"""
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


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-300))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "step_r9_s32_b1"
    z, meta = load(name)
    A, B = inputs(meta, 0)
    model = build_model(meta, "/tmp/diag_ck")
    model.set_input([A, B])
    model.optimize_parameters()
    torch.cuda.synchronize()
    res = {}
    for dt in (torch.float64, torch.float32):
        torch.manual_seed(meta["seed"])
        orc = CycleGANOracle(dtype=dt, pool_rng=random.Random(meta["seed"]), **CASE_KW[name])
        orc.optimize_parameters(A, B)
        res[dt] = orc
    o64, o32 = res[torch.float64], res[torch.float32]
    rows = []
    for net in ("G_A", "G_B", "D_A", "D_B"):
        for k, p in getattr(model, "net" + net).named_parameters():
            if is_pre_in_bias(net, k):
                continue
            g64 = o64.grads[net][k]
            rows.append((rel(p.grad.cpu(), g64), rel(o32.grads[net][k], g64), net, k))
    print(f"{'ours':>10} {'oracle32':>10}  param")
    for r in rows:
        print(f"{r[0]:10.2e} {r[1]:10.2e}  {r[2]}:{r[3]}")
    for vis in ("fake_B", "rec_A", "fake_A", "rec_B", "idt_A", "idt_B"):
        print(vis, f"{rel(getattr(model, vis).cpu(), getattr(o64, vis)):.2e}", f"{rel(getattr(o32, vis), getattr(o64, vis)):.2e}")


if __name__ == "__main__":
    main()
