#!/usr/bin/env python3
"""Measure each contraction precision's error envelope against the reference's fp64 fixtures
(tests/golden, made by tools/gen_fixtures.py): step-1 losses, generated volumes, running
statistics and whole-network gradients (rel-L2 over the sampled elements, every parameter
normalised), plus the later-step losses.  The numbers calibrate tests/test_step_gpu.py's gates.

    python tools/precision_envelope.py [case ...] [--precisions f32,bf16x3,bf16,fp16]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mra-gan_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_util import available_cases, inputs, is_pre_in_bias, load, rel_err, sampled  # noqa: E402
from test_step_gpu import build_model  # noqa: E402


def measure(name, precision, tmp):
    z, meta = load(name)
    model = build_model(meta, tmp, precision)
    out = {}
    hist = []
    for step in range(meta["steps"]):
        A, B = inputs(meta, step)
        model.set_input([A, B])
        model.optimize_parameters()
        hist.append(np.array(list(model.get_current_losses().values())))
        if step == 0:
            out["losses"] = rel_err(hist[0], z["fp64/step0/losses"])
            out["vol"] = max(rel_err(*sampled(z, f"fp64/step0/{v}", getattr(model, v).detach().cpu()))
                             for v in ("fake_B", "rec_A", "fake_A", "rec_B") if f"fp64/step0/{v}/idx" in z.files)
            ours, ref = [], []
            for net in ("G_A", "G_B", "D_A", "D_B"):
                for k, p in getattr(model, "net" + net).named_parameters():
                    if is_pre_in_bias(net, k):
                        continue
                    g, w = sampled(z, f"fp64/step0/grad/{net}/{k}", p.grad.detach().cpu() / model.loss_scale)
                    s = 1.0 / max(float(np.linalg.norm(w)), 1e-30)
                    ours.append(g * s)
                    ref.append(w * s)
            out["grad_whole"] = rel_err(np.concatenate(ours), np.concatenate(ref))
            rs = []
            for net in ("G_A", "G_B", "D_A", "D_B"):
                for k, b in getattr(model, "net" + net).state_dict().items():
                    if "running" in k:
                        g, w = sampled(z, f"fp64/step0/buf/{net}/{k}", b.detach().cpu())
                        rs.append(rel_err(g, w))
            out["running"] = max(rs)
    out["later"] = [rel_err(hist[s], z[f"fp64/step{s}/losses"]) for s in range(1, meta["steps"])]
    out["later_ref32"] = [rel_err(z[f"fp32/step{s}/losses"], z[f"fp64/step{s}/losses"]) for s in range(1, meta["steps"])]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*")
    ap.add_argument("--precisions", default="f32,bf16x3,bf16,fp16")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cases = a.cases or available_cases()
    res = {}
    for c in cases:
        for p in a.precisions.split(","):
            r = measure(c, p, f"/tmp/penv_{c}_{p}")
            res[f"{c}/{p}"] = r
            print(json.dumps({f"{c}/{p}": r}), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
