#!/usr/bin/env python3
"""Golden fixtures for the engine's reduced-precision modes (bf16 / fp16 conv operands).

The reference computes in fp32 only; BASELINE configs[1]/[2] ("bf16") and configs[4] ("fp16")
name arithmetic it does not have.  Their parity target is the reference's algorithm with every
convolution operand rounded exactly where the engine's 16-bit modes round it — the oracle's
`operand_rounding` mode (oracle/cyclegan_oracle.py RoundedConv; the rounding placement itself is
pinned per kernel by tests/test_kernels_gpu.py, every kernel = fp64 convolution of the rounded
operands to ~1e-6).  The oracle's exact mode is pinned to the reference-run fixtures
(tests/test_oracle_golden.py); this script only adds the rounding.

For each case (the reference fixture's seed, shapes, weights and inputs) and each mode it runs
  emu64 — the rounded-operand step in fp64 (the parity target), and
  emu32 — the same in fp32 (the calibration twin: how far fp32 accumulation order alone moves a
          rounded-operand step, the analogue of the reference's own fp32-vs-fp64 gap),
sampling losses, generated volumes, gradients, post-Adam parameters and running statistics at
the same indices in both, into tests/golden/prec_<case>.npz.  Data only.

Usage:  python tools/gen_precision_fixtures.py [case ...]       (default: every case below)
        PREC_MODES=bf16x3 python tools/gen_precision_fixtures.py ...   (a subset of the modes)
"""
import os
import random
import sys
import zlib

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from golden_util import CASE_KW, inputs, load  # noqa: E402
from oracle.cyclegan_oracle import CycleGANOracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
# mode → the engine's loss scale (CycleGANModel default).  bf16x3: the fp32-grade split mode's
# products (oracle RoundedConv.x3), the target of its multi-step gates (tests/test_step_gpu.py)
MODES = {"bf16": 1.0, "fp16": 1024.0, "bf16x3": 1.0}
SMALL = ["step_r9_s32_b1", "step_r6_s24_b2_nc2_lsgan", "step_unet_s32_b2_ngf8", "step_r6_s24_b1_noidt",
         "step_r6_s24_b1_pool1", "step_r9_s32_b2_ngf16"]
BIG = ["step_r9_s64_b2", "step_unet_s64_b1_ngf32", "step_r9_s96_b1_nc2", "step_r9_s128_b1",
       "step_unet256_s256_b1_ngf4"]
# emu32p1 / emu32p2: the fp32 twin at inputs perturbed by ~2 fp32 ulps (relative 1e-7 N(0,1) noise):
# further independent realisations of how far fp32 accumulation alone moves a rounded-operand step
# (the tests gate on the largest of the three gaps — one realisation under-states it for
# few-element quantities like the 8 losses)
RUNS = ("emu64", "emu32", "emu32p1", "emu32p2")
PERTURB = 1e-7


def sample(t, key, out, n):
    flat = t.detach().reshape(-1).double()
    name = key.split("/", 2)[2]              # strip "<mode>/<run>/": same indices in every run
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    idx = np.sort(rng.choice(flat.numel(), size=min(n, flat.numel()), replace=False))
    if key.split("/")[1] == "emu64":         # the other runs share the emu64 run's positions
        out[key + "/idx"] = idx.astype(np.int64)
    out[key + "/val"] = flat[torch.from_numpy(idx)].numpy()
    out[key + "/norm"] = np.array(flat.norm().item())


def _steps(case):
    """The reference fixture's step count; the BIG cases one step, except the headline's 64³ b2
    (two: its step 1 is the first HIP-graph replay, which the GPU gates then pin — VERDICT r05)."""
    _, meta = load(case)
    return meta["steps"] if case not in BIG or case == "step_r9_s64_b2" else 1


def run(case, mode, run_name, out):
    _, meta = load(case)
    steps = _steps(case)
    dtype = torch.float64 if run_name == "emu64" else torch.float32
    torch.manual_seed(meta["seed"])
    orc = CycleGANOracle(dtype=dtype, pool_rng=random.Random(meta["seed"]), operand_rounding=mode,
                         loss_scale=MODES[mode], **CASE_KW[case])
    pre = f"{mode}/{run_name}"
    for step in range(steps):
        A, B = inputs(meta, step)
        if run_name.startswith("emu32p"):
            g = torch.Generator().manual_seed(90 + int(run_name[-1]) * 1000 + step)
            A = A * (1 + PERTURB * torch.randn(A.shape, generator=g))
            B = B * (1 + PERTURB * torch.randn(B.shape, generator=g))
        losses = orc.optimize_parameters(A, B)
        out[f"{pre}/step{step}/losses"] = np.array(list(losses.values()), dtype=np.float64)
        if step:
            continue
        for vis in ("fake_B", "rec_A", "fake_A", "rec_B", "idt_A", "idt_B"):
            t = getattr(orc, vis)
            if t is not None:
                sample(t, f"{pre}/step0/{vis}", out, 256)
        for net, grads in orc.grads.items():
            for k, g in grads.items():
                sample(g, f"{pre}/step0/grad/{net}/{k}", out, 64)
        for net, params in orc.params.items():
            for k, p in params.items():
                sample(p, f"{pre}/step0/param/{net}/{k}", out, 64)
        for net, st in orc.state.items():
            for k, b in st.items():
                if "running" in k:
                    sample(b, f"{pre}/step0/buf/{net}/{k}", out, 16)
    out[f"{pre}/steps"] = np.array(steps)


def main():
    torch.set_num_threads(os.cpu_count())
    import tools_conv_chunk  # noqa: F401  (fp64 CPU convolutions in depth slabs: bounded im2col)
    cases = sys.argv[1:] or SMALL + BIG
    for case in cases:
        path = os.path.join(OUT, f"prec_{case}.npz")
        out = dict(np.load(path, allow_pickle=False)) if os.path.exists(path) else {}
        modes = os.environ.get("PREC_MODES", ",".join(MODES)).split(",")
        for mode in modes:
            for r in RUNS:
                if f"{mode}/{r}/steps" in out and int(out[f"{mode}/{r}/steps"]) >= _steps(case):
                    continue
                import time
                t0 = time.time()
                run(case, mode, r, out)
                print(f"{case} {mode} {r}: {time.time() - t0:.1f} s", flush=True)
                np.savez_compressed(path, **out)
        print("wrote", path, os.path.getsize(path), "bytes", flush=True)


if __name__ == "__main__":
    main()
