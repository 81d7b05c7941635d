"""Helpers to read the golden fixtures made by tools/gen_fixtures.py (reference run)."""
import ast
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# argv flags of each case → oracle / engine constructor kwargs
CASE_KW = {
    "step_r9_s32_b1": dict(input_nc=1, output_nc=1, ngf=32, ndf=32, n_blocks=9, use_lsgan=False),
    "step_r6_s24_b2_nc2_lsgan": dict(input_nc=2, output_nc=2, ngf=8, ndf=8, n_blocks=6, use_lsgan=True),
    "step_r9_s32_b2_ngf16": dict(input_nc=1, output_nc=1, ngf=16, ndf=16, n_blocks=9, use_lsgan=False),
    "step_unet_s32_b2_ngf8": dict(input_nc=1, output_nc=1, ngf=8, ndf=8, netG="unet_custom", use_lsgan=False),
    "step_r6_s24_b1_noidt": dict(input_nc=1, output_nc=1, ngf=8, ndf=8, n_blocks=6, use_lsgan=False, lambda_identity=0.0),
    # BASELINE-size workloads (per-GPU units of configs[1]..[4]); their fixtures carry fp64 runs at
    # perturbed inputs (fp64p4e-6 / fp64p4e-5), so the tests need no fp64 oracle run of their own
    "step_r9_s64_b2": dict(input_nc=1, output_nc=1, ngf=32, ndf=32, n_blocks=9, use_lsgan=False),
    "step_unet_s64_b1_ngf32": dict(input_nc=1, output_nc=1, ngf=32, ndf=32, netG="unet_custom", use_lsgan=False),
    "step_r9_s96_b1_nc2": dict(input_nc=2, output_nc=2, ngf=32, ndf=32, n_blocks=9, use_lsgan=False),
    "step_r9_s128_b1": dict(input_nc=1, output_nc=1, ngf=32, ndf=32, n_blocks=9, use_lsgan=False),
    # pool of one image: the step takes the ImagePool swap path from step 2 on
    "step_r6_s24_b1_pool1": dict(input_nc=1, output_nc=1, ngf=4, ndf=4, n_blocks=6, use_lsgan=False, pool_size=1),
    # --netG unet_256 (8 downsamplings) at the smallest size it trains at
    "step_unet256_s256_b1_ngf4": dict(input_nc=1, output_nc=1, ngf=4, ndf=4, netG="unet_256", use_lsgan=False),
}


def available_cases():
    """Step cases whose fixture file is present (the BASELINE-size ones are generated separately)."""
    return [c for c in CASE_KW if os.path.exists(os.path.join(GOLDEN, c + ".npz"))]


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = ast.literal_eval(str(z["meta"]))
    return z, meta


def sampled(z, key, t: torch.Tensor):
    flat = t.detach().reshape(-1).double().cpu()
    idx = torch.from_numpy(z[key + "/idx"])
    return flat[idx].numpy(), z[key + "/val"]


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def inputs(meta, step):
    g = torch.Generator().manual_seed(1000 + meta["seed"] + step)
    shape = (meta["B"], meta["nc"], meta["S"], meta["S"], meta["S"])
    return torch.randn(shape, generator=g), torch.randn(shape, generator=g)


# Pre-InstanceNorm conv biases have an identically-zero true gradient (IN without affine
# cancels any per-channel constant).  Their fp32 reference gradient is round-off noise.
def is_pre_in_bias(net, key, n_layers_D=3):
    if not key.endswith(".bias"):
        return False
    if net.startswith("G"):
        if key.startswith("model.model"):    # UnetGenerator: only the outermost upconv has a bias
            return False
        return "conv_block" in key or not _is_g_head(key)
    # D: model.0 (no IN) and the final conv have real gradients
    idx = int(key.split(".")[1])
    return idx not in (0, 3 * n_layers_D + 2)


def _is_g_head(key):
    # the head conv is the last conv of the generator; its index depends on n_blocks
    return key in ("model.26.bias", "model.23.bias")


def over_envelope(err, env) -> bool:
    """A per-tensor gate's verdict: True unless err is a finite number within env.  A NaN error
    compares False against any bound, so `err > env` would let a NaN tensor through; this does not."""
    return not (np.isfinite(err) and err <= env)


def assert_finite(label, *arrays):
    """Every value finite (a NaN / Inf anywhere fails the gate, whatever its error norm says)."""
    for a in arrays:
        a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
        bad = int((~np.isfinite(a)).sum())
        assert bad == 0, f"{label}: {bad} non-finite values"
