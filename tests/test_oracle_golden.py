"""Pin the CPU oracle (oracle/cyclegan_oracle.py) against the reference's own outputs.

The fixtures in tests/golden/ were produced by running the reference's
CycleGANModel.optimize_parameters() (tools/gen_fixtures.py).  The oracle must
(1) reproduce the reference's initial weights bit-exactly from the same torch seed,
(2) match its fp64 step to ~1e-9 (same math, same precision), and
(3) match its fp32 step within the fp32 envelope calibrated in SURVEY §8(c).
"""
import os
import random

import numpy as np
import pytest
import torch

from golden_util import CASE_KW, available_cases, inputs, is_pre_in_bias, load, rel_err, sampled
from oracle.cyclegan_oracle import CycleGANOracle

# the CPU oracle replays the small fixtures (the BASELINE-size ones compare the HIP engine with
# the reference directly, tests/test_step_gpu.py; an fp64 CPU step at 128³ takes minutes)
CASES = [c for c in available_cases() if load(c)[1]["S"] <= 32]
# the two 9-block 32³ fp64 replays take 3–4 minutes each on the container's 8 CPUs; the 6-block
# 24³ and UNet 32³ replays pin the same oracle code paths (every layer kind, ImagePool, both
# losses) in seconds, so the full-size ones run on request (MRAGAN_SLOW_ORACLE=1)
SLOW = {"step_r9_s32_b1", "step_r9_s32_b2_ngf16"}
_RUN_SLOW = os.environ.get("MRAGAN_SLOW_ORACLE") == "1"


def _gate(name):
    if name in SLOW and not _RUN_SLOW:
        pytest.skip(f"{name}: fp64 CPU replay of a 9-block 32³ step (minutes); set MRAGAN_SLOW_ORACLE=1")


def _build(name, dtype):
    z, meta = load(name)
    torch.manual_seed(meta["seed"])
    orc = CycleGANOracle(dtype=dtype, pool_rng=random.Random(meta["seed"]), **CASE_KW[name])
    return z, meta, orc


@pytest.mark.parametrize("name", CASES)
def test_init_bit_exact(name):
    z, meta, orc = _build(name, torch.float32)
    n_checked = 0
    for net in ("G_A", "G_B", "D_A", "D_B"):
        for k, v in orc.state[net].items():
            key = f"init/{net}/{k}"
            if key + "/idx" not in z.files:
                continue
            got, want = sampled(z, key, v)
            np.testing.assert_array_equal(got, want)
            assert float(v.double().sum()) == pytest.approx(float(z[key + "/sum"]), rel=1e-12, abs=1e-12)
            n_checked += 1
    assert n_checked > 20


@pytest.mark.parametrize("name", CASES)
def test_step_fp64_matches_reference(name):
    _gate(name)
    z, meta, orc = _build(name, torch.float64)
    for step in range(meta["steps"]):
        A, B = inputs(meta, step)
        losses = orc.optimize_parameters(A, B)
        want = z[f"fp64/step{step}/losses"]
        got = np.array(list(losses.values()))
        assert rel_err(got, want) < 1e-9, (step, got, want)
        if step == 0:
            for vis in ("fake_B", "rec_A", "fake_A", "rec_B", "idt_A", "idt_B"):
                if f"fp64/step0/{vis}/idx" not in z.files:
                    assert getattr(orc, vis) is None      # lambda_identity = 0: no identity pass
                    continue
                g, w = sampled(z, f"fp64/step0/{vis}", getattr(orc, vis))
                assert rel_err(g, w) < 1e-9, vis
            for net in ("G_A", "G_B", "D_A", "D_B"):
                for k, gr in orc.grads[net].items():
                    key = f"fp64/step0/grad/{net}/{k}"
                    gn = float(gr.norm())
                    wn = float(z[key + "/norm"])
                    if is_pre_in_bias(net, k):
                        assert wn < 1e-9 and gn < 1e-9, (net, k, gn, wn)
                        continue
                    assert abs(gn - wn) <= 1e-7 * wn + 1e-12, (net, k, gn, wn)
                    g, w = sampled(z, key, gr)
                    assert np.allclose(g, w, rtol=1e-6, atol=1e-9 * max(wn, 1e-30)), (net, k)
                for k, p in orc.params[net].items():
                    g, w = sampled(z, f"fp64/step0/param/{net}/{k}", p)
                    if is_pre_in_bias(net, k):
                        continue   # Adam amplifies the zero-gradient noise into ±lr steps
                    assert np.allclose(g, w, rtol=1e-7, atol=1e-10), (net, k)
                for k, b in orc.state[net].items():
                    if "running" in k:
                        g, w = sampled(z, f"fp64/step0/buf/{net}/{k}", b)
                        assert np.allclose(g, w, rtol=1e-9, atol=1e-12), (net, k)


@pytest.mark.parametrize("name", CASES[:2] + ["step_unet_s32_b2_ngf8"])
def test_step_fp32_within_envelope(name):
    """fp32 oracle vs fp32 reference: losses/outputs to 1e-4 rel; whole-network gradients
    (all sampled elements, each parameter normalised) within 3× the reference's own
    fp32-vs-fp64 error or 1e-3 — an fp32 run is one sample of ReLU-kink-flip noise
    (tests/test_step_gpu.py::conditioning).  The fp64 path is pinned at 1e-9 above."""
    _gate(name)
    z, meta, orc = _build(name, torch.float32)
    A, B = inputs(meta, 0)
    losses = orc.optimize_parameters(A, B)
    assert rel_err(list(losses.values()), z["fp32/step0/losses"]) < 1e-4
    for vis in ("fake_B", "rec_A", "idt_A"):
        g, w = sampled(z, f"fp32/step0/{vis}", getattr(orc, vis))
        assert rel_err(g, w) < 1e-4, vis
    ours, r32, r64 = [], [], []
    for net in ("G_A", "G_B", "D_A", "D_B"):
        for k, gr in orc.grads[net].items():
            if is_pre_in_bias(net, k):
                continue
            key64 = f"fp64/step0/grad/{net}/{k}"
            g, w64 = sampled(z, key64, gr)
            w32 = z[f"fp32/step0/grad/{net}/{k}/val"]
            s = 1.0 / max(float(np.linalg.norm(w64)), 1e-30)
            ours.append(g * s)
            r32.append(w32 * s)
            r64.append(w64 * s)
    whole = rel_err(np.concatenate(ours), np.concatenate(r64))
    whole_ref = rel_err(np.concatenate(r32), np.concatenate(r64))
    assert whole <= max(1e-3, 3 * whole_ref), (whole, whole_ref)
