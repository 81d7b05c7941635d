"""Whole-step parity on the GPU: the drop-in CycleGANModel (HIP engine) against the golden
fixtures produced by the reference itself (tools/gen_fixtures.py) and against the oracle.

fp32-grade modes (f32, bf16x3) — gates calibrated on the reference's own fp32-vs-fp64 error
(SURVEY §8c):
  * initial weights: bit-exact (same torch seed → same RNG consumption);
  * losses and generated volumes at step 1: rel ≤ 1e-4 (f32) / 1e-3 (bf16x3) vs the fp64 reference;
  * step-1 gradients: ‖g − g64‖ ≤ max(1e-3‖g64‖, 2‖g_ref32 − g64‖) on the sampled elements;
    pre-InstanceNorm conv biases: exactly 0 (their true gradient is identically zero);
  * InstanceNorm running statistics after step 1: rel ≤ 1e-4 / 1e-3;
  * later steps: losses within max(1e-3, k × the reference's own fp32-vs-fp64 divergence at that
    step) — fp32 noise amplified by Adam, as for the reference (k = 4 exact f32, 10 bf16x3).

bf16x3 against its own emulation: the oracle's operand_rounding="bf16x3" (RoundedConv.x3: the
split products exactly where the engine's MFMA kernels split them, exact fp32 products where its
VALU / fp32 kernels run) in fp64 ("emu64") and fp32 ("emu32", "emu32p1/p2"), tests/golden/prec_*.npz.
The GPU's distance to emu64 is then fp32 accumulation order only: step-0 losses, volumes and
running statistics within max(1e-4, 4 × the fp32 realisations' gap), gradients as the reduced
modes below, later-step losses within max(1e-3, 10 × the gap at that step) — every gate value from
the oracle, none from a GPU run.

Reduced modes (bf16, fp16: every conv operand rounded) — against the oracle's rounded-operand
step (tests/golden/prec_<case>.npz, tools/gen_precision_fixtures.py): "emu64" is the step with
the engine's operand rounding evaluated in fp64, "emu32" the same in fp32 (and "emu32p1/p2" at
inputs moved by ~2 fp32 ulps: further realisations).  The same calibrated rule as above with the
fp32 realisations in the reference-fp32 role: every quantity within max(1e-3, 2 × the largest
fp32-vs-emu64 gap) of emu64 (gradients per tensor with the same outlier budget, and for the whole
network with none).  Measured (r03c, MI355X): the GPU's distance to emu64 tracks emu32's within
0.7-1.3× for every volume, loss vector and whole-network gradient at 24³-256³ — bf16 operand
rounding is chaotic at the 1e-2 level (rec_A 4e-2, whole-network gradient 0.2-0.3), for ANY
accumulation order, so a fixed 1e-3 gate on volumes is below the arithmetic's reproducibility.
"""
import random
import sys

import numpy as np
import pytest
import torch

from golden_util import (CASE_KW, assert_finite, available_cases, inputs, is_pre_in_bias, load, over_envelope, rel_err,
                         sampled)

pytestmark = pytest.mark.gpu

CASES = available_cases()


def build_model(meta, ckdir, precision="f32"):
    from models import create_model
    from options.train_options import TrainOptions
    argv = sys.argv
    try:
        sys.argv = ["train.py", "--checkpoints_dir", str(ckdir), "--conv_precision", precision] + meta["argv"].split()
        opt = TrainOptions().gather_options()
    finally:
        sys.argv = argv
    opt.isTrain = True
    opt.gpu_ids = 0
    torch.manual_seed(meta["seed"])
    random.seed(meta["seed"])
    model = create_model(opt)
    model.setup(opt)
    return model


# every case in every contraction precision of the MFMA convolutions (include/mragan_hip.h)
PRECISIONS = ("f32", "bf16x3", "bf16", "fp16")
PARAMS = [(c, p) for p in PRECISIONS for c in CASES]
# bf16 / fp16 round every MFMA operand once (one MFMA per product): gated against the oracle's
# rounded-operand step (below)
REDUCED = ("bf16", "fp16")
# per-tensor gradient outlier budget (all gradient gates): at most this fraction of the parameter
# tensors (and at least 2) may exceed their envelope, none by more than OUTLIER_X×.  Both constants
# are fixed by the protocol, not by a GPU run: the envelope of each tensor is the largest of the
# reference's fp32 error and the fp64 gradient's movement under ≥ 3 input-perturbation
# realisations (the BASELINE-size fixtures store three, tools/gen_fixtures.py; the small cases
# compute three at test time), so a tensor past it is a tail event of an estimated spread.
OUTLIER_FRAC, OUTLIER_X = 0.1, 5.0


def check_outliers(label, bad, n_params):
    worst = max(bad, key=lambda b: b[2] / b[3]) if bad else None
    print(f"{label}: {len(bad)}/{n_params} parameter tensors over their envelope"
          + (f"; worst {worst[0]}.{worst[1]} at {worst[2] / worst[3]:.2f}x" if worst else ""))
    assert len(bad) <= max(2, int(OUTLIER_FRAC * n_params)), bad
    assert all(np.isfinite(r) and r <= OUTLIER_X * env for _, _, r, env in bad), bad


@pytest.fixture(scope="module", params=PARAMS, ids=[f"{c}-{p}" for c, p in PARAMS])
def stepped(request, tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    name, precision = request.param
    z, meta = load(name)
    meta = dict(meta, precision=precision)
    model = build_model(meta, tmp_path_factory.mktemp(name), precision)
    init = {}
    for net in ("G_A", "G_B", "D_A", "D_B"):
        for k, v in getattr(model, "net" + net).state_dict().items():
            init[f"init/{net}/{k}"] = v.detach().cpu().clone()
    history = []
    snap = None
    for step in range(meta["steps"]):
        A, B = inputs(meta, step)
        model.set_input([A, B])
        model.optimize_parameters()
        history.append(np.array(list(model.get_current_losses().values())))
        if step == 0:
            ls = model.loss_scale            # fp16: p.grad carries the static loss scale
            snap = dict(
                vis={v: getattr(model, v).detach().cpu().clone() for v in
                     ("fake_B", "rec_A", "fake_A", "rec_B", "idt_A", "idt_B") if f"fp64/step0/{v}/idx" in z.files},
                grads={n: {k: p.grad.detach().cpu().clone() / ls for k, p in getattr(model, "net" + n).named_parameters()}
                       for n in ("G_A", "G_B", "D_A", "D_B")},
                params={n: {k: p.detach().cpu().clone() for k, p in getattr(model, "net" + n).named_parameters()}
                        for n in ("G_A", "G_B", "D_A", "D_B")},
                bufs={n: {k: b.detach().cpu().clone() for k, b in getattr(model, "net" + n).state_dict().items()
                          if "running" in k} for n in ("G_A", "G_B", "D_A", "D_B")},
            )
    torch.cuda.synchronize()
    from mragan_hip import ops
    ops.set_conv_precision("f32")
    return name, z, meta, init, history, snap


def test_all_finite(stepped):
    """Every loss, generated volume, gradient, updated parameter and running statistic of the
    snapshot is finite in full (the sampled gates below see 64-256 elements per tensor)."""
    name, _, meta, _, history, snap = stepped
    assert_finite(f"{name} losses", np.stack(history))
    for vis, t in snap["vis"].items():
        assert_finite(vis, t)
    for what in ("grads", "params", "bufs"):
        for net, d in snap[what].items():
            for k, t in d.items():
                assert_finite(f"{what} {net}.{k}", t)


def test_init_bit_exact(stepped):
    name, z, meta, init, _, _ = stepped
    n = 0
    for key, v in init.items():
        if key + "/idx" in z.files:
            g, w = sampled(z, key, v)
            np.testing.assert_array_equal(g, w)
            n += 1
    assert n > 20


# forward-value gates: exact-f32 MFMA 1e-4 (measured 1e-6…2e-5); bf16x3 split MFMA (≤ 3·2⁻¹⁸ per
# product) the north star's 1e-3 (measured ≤ 1.5e-4)
LOSS_TOL = {"f32": 1e-4, "bf16x3": 1e-3}
VOL_TOL = {"f32": 1e-4, "bf16x3": 1e-3}
RS_TOL = {"f32": 1e-4, "bf16x3": 1e-3}
# later-step losses: multiple of the reference's own fp32-vs-fp64 divergence at that step, and at
# least LATER_MIN
# least LATER_MIN.  bf16x3's per-product error (≤ 3·2⁻¹⁸) is ~50× fp32's, so more of the first Adam
# step's ±lr signs (elements with a round-off-sized gradient) differ from fp64 and a multi-step
# trajectory departs further: on the 6-step pool-1 case (r03a) 1.8e-4, 7.0e-4, 8.6e-4, 1.05e-3 at
# steps 1-4, against the reference fp32's 5e-8 … 3.3e-5
LATER_STEP_FACTOR = {"f32": 4.0, "bf16x3": 10.0}
LATER_MIN = {"f32": 1e-3, "bf16x3": 1e-3}


# ---- reduced precisions: against the rounded-operand oracle ----------------------------------

def prec_fixture(name):
    import os
    from golden_util import GOLDEN
    path = os.path.join(GOLDEN, f"prec_{name}.npz")
    return np.load(path, allow_pickle=False) if os.path.exists(path) else None


CAL_RUNS = ("emu32", "emu32p1", "emu32p2")


def _cal_runs(p, mode):
    """The fp32 calibration realisations the fixture holds (emu32, and the input-perturbed twins)."""
    return [r for r in CAL_RUNS if f"{mode}/{r}/steps" in p.files]


def _pgap(p, mode, key, got):
    """(rel err of `got` vs emu64, largest rel gap of an fp32 realisation vs emu64, got, emu64,
    emu32) at the fixture's sampled indices."""
    flat = got.detach().reshape(-1).double().cpu()
    w64 = p[f"{mode}/emu64/{key}/val"]
    w32 = p[f"{mode}/emu32/{key}/val"]
    gap = max(rel_err(p[f"{mode}/{r}/{key}/val"], w64) for r in _cal_runs(p, mode))
    g = flat[torch.from_numpy(p[f"{mode}/emu64/{key}/idx"])].numpy()
    assert_finite(key, g)
    return rel_err(g, w64), gap, g, w64, w32


REDUCED_MIN = 1e-3        # the north star's gate; the calibrated term can only widen it
X3_MIN = 1e-4             # bf16x3 vs its emulation: the exact-f32 mode's gate vs the fp64 reference


def _has_x3(name):
    p = prec_fixture(name)
    return p is not None and "bf16x3/emu64/steps" in p.files and "bf16x3/emu32/steps" in p.files


def test_x3_against_emulation(stepped):
    """bf16x3, step 0: losses, generated volumes and running statistics against the oracle's
    bf16x3 emulation in fp64, within max(1e-4, 4 × the fp32 realisations' gap)."""
    if stepped[2]["precision"] != "bf16x3":
        pytest.skip("bf16x3 only")
    name, mode, p, history, snap = _reduced(stepped)
    w64 = p[f"{mode}/emu64/step0/losses"]
    gap = max(rel_err(p[f"{mode}/{r}/step0/losses"], w64) for r in _cal_runs(p, mode))
    err = rel_err(history[0], w64)
    print(f"{name} bf16x3 step 0: loss rel err vs emulation {err:.2e} (fp32 gap {gap:.2e})")
    assert err < max(X3_MIN, 4 * gap), (history[0], w64)
    for vis, t in snap["vis"].items():
        err, gap, *_ = _pgap(p, mode, f"step0/{vis}", t)
        print(f"{name} bf16x3 {vis}: rel err vs emulation {err:.2e} (fp32 gap {gap:.2e})")
        assert err < max(X3_MIN, 4 * gap), vis
    for net, bufs in snap["bufs"].items():
        for k, b in bufs.items():
            err, gap, *_ = _pgap(p, mode, f"step0/buf/{net}/{k}", b)
            assert err < max(X3_MIN, 4 * gap), (net, k, err, gap)


def _reduced(stepped):
    name, z, meta, _, history, snap = stepped
    p = prec_fixture(name)
    mode = meta["precision"]
    if mode == "bf16x3" and not _has_x3(name):
        pytest.skip(f"no bf16x3 emulation fixture for {name} (tools/gen_precision_fixtures.py)")
    if p is None or f"{mode}/emu64/steps" not in p.files or f"{mode}/emu32/steps" not in p.files:
        pytest.skip(f"no rounded-operand fixture for {name} {mode} (tools/gen_precision_fixtures.py)")
    return name, mode, p, history, snap


def test_reduced_losses(stepped):
    if stepped[2]["precision"] not in REDUCED + ("bf16x3",):
        pytest.skip("exact f32")
    name, mode, p, history, _ = _reduced(stepped)
    for step in range(int(p[f"{mode}/emu64/steps"])):
        w64 = p[f"{mode}/emu64/step{step}/losses"]
        err = rel_err(history[step], w64)
        gap = max(rel_err(p[f"{mode}/{r}/step{step}/losses"], w64) for r in _cal_runs(p, mode))
        # after the first Adam step the runs separate like the reference's fp32 and fp64 (±lr steps
        # of round-off-sized gradients): the later-step factor of the fp32-grade modes
        env = max(REDUCED_MIN, (2.0 if step == 0 else 10.0) * gap)
        print(f"{name} {mode} step {step}: loss rel err {err:.2e} (emu32 gap {gap:.2e}, gate {env:.2e})")
        assert err < env, (step, history[step], w64)


def test_reduced_volumes_and_running_stats(stepped):
    if stepped[2]["precision"] not in REDUCED:
        pytest.skip("fp32-grade mode")
    name, mode, p, _, snap = _reduced(stepped)
    for vis, t in snap["vis"].items():
        err, gap, *_ = _pgap(p, mode, f"step0/{vis}", t)
        print(f"{name} {mode} {vis}: rel err {err:.2e} (emu32 gap {gap:.2e})")
        assert err < max(REDUCED_MIN, 2 * gap), vis
    for net, bufs in snap["bufs"].items():
        for k, b in bufs.items():
            err, gap, *_ = _pgap(p, mode, f"step0/buf/{net}/{k}", b)
            assert err < max(REDUCED_MIN, 2 * gap), (net, k, err, gap)


def test_reduced_gradients(stepped):
    if stepped[2]["precision"] not in REDUCED + ("bf16x3",):
        pytest.skip("exact f32")
    name, mode, p, _, snap = _reduced(stepped)
    bad, n_params = [], 0
    ours, r32, r64 = [], [], []
    for net, grads in snap["grads"].items():
        for k, gr in grads.items():
            if is_pre_in_bias(net, k):
                assert float(gr.abs().max()) == 0.0, (net, k)
                continue
            err, gap, g, w64, w32 = _pgap(p, mode, f"step0/grad/{net}/{k}", gr)
            env = max(REDUCED_MIN, 2 * gap)
            n_params += 1
            if over_envelope(err, env):
                bad.append((net, k, err, env))
            scale = 1.0 / max(float(np.linalg.norm(w64)), 1e-30)
            ours.append(g * scale)
            r64.append(w64 * scale)
            r32.append(w32 * scale)
    check_outliers(f"{name} {mode}", bad, n_params)
    whole = rel_err(np.concatenate(ours), np.concatenate(r64))
    whole_ref = rel_err(np.concatenate(r32), np.concatenate(r64))
    print(f"{name} {mode}: whole-net grad rel err {whole:.2e} (emu32 gap {whole_ref:.2e})")
    assert whole <= max(REDUCED_MIN, 2 * whole_ref), (whole, whole_ref)


def test_reduced_params_after_adam(stepped):
    """Adam's first step is ≈ ±lr·sign(g): count the sampled weights that stepped differently from
    emu64, against twice the emu32 run's count (and at least 2 %)."""
    if stepped[2]["precision"] not in REDUCED + ("bf16x3",):
        pytest.skip("exact f32")
    name, mode, p, _, snap = _reduced(stepped)
    total = bad = bad32 = 0
    for net, params in snap["params"].items():
        for k, t in params.items():
            if is_pre_in_bias(net, k):
                continue
            _, _, g, w64, w32 = _pgap(p, mode, f"step0/param/{net}/{k}", t)
            assert np.abs(g - w64).max() <= 2.05 * 2e-4, (net, k)
            total += g.size
            bad += int((np.abs(g - w64) > 1e-6).sum())
            bad32 += int((np.abs(w32 - w64) > 1e-6).sum())
    print(f"{name} {mode}: {bad}/{total} sampled weights stepped differently (emu32: {bad32})")
    assert bad <= max(0.02 * total, 2 * bad32), (bad, bad32, total)


# ---- fp32-grade modes: against the reference's own fp32 / fp64 runs ------------------------

def test_losses(stepped):
    name, z, meta, _, history, _ = stepped
    if meta["precision"] in REDUCED:
        pytest.skip("reduced precision: test_reduced_losses")
    got = history[0]
    want = z["fp64/step0/losses"]
    assert rel_err(got, want) < LOSS_TOL[meta["precision"]], (got, want)
    if meta["precision"] == "bf16x3" and _has_x3(name):
        return          # later steps: against the bf16x3 emulation's trajectory (test_reduced_losses)
    for step in range(1, meta["steps"]):
        # after an Adam step the reference's own fp32 run has left its fp64 run (elements with a
        # round-off-sized gradient step by ±lr either way): gate on that measured divergence
        w = z[f"fp64/step{step}/losses"]
        ref32 = rel_err(z[f"fp32/step{step}/losses"], w)
        env = max(LATER_MIN[meta["precision"]], LATER_STEP_FACTOR[meta["precision"]] * ref32)
        err = rel_err(history[step], w)
        print(f"{name} step {step}: loss rel err {err:.2e} (reference fp32 {ref32:.2e}, gate {env:.2e})")
        assert err < env, (step, history[step], w)


def test_generated_volumes(stepped):
    name, z, meta, _, _, snap = stepped
    if meta["precision"] in REDUCED:
        pytest.skip("reduced precision: test_reduced_volumes_and_running_stats")
    for vis, t in snap["vis"].items():
        g, w = sampled(z, f"fp64/step0/{vis}", t)
        assert rel_err(g, w) < VOL_TOL[meta["precision"]], vis


# relative input perturbation ≈ the forward error of the generated volumes in each precision
# (exact f32: ≈2e-5 volume error → 4e-6; bf16x3: ≈1.5e-4 → 4e-5)
PERTURB = {"f32": 4e-6, "bf16x3": 4e-5}


@pytest.fixture(scope="module")
def conditioning(stepped):
    """fp64 oracle gradients at inputs perturbed by PERTURB (three realizations): how far the
    exact gradient moves when the forward pass moves by fp32 rounding.  ReLU / LeakyReLU
    pre-activations within ~1e-5 of 0 flip their derivative under such perturbations, which
    makes the step's gradients 1e-3…1e-2-conditioned (tools/diag_d.py traces it)."""
    from oracle.cyclegan_oracle import CycleGANOracle
    name, z, meta, _, _, _ = stepped
    if meta["precision"] in REDUCED or (meta["precision"] == "bf16x3" and _has_x3(name)):
        return None                 # reduced precisions / emulated bf16x3: test_reduced_gradients
    eps = PERTURB[meta["precision"]]
    pre = {4e-6: "fp64p4e-6", 4e-5: "fp64p4e-5"}[eps]
    stored = [q for q in (pre, pre + "r1", pre + "r2", pre + "r3") if f"{q}/loss_names" in z.files]
    if stored:
        # BASELINE-size cases: the fixture holds the perturbed fp64 runs (same protocol, generator
        # seeds 77, 78, 79 — tools/gen_fixtures.py) — returned as sampled vectors keyed like the grads
        return [{"sampled": q} for q in stored]
    A, B = inputs(meta, 0)
    out = []
    for r in range(3):
        g = torch.Generator().manual_seed(77 + r)
        Ap = A.double() * (1 + eps * torch.randn(A.shape, generator=g, dtype=torch.float64))
        Bp = B.double() * (1 + eps * torch.randn(B.shape, generator=g, dtype=torch.float64))
        torch.manual_seed(meta["seed"])
        orc = CycleGANOracle(dtype=torch.float64, pool_rng=random.Random(meta["seed"]), **CASE_KW[name])
        orc.optimize_parameters(Ap, Bp)
        out.append(orc.grads)
    return out


def test_gradients(stepped, conditioning):
    """Per parameter: ‖g − g64‖ ≤ max(1e-3, 2·‖g_ref32 − g64‖, 2·‖g64(perturbed) − g64‖)·‖g64‖
    (SURVEY §8c calibrated protocol, plus the measured conditioning of this step) for all but
    OUTLIER_FRAC of the parameter tensors, and every tensor within OUTLIER_X× its envelope.
    Pre-IN conv biases: exactly 0.  Whole network: the same rule on all sampled elements together,
    no exceptions.  bf16x3 with an emulation fixture: test_reduced_gradients against it instead
    (the split products move the gradients of this ill-conditioned step by more than fp32 does)."""
    name, z, meta, _, _, snap = stepped
    if meta["precision"] in REDUCED:
        pytest.skip("reduced precision: test_reduced_gradients")
    if meta["precision"] == "bf16x3" and _has_x3(name):
        pytest.skip("bf16x3: test_reduced_gradients against the bf16x3 emulation")
    bad = []
    n_params = 0
    ours, ref32, ref64, pert = [], [], [], [[] for _ in conditioning]
    for net, grads in snap["grads"].items():
        for k, gr in grads.items():
            if is_pre_in_bias(net, k):
                assert float(gr.abs().max()) == 0.0, (net, k)
                continue
            key64 = f"fp64/step0/grad/{net}/{k}"
            g, w64 = sampled(z, key64, gr)
            w32 = z[f"fp32/step0/grad/{net}/{k}/val"]
            wp = [z[f"{c['sampled']}/step0/grad/{net}/{k}/val"] if "sampled" in c else sampled(z, key64, c[net][k])[0]
                  for c in conditioning]
            env = max(1e-3, 2 * rel_err(w32, w64), *[2 * rel_err(x, w64) for x in wp])
            assert_finite(f"grad {net}.{k}", g)
            r = rel_err(g, w64)
            n_params += 1
            if over_envelope(r, env):
                bad.append((net, k, r, env))
            scale = 1.0 / max(float(np.linalg.norm(w64)), 1e-30)
            ours.append(g * scale)
            ref32.append(w32 * scale)
            ref64.append(w64 * scale)
            for lst, x in zip(pert, wp):
                lst.append(x * scale)
    # outlier budget: one realization of the perturbation envelope is a noisy estimate and
    # under-states some kink-dominated tensors (measured at 64³: up to 6 of 36 UNet tensors at
    # ≤ 2.3×, 3 of 64 ResNet tensors at ≤ 13×); a kernel bug moves errors to O(1) in many tensors
    check_outliers(f"{name} {meta['precision']}", bad, n_params)
    cat = np.concatenate
    whole = rel_err(cat(ours), cat(ref64))
    whole_ref = rel_err(cat(ref32), cat(ref64))
    whole_pert = max(rel_err(cat(p), cat(ref64)) for p in pert)
    print(f"{name}: whole-net grad rel err {whole:.2e} (reference fp32 {whole_ref:.2e}, "
          f"fp64 under {PERTURB[meta['precision']]:g} input perturbation {whole_pert:.2e})")
    assert whole <= max(1e-3, 2 * whole_ref, 2 * whole_pert), (whole, whole_ref, whole_pert)


def test_running_stats(stepped):
    name, z, meta, _, _, snap = stepped
    if meta["precision"] in REDUCED:
        pytest.skip("reduced precision: test_reduced_volumes_and_running_stats")
    for net, bufs in snap["bufs"].items():
        for k, b in bufs.items():
            g, w = sampled(z, f"fp64/step0/buf/{net}/{k}", b)
            assert rel_err(g, w) < RS_TOL[meta["precision"]], (net, k)


def test_params_after_adam(stepped):
    """Adam's first step moves each weight by ≈ lr·sign(g); elements whose reference gradient
    is at fp32 round-off may flip sign, so gate on the fraction that moved differently."""
    name, z, meta, _, _, snap = stepped
    if meta["precision"] in REDUCED:
        pytest.skip("reduced precision: test_reduced_params_after_adam")
    lr = 2e-4
    total = bad = 0
    for net, params in snap["params"].items():
        for k, p in params.items():
            if is_pre_in_bias(net, k):
                continue
            g, w = sampled(z, f"fp64/step0/param/{net}/{k}", p)
            assert_finite(f"param {net}.{k}", g)
            d = np.abs(g - w)
            assert d.max() <= 2.05 * lr, (net, k, d.max())
            total += d.size
            bad += int((d > 1e-6).sum())
    print(f"{name} {meta['precision']}: {bad}/{total} sampled weights stepped differently")
    assert bad / total < ADAM_FLIP_TOL[meta["precision"]], (bad, total)


# fraction of weights whose first Adam step (≈ ±lr) went the other way: f32-grade modes flip only
# round-off-sized gradients (measured 0.2-0.3 %)
ADAM_FLIP_TOL = {"f32": 0.02, "bf16x3": 0.02}
