"""CPU-side checks: the C-ABI library loads and exports every symbol include/mragan_hip.h
declares (no compute calls without a GPU), and the drop-in model layer reproduces the
reference's construction (state_dict keys, init weights) from the golden fixtures."""
import os
import random
import re
import sys

import numpy as np
import pytest
import torch

from golden_util import CASE_KW, available_cases, load, sampled

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mragan_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mragan_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    fns = header_functions()
    for f in ("mragan_conv3d_fwd", "mragan_conv3d_transposed", "mragan_conv3d_presplit", "mragan_conv3d_wgrad", "mragan_instnorm_fwd",
              "mragan_instnorm_bwd", "mragan_adam", "mragan_gan_loss", "mragan_l1_loss"):
        assert f in fns


def test_library_exports_every_header_symbol():
    import mragan_hip
    lib = mragan_hip.lib()
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert set(header_functions()) == set(mragan_hip.exported_symbols())
    assert lib.mragan_abi_version() == 19


def test_library_built_for_gfx950():
    import mragan_hip
    data = open(mragan_hip.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_bad_args_reported_without_gpu():
    """Argument validation runs on the host: a null pointer is rejected with a message."""
    import mragan_hip
    from mragan_hip._lib import MraganError, call
    with pytest.raises(MraganError, match="null pointer"):
        call("mragan_conv3d_fwd", None, 1, 4, 4, 4, 8, None, None, 8, 3, 1, 1, 0, None, 4, 4, 4, None, 0, None)


def test_dgrad_split_rule_query():
    """ABI 19: the interior + shell data-gradient rule is the library's (host-side, no GPU), and the
    engine schedules by the same query — there is no mirrored copy to drift.  Split for N ≥ 2 at
    24³ / 32³ in the one-plane modes; never at 16³, at N = 1, or in the fp32-grade modes."""
    import mragan_hip
    from mragan_hip import engine, ops
    lib = mragan_hip.lib()
    try:
        for prec in ("bf16", "fp16"):
            ops.set_conv_precision(prec)
            for N, S, want in [(2, 32, 1), (2, 24, 1), (4, 24, 1), (4, 16, 0), (2, 16, 0), (1, 32, 0), (2, 28, 0)]:
                assert lib.mragan_conv3d_dgrad_split(N, S, S, S, 128, 128) == want, (prec, N, S)
                assert engine._dgrad_split(N, S, S, S, 128) == bool(want)
        for prec in ("f32", "bf16x3"):
            ops.set_conv_precision(prec)
            assert lib.mragan_conv3d_dgrad_split(2, 32, 32, 32, 128, 128) == 0
    finally:
        ops.set_conv_precision("f32")


def _build(name):
    from models import create_model
    from options.train_options import TrainOptions
    z, meta = load(name)
    argv = sys.argv
    try:
        sys.argv = ["train.py", "--checkpoints_dir", "/tmp/mragan_cpu_test"] + meta["argv"].split()
        opt = TrainOptions().gather_options()
    finally:
        sys.argv = argv
    opt.isTrain = True
    opt.gpu_ids = 0
    torch.manual_seed(meta["seed"])
    random.seed(meta["seed"])
    return z, meta, create_model(opt)


@pytest.mark.parametrize("name", available_cases())
def test_model_init_matches_reference(name):
    """The drop-in define_G/define_D consume the RNG like the reference: bit-identical weights."""
    z, meta, model = _build(name)
    n = 0
    for net in ("G_A", "G_B", "D_A", "D_B"):
        sd = getattr(model, "net" + net).state_dict()
        for k, v in sd.items():
            key = f"init/{net}/{k}"
            if key + "/idx" in z.files:
                g, w = sampled(z, key, v)
                np.testing.assert_array_equal(g, w)
                n += 1
    assert n > 20


def test_state_dict_keys_and_counts():
    z, meta, model = _build("step_r9_s32_b1")
    sd = model.netG_A.state_dict()
    assert len(sd) == 117                       # 117 entries for resnet_9blocks
    assert "model.10.conv_block.1.weight" in sd and "model.26.bias" in sd
    assert len(model.netD_A.state_dict()) == 19
    assert sum(p.numel() for p in model.netG_A.parameters()) == 8540161
    assert sum(p.numel() for p in model.netD_A.parameters()) == 2771425   # A16


def test_checkpoint_roundtrip(tmp_path):
    """save_networks/load_networks (reference base_model.py:89-148): '{epoch}_net_{name}.pth' files
    holding CPU state_dicts with the reference's keys; loading restores the weights in place (the
    flat-buffer parameter views stay valid) and fills num_batches_tracked like the reference's
    InstanceNorm patching does."""
    z, meta, model = _build("step_r6_s24_b2_nc2_lsgan")
    model.save_dir = str(tmp_path)
    model.save_networks("latest")
    ref_keys = {f.split("/")[2] for f in z.files if f.startswith("init/G_A/")}
    sd = torch.load(tmp_path / "latest_net_G_A.pth", weights_only=True)
    assert ref_keys <= set(sd) and all(v.device.type == "cpu" for v in sd.values())
    torch.manual_seed(123)
    _, _, other = _build("step_r6_s24_b2_nc2_lsgan")
    other.save_dir = str(tmp_path)
    ptr = other.netG_A.model[1].weight.data_ptr()
    other.load_networks("latest")
    assert other.netG_A.model[1].weight.data_ptr() == ptr
    for net in ("G_A", "G_B", "D_A", "D_B"):
        a = getattr(model, "net" + net).state_dict()
        b = getattr(other, "net" + net).state_dict()
        assert a.keys() == b.keys()
        for k in a:
            assert torch.equal(a[k].cpu(), b[k].cpu()), (net, k)


def test_options_defaults_and_quirks():
    from options.train_options import TrainOptions
    argv = sys.argv
    try:
        sys.argv = ["train.py"]
        opt = TrainOptions().gather_options()
        sys.argv = ["train.py", "--no_lsgan"]
        opt2 = TrainOptions().gather_options()
    finally:
        sys.argv = argv
    assert opt.netG == "resnet_6blocks" and opt.ngf == 32 and opt.ndf == 32
    assert opt.no_lsgan is True and opt2.no_lsgan is False      # store_false quirk
    assert opt.lambda_A == 10.0 and opt.lambda_identity == 0.5 and opt.no_dropout is True
    assert opt.patch_size == [64.0, 64.0, 64.0]


def test_unknown_model_exits_zero(capsys):
    from models import find_model_using_name
    with pytest.raises(ModuleNotFoundError):
        find_model_using_name("nonexistent")


def test_plan_compiles_on_cpu():
    from mragan_hip.engine import compile_nlayer_discriminator, compile_resnet_generator
    z, meta, model = _build("step_r9_s32_b1")
    pg = compile_resnet_generator(model.netG_A)
    kinds = [s.kind for s in pg.stages]
    assert kinds == ["conv"] * 3 + ["block"] * 9 + ["conv"] * 3
    assert pg.stages[0].prepad == 3 and pg.stages[-1].prepad == 3 and pg.stages[-1].act == "tanh"
    assert pg.stages[-1].use_bias and not pg.stages[0].use_bias
    pd = compile_nlayer_discriminator(model.netD_A)
    assert [s.norm is not None for s in pd.stages] == [False, True, True, True, False]
    assert pd.stages[-1].act == "sigmoid" and pd.stages[0].act == "lrelu"


def test_engine_refuses_cpu_tensors():
    z, meta, model = _build("step_r6_s24_b2_nc2_lsgan")
    with pytest.raises(RuntimeError, match="HIP device only"):
        model.netG_A(torch.zeros(1, 2, 8, 8, 8))


def test_unet_state_dict_and_plan():
    """UnetGenerator (networks3D.py:270-343): the reference's nested keys (every weight the
    reference fixture sampled exists here), only the outermost upconv has a bias, and the plan
    runs outermost → innermost with the norms where the reference puts them."""
    from mragan_hip.engine import compile_unet_generator
    z, meta, model = _build("step_unet_s32_b2_ngf8")
    sd = model.netG_A.state_dict()
    ref_keys = {f.split("/")[2] for f in z.files if f.startswith("init/G_A/") and f.endswith("/idx")}
    assert ref_keys and ref_keys <= set(sd)
    assert [k for k in sd if k.endswith(".bias")] == ["model.model.3.bias"]
    plan = compile_unet_generator(model.netG_A)
    assert [lv.kind for lv in plan.levels] == ["outer", "mid", "mid", "mid", "inner"]
    assert [lv.down.cout for lv in plan.levels] == [8, 16, 32, 64, 64]
    assert [lv.up.cin for lv in plan.levels] == [16, 32, 64, 128, 64]
    assert all(lv.down_norm is not None for lv in plan.levels[1:4])
    assert plan.levels[-1].up_norm is not None and plan.levels[0].up_norm is None


def test_unet_256_too_small_raises():
    """unet_256 (8 downsamplings) cannot run on a 64³ patch in the reference either (SURVEY §8a
    A18: an InstanceNorm over one voxel raises ValueError)."""
    from mragan_hip.engine import UnetPlan, compile_unet_generator
    from models import networks3D
    net = networks3D.UnetGenerator(1, 1, 8, 8, norm_layer=networks3D.get_norm_layer('instance'))
    plan = compile_unet_generator(net)
    with pytest.raises(ValueError, match="more than 1 spatial element"):
        UnetPlan._check_spatial((1, 64, 64, 64, 1), plan.levels)
    UnetPlan._check_spatial((1, 256, 256, 256, 1), plan.levels)
