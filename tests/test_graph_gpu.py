"""The HIP-graph step (default from the 2nd optimize_parameters() on) against the eager step
(--no_cuda_graph): identical kernels in identical order, so losses, parameters, running
statistics and generated volumes must agree bit for bit over several steps — with a 2-image
pool, so the steps exercise the pool's swaps, and with an lr scheduler changing lr between
steps (the graph reads Adam's scalars from device memory)."""
import random
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(tmp_path, graph, steps, precision, batches=None, extra=(), size=24, nc=1):
    from models import create_model
    from options.train_options import TrainOptions
    argv = sys.argv
    try:
        sys.argv = ["train.py", "--checkpoints_dir", str(tmp_path), "--conv_precision", precision,
                    "--netG", "resnet_6blocks", "--ngf", "8", "--ndf", "8", "--pool_size", "2",
                    "--batch_size", "2", "--lr_policy", "step", "--lr_decay_iters", "1"] + list(extra)
        if not graph:
            sys.argv.append("--no_cuda_graph")
        opt = TrainOptions().gather_options()
    finally:
        sys.argv = argv
    opt.isTrain, opt.gpu_ids = True, 0
    torch.manual_seed(3)
    random.seed(3)
    model = create_model(opt)
    model.setup(opt)
    g = torch.Generator().manual_seed(5)
    losses = []
    for step in range(steps):
        b = batches[step] if batches else 2
        A = torch.randn(b, nc, size, size, size, generator=g)
        B = torch.randn(b, nc, size, size, size, generator=g)
        model.set_input([A, B])
        model.optimize_parameters()
        losses.append(torch.stack([getattr(model, "loss_" + n).detach().clone() for n in model.loss_names]))
        if step == 2:
            model.update_learning_rate()
    torch.cuda.synchronize()
    state = {}
    for n in ("G_A", "G_B", "D_A", "D_B"):
        for k, v in getattr(model, "net" + n).state_dict().items():
            state[f"{n}/{k}"] = v.detach().cpu().clone()
    vis = {v: getattr(model, v).detach().cpu().clone() for v in ("fake_B", "rec_A", "fake_A", "rec_B", "idt_A")
           if hasattr(model, v)}
    return torch.stack(losses).cpu(), state, vis, model


@pytest.mark.parametrize("precision", ["f32", "bf16x3", "bf16", "fp16"])
def test_graph_step_bit_identical_to_eager(tmp_path, precision):
    from mragan_hip import ops
    try:
        le, se, ve, me = _run(tmp_path / "e", False, 6, precision)
        lg, sg, vg, mg = _run(tmp_path / "g", True, 6, precision)
    finally:
        ops.set_conv_precision("f32")
    assert me._graphs is None and mg._graphs is not None
    assert mg.fake_B_pool.num_imgs == 2
    assert torch.equal(le, lg), (le - lg).abs().max()
    for k in se:
        assert torch.equal(se[k], sg[k]), k
    for k in ve:
        assert torch.equal(ve[k], vg[k]), k


def test_graph_step_changing_batch_and_no_identity(tmp_path):
    """An epoch's smaller last batch (train.py:52, no drop_last) between full ones, with
    --lambda_identity 0 (no identity passes): the graphed step captures once per batch shape and replays the cached captures, the
    pool keeps its images across the change, and everything stays bit-identical to eager."""
    batches = [2, 2, 1, 2, 2, 1, 2]
    extra = ["--lambda_identity", "0"]
    le, se, ve, me = _run(tmp_path / "e", False, len(batches), "f32", batches, extra)
    lg, sg, vg, mg = _run(tmp_path / "g", True, len(batches), "f32", batches, extra)
    assert mg._graphs is not None and not hasattr(mg, "idt_A")
    # one capture per batch shape: the alternation replays cached captures (no recapture)
    assert mg._n_captures == 2 and len(mg._graph_cache) == 2
    assert mg.fake_B_pool.num_imgs == 2
    assert torch.equal(le, lg), (le - lg).abs().max()
    assert float(le[:, 3].abs().max()) == 0.0 and float(le[:, 7].abs().max()) == 0.0   # loss_idt_*
    for k in se:
        assert torch.equal(se[k], sg[k]), k
    for k in ve:
        assert torch.equal(ve[k], vg[k]), k


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_stride2_planes_bit_identical(tmp_path, precision, monkeypatch):
    """ABI 14 / 16: in the one-plane modes the stride-2 layers' operands exist as 16-bit planes —
    the stem's and down1's IN outputs (down1 / down2 inputs), the last block's output (up1's
    input), the IN-backward outputs of up1 / up2 / down2 — read by the implicit GEMMs and wgrad3s2.  The step must
    agree bit for bit with the step that keeps that tensor in fp32 (the kernels round it to the very
    same words) — and the plane path must actually have run."""
    from mragan_hip import engine, ops
    calls = []
    g16, op16 = ops.conv3d_wgrad_g16, ops.conv3d_wgrad_op16
    monkeypatch.setattr(ops, "conv3d_wgrad_g16",
                        lambda dense, gath, k, s, *a, **kw: (calls.append(("g16", gath.shape[-1])),
                                                             g16(dense, gath, k, s, *a, **kw))[1])
    monkeypatch.setattr(ops, "conv3d_wgrad_op16",
                        lambda dense, gath, k, s, *a, **kw: (s == 2 and calls.append(("both", gath.shape[-1])),
                                                             op16(dense, gath, k, s, *a, **kw))[1])
    extra = ["--ngf", "32"]
    try:
        monkeypatch.setattr(engine, "_NO_S2_PLANES", True)
        lr, sr, vr, _ = _run(tmp_path / "r", False, 3, precision, extra=extra, size=64)
        assert not calls
        monkeypatch.setattr(engine, "_NO_S2_PLANES", False)
        lp, sp, vp, _ = _run(tmp_path / "p", False, 3, precision, extra=extra, size=64)
    finally:
        ops.set_conv_precision("f32")
        ops.set_loss_scale(1.0)
    # down1 / up2 (32-channel gathered plane; both operands as planes with brickT on planes), up1
    # (64, dense fp32), down2 (both operands as planes, 64-channel gathered)
    want = {("both" if engine._BRICKT_PLANES else "g16", 32), ("g16", 64), ("both", 64)}
    assert set(calls) == want, f"plane paths that ran: {set(calls)}"
    assert torch.equal(lr, lp), (lr - lp).abs().max()
    for k in sr:
        assert torch.equal(sr[k], sp[k]), k
    for k in vr:
        assert torch.equal(vr[k], vp[k]), k


# the dispatch the bench times (BASELINE configs[1]: resnet_9blocks, ngf 32, 64³ b2, two lanes) and
# configs[4]'s per-GPU unit (96³ nc2 b1 fp16: its first passes run N = 2 at the 24³ level — the
# interior + shell data gradient)
HEADLINE = ["--netG", "resnet_9blocks", "--ngf", "32", "--ndf", "32"]
HEADLINE_CASES = [("bf16", 64, 2, 1), ("fp16", 64, 2, 1), ("fp16", 96, 1, 2)]


@pytest.mark.parametrize("precision,size,batch,nc", HEADLINE_CASES,
                         ids=[f"{p}-{s}-b{b}-nc{c}" for p, s, b, c in HEADLINE_CASES])
def test_graph_step_bit_identical_headline(tmp_path, precision, size, batch, nc, monkeypatch):
    """the replayed two-lane step at the BASELINE sizes is the eager step, bit
    for bit, over 3 steps (the eager step 0 is what tests/test_step_gpu.py gates against the oracle;
    steps 1-2 replay the capture) — and the dispatch under test is the headline's: counted at the
    library boundary, the K-split brick's in-launch finalize (ABI 15), the skip-gradient statistics
    epilogue (ABI 18) and, where the size rule holds, the interior + shell data gradient ran."""
    from mragan_hip import ops
    seen = {"fin": 0, "skip_stats": 0, "split": 0}
    op16, fin16, st16 = ops.conv3d_op16, ops._conv3d_op16_fin, ops.conv3d_op16_dgrad_in_stats

    def fin_w(*a, **kw):
        r = fin16(*a, **kw)
        seen["fin"] += r[2] is not None
        return r

    def op16_w(x16, wp, cout, k, s, p, osp, wsplit, part=None, transposed=False, fin=False):
        if transposed and k == 3 and s == 1 and ops.dgrad_split(*x16.shape, cout):
            seen["split"] += 1
        return op16(x16, wp, cout, k, s, p, osp, wsplit, part=part, transposed=transposed, fin=fin)

    def st_w(*a, x_add=None, **kw):
        r = st16(*a, x_add=x_add, **kw)
        seen["skip_stats"] += x_add is not None and r[1] > 0
        return r

    monkeypatch.setattr(ops, "_conv3d_op16_fin", fin_w)
    monkeypatch.setattr(ops, "conv3d_op16", op16_w)
    monkeypatch.setattr(ops, "conv3d_op16_dgrad_in_stats", st_w)
    extra = HEADLINE + ["--batch_size", str(batch), "--input_nc", str(nc), "--output_nc", str(nc)]
    try:
        le, se, ve, me = _run(tmp_path / "e", False, 3, precision, [batch] * 3, extra, size=size, nc=nc)
        assert me.parallel_lanes and me._aux_stream is not None
        del me
        torch.cuda.empty_cache()
        eager_seen = dict(seen)
        lg, sg, vg, mg = _run(tmp_path / "g", True, 3, precision, [batch] * 3, extra, size=size, nc=nc)
        assert mg._graphs is not None and mg._n_captures == 1
        del mg
    finally:
        ops.set_conv_precision("f32")
        ops.set_loss_scale(1.0)
        torch.cuda.empty_cache()
    print(f"{precision} {size}³ b{batch} nc{nc}: library paths per eager run {eager_seen}")
    assert eager_seen["skip_stats"] > 0, eager_seen
    if size == 64:      # the 16³ level: K-split bricks with the in-launch finalize, no split
        assert eager_seen["fin"] > 0 and eager_seen["split"] == 0, eager_seen
    else:               # the 24³ level at N = 2: the interior + shell data gradient
        assert eager_seen["split"] > 0, eager_seen
    assert torch.isfinite(le).all()
    assert torch.equal(le, lg), (le - lg).abs().max()
    for k in se:
        assert torch.equal(se[k], sg[k]), k
    for k in ve:
        assert torch.equal(ve[k], vg[k]), k


@pytest.mark.parametrize("precision", ["bf16", "f32"])
def test_overlapped_d_phase_bit_identical(tmp_path, precision, monkeypatch):
    """Round 6: on one GPU the D phase — and the frozen discriminator passes of backward_G — run
    beside the G backward on two more streams, in the same graph (CycleGANModel._phase_GD).  They
    compute the same kernels on the same operands and form the same sums as the two-phase schedule
    (MRAGAN_TWO_PHASE: G phase, G Adam, D phase, D Adam) and as the overlapped schedule with the
    frozen passes on the lanes (MRAGAN_FROZEN_D_ON_LANES), so over several replayed steps every
    loss, parameter, running statistic and volume is bit-identical."""
    from models import cycle_gan_model as cgm
    extra = ["--netG", "resnet_9blocks", "--ngf", "16", "--ndf", "16"]
    try:
        monkeypatch.setattr(cgm, "_TWO_PHASE", True)
        lt, st, vt, mt = _run(tmp_path / "t", True, 4, precision, extra=extra, size=32)
        assert mt._graphs[1] is not None
        del mt
        monkeypatch.setattr(cgm, "_TWO_PHASE", False)
        monkeypatch.setattr(cgm, "_FROZEN_D_ON_LANES", True)
        lf, sf, vf, mf = _run(tmp_path / "f", True, 4, precision, extra=extra, size=32)
        del mf
        monkeypatch.setattr(cgm, "_FROZEN_D_ON_LANES", False)
        lo, so, vo, mo = _run(tmp_path / "o", True, 4, precision, extra=extra, size=32)
        assert mo._graphs[1] is None and mo._d_streams is not None
        del mo
    finally:
        from mragan_hip import ops
        ops.set_conv_precision("f32")
        ops.set_loss_scale(1.0)
    for l2, s2, v2 in ((lf, sf, vf), (lo, so, vo)):   # frozen D passes on the lanes / on the side streams
        assert torch.equal(lt, l2), (lt - l2).abs().max()
        for k in st:
            assert torch.equal(st[k], s2[k]), k
        for k in vt:
            assert torch.equal(vt[k], v2[k]), k
