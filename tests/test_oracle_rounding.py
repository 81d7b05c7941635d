"""The oracle's reduced-precision mode (RoundedConv, oracle/cyclegan_oracle.py) — the parity
target of the engine's bf16 / fp16 steps: forward = conv of the rounded operands (+ unrounded
bias), data gradient = from R(dY) and R(W), weight gradient = from R(X) and R(dY), fp16 gradients
rounded under the loss scale.  CPU only."""
import pytest
import torch
import torch.nn.functional as F

from oracle.cyclegan_oracle import CycleGANOracle, RoundedConv, synthetic_pair


def _r(t, dt):
    return t.float().to(dt).double()


@pytest.mark.parametrize("mode,scale", [("bf16", 1.0), ("fp16", 1024.0)])
@pytest.mark.parametrize("transposed", [False, True])
def test_rounded_conv_formulas(mode, scale, transposed):
    g = torch.Generator().manual_seed(3)
    dt = torch.bfloat16 if mode == "bf16" else torch.float16
    x = torch.randn(2, 6, 5, 6, 7, generator=g, dtype=torch.float64, requires_grad=True)
    cw = (6, 4) if transposed else (4, 6)
    w = (torch.randn(*cw, 3, 3, 3, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    b = torch.randn(4, generator=g, dtype=torch.float64, requires_grad=True)
    rc = RoundedConv(mode, scale)
    kw = dict(stride=2, padding=1)
    if transposed:
        y = rc.conv_transpose3d(x, w, b, output_padding=1, **kw)
        ref = F.conv_transpose3d(_r(x, dt), _r(w, dt), b.detach(), output_padding=1, **kw)
    else:
        y = rc.conv3d(x, w, b, **kw)
        ref = F.conv3d(_r(x, dt), _r(w, dt), b.detach(), **kw)
    assert torch.equal(y.detach(), ref)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64) * 1e-3
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), dy)
    dyr = (dy.float() * scale).to(dt).double() / scale
    xr, wr = _r(x.detach(), dt).requires_grad_(), _r(w.detach(), dt).requires_grad_()
    yy = (F.conv_transpose3d(xr, wr, output_padding=1, **kw) if transposed else F.conv3d(xr, wr, **kw))
    ex, ew = torch.autograd.grad(yy, (xr, wr), dyr)
    assert torch.allclose(gx, ex, rtol=0, atol=1e-15) and torch.allclose(gw, ew, rtol=0, atol=1e-15)
    assert torch.allclose(gb, dy.sum((0, 2, 3, 4)))
    # the rounding is real: the exact gradient differs at the operand roundoff
    xe, we = x.detach().requires_grad_(), w.detach().requires_grad_()
    ye = F.conv_transpose3d(xe, we, output_padding=1, **kw) if transposed else F.conv3d(xe, we, **kw)
    (gwe,) = torch.autograd.grad(ye, we, dy)
    assert float((gw - gwe).norm() / gwe.norm()) > (1e-4 if mode == "fp16" else 1e-3)


def test_rounded_step_runs_and_moves_by_operand_roundoff():
    """A whole step (resnet_6blocks ngf 8, 2 channels, 24³) in each mode: finite, close to the
    exact step at the scale of the operand rounding, not identical to it."""
    A, B = synthetic_pair((1, 2, 24, 24, 24), 5)
    res = {}
    for mode in (None, "bf16", "fp16"):
        torch.manual_seed(0)
        orc = CycleGANOracle(input_nc=2, output_nc=2, ngf=8, ndf=8, n_blocks=6, dtype=torch.float64,
                             operand_rounding=mode, loss_scale=1024.0 if mode == "fp16" else 1.0)
        losses = orc.optimize_parameters(A, B)
        res[mode] = (torch.tensor(list(losses.values())), orc.fake_B)
    for mode, hi in (("bf16", 0.2), ("fp16", 0.03)):
        dl = float((res[mode][0] - res[None][0]).norm() / res[None][0].norm())
        dv = float((res[mode][1] - res[None][1]).norm() / res[None][1].norm())
        assert 0 < dl < hi and 0 < dv < hi, (mode, dl, dv)
