"""`torch.ops.mragan.*`: the C-ABI kernels registered as PyTorch custom operators (SURVEY §7.3,
§8(b)), for code that composes its own networks from the engine's kernels instead of driving
the whole CycleGAN step through `models.cycle_gan_model`.

Each op is a `torch.library.custom_op` with a HIP ("cuda") kernel only — there is no CPU kernel,
so a call on a CPU tensor fails loudly — a fake (meta) kernel for shape propagation, and an
autograd formula built from the same library's backward kernels.  Activations are NDHWC
([N, D, H, W, C], fp32, contiguous), the layout of every ops.py call; weights are in torch's own
layout (Conv3d [Cout][Cin][k][k][k], ConvTranspose3d [Cin][Cout][k][k][k]) and are packed per
call (one pack launch in the forward, one for the data gradient in the backward).  Every tensor
argument must be float32 on the input's device (checked: the kernels take raw pointers).  The contraction precision is ops.set_conv_precision's process mode.

  mragan::conv3d           nn.Conv3d / nn.ConvTranspose3d (+ bias, + act)   networks3D.py:185-213
  mragan::instance_norm    nn.InstanceNorm3d(affine=False) (+ act, + replication-padded output)
                                                                            networks3D.py:15-24
  mragan::replication_pad  nn.ReplicationPad3d / the RPad3 of the G stem   networks3D.py:183, 233
  mragan::l1_loss          nn.L1Loss (the cycle / identity losses)          cycle_gan_model.py:104-105
  mragan::gan_loss         GANLoss (BCE on D's sigmoid output, or MSE)      networks3D.py:130-150
  mragan::adam_            torch.optim.Adam step on a flat parameter buffer cycle_gan_model.py:107-110

The loss ops' gradients are the kernels' (sign(a − b)/n, dGANLoss/dp) times the incoming gradient;
they need the process-wide loss scale at 1 (ops.set_loss_scale), which they check.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from . import ops

ACTS = ("none", "relu", "lrelu", "tanh", "sigmoid")


def _act(act: str):
    if act not in ACTS:
        raise ValueError(f"act must be one of {ACTS}, got {act!r}")
    return None if act == "none" else act


def _conv_geometry(x_shape, weight_shape, stride: int, padding: int, output_padding: int, transposed: bool):
    N, D, H, W, cin_x = x_shape
    if len(weight_shape) != 5 or not (weight_shape[2] == weight_shape[3] == weight_shape[4]):
        raise ValueError(f"conv3d: weight must be [A][B][k][k][k], got {tuple(weight_shape)}")
    k = weight_shape[2]
    cin, cout = (weight_shape[0], weight_shape[1]) if transposed else (weight_shape[1], weight_shape[0])
    if cin != cin_x:
        raise ValueError(f"conv3d: input has {cin_x} channels, weight expects {cin}")
    if transposed:
        f = lambda n: ops.convT_out_size(n, k, stride, padding, output_padding)
    else:
        if output_padding:
            raise ValueError("conv3d: output_padding applies to the transposed form only")
        f = lambda n: ops.conv_out_size(n, k, stride, padding)
    return N, (D, H, W), cin, cout, k, (f(D), f(H), f(W))


def _need_f32(t: Optional[torch.Tensor], name: str, device: torch.device, numel: Optional[int] = None):
    """The kernels take raw fp32 device pointers: refuse any other dtype, a tensor on another
    device (a host pointer handed to a device kernel) or a wrong element count before the call."""
    if t is None:
        return
    if t.dtype != torch.float32:
        raise ValueError(f"{name} must be float32, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name} must be on {device}, got {t.device}")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name} must have {numel} elements, got {t.numel()}")


def _pack(weight: torch.Tensor, transposed: bool, data_gradient: bool) -> torch.Tensor:
    """One pack of a torch-layout weight, as engine.ConvLayer.packs: the forward pack
    [t][Cout][Cin] (data_gradient False) or the data-gradient pack [t][Cin][Cout] — one launch."""
    w = weight.contiguous()
    A, B, T = w.shape[0], w.shape[1], w.shape[2] ** 3
    wp = torch.empty(w.numel(), device=w.device, dtype=torch.float32)
    ops.pack_weight(w, A, B, T, transposed != data_gradient, wp)
    return wp


@torch.library.custom_op("mragan::conv3d", mutates_args=(), device_types="cuda")
def conv3d(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int, padding: int,
           output_padding: int, transposed: bool, act: str) -> torch.Tensor:
    N, _, cin, cout, k, osp = _conv_geometry(x.shape, weight.shape, stride, padding, output_padding, transposed)
    _need_f32(x, "conv3d: x", x.device)
    _need_f32(weight, "conv3d: weight", x.device)
    _need_f32(bias, "conv3d: bias", x.device, cout)
    wf = _pack(weight, transposed, data_gradient=False)
    return ops.conv3d(x.contiguous(), wf, cout, k, stride, padding, osp, bias=bias, act=_act(act),
                      transposed=transposed)


@conv3d.register_fake
def _(x, weight, bias, stride, padding, output_padding, transposed, act):
    N, _, _, cout, _, osp = _conv_geometry(x.shape, weight.shape, stride, padding, output_padding, transposed)
    return x.new_empty((N,) + tuple(osp) + (cout,))


def _conv_setup(ctx, inputs, output):
    x, weight, bias, stride, padding, output_padding, transposed, act = inputs
    ctx.save_for_backward(x, weight, output if act != "none" else None)
    ctx.cfg = (bias is not None, stride, padding, transposed, act)


def _conv_backward(ctx, dy):
    x, weight, y = ctx.saved_tensors
    has_bias, stride, padding, transposed, act = ctx.cfg
    g = dy.contiguous()
    _need_f32(g, "conv3d backward: grad_output", x.device)
    if act != "none":                                  # act'(y) from the saved output
        g2 = torch.empty_like(g)
        ops.act_bwd(y, [g], act, g2)
        g = g2
    _, in_sp, cin, cout, k, _ = _conv_geometry(x.shape, weight.shape, stride, padding, 0, transposed)
    dx = dw = db = None
    if ctx.needs_input_grad[0]:
        wb = _pack(weight, transposed, data_gradient=True)
        dx = ops.conv3d(g, wb, cin, k, stride, padding, in_sp, transposed=not transposed)
    if ctx.needs_input_grad[1]:
        dw = torch.empty(weight.shape, device=weight.device, dtype=torch.float32)
        if transposed:
            ops.conv3d_wgrad(x.contiguous(), g, k, stride, padding, dw, False)     # dW[Cin][Cout][t]
        else:
            ops.conv3d_wgrad(g, x.contiguous(), k, stride, padding, dw, False)     # dW[Cout][Cin][t]
    if has_bias and ctx.needs_input_grad[2]:
        db = torch.empty(cout, device=dy.device, dtype=torch.float32)
        ops.channel_sum(g, db)
    return dx, dw, db, None, None, None, None, None


conv3d.register_autograd(_conv_backward, setup_context=_conv_setup)


@torch.library.custom_op("mragan::instance_norm", mutates_args=(), device_types="cuda")
def instance_norm(x: torch.Tensor, act: str, ypad: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    y, mean, rstd = ops.instnorm_fwd(x.contiguous(), act=_act(act), ypad=ypad)
    return y, mean, rstd


@instance_norm.register_fake
def _(x, act, ypad):
    N, D, H, W, C = x.shape
    return (x.new_empty((N, D + 2 * ypad, H + 2 * ypad, W + 2 * ypad, C)), x.new_empty((N, C)),
            x.new_empty((N, C)))


def _in_setup(ctx, inputs, output):
    x, act, ypad = inputs
    _, mean, rstd = output
    ctx.save_for_backward(x, mean, rstd)
    ctx.cfg = (act, ypad)
    ctx.mark_non_differentiable(mean, rstd)


def _in_backward(ctx, dy, _dmean, _drstd):
    x, mean, rstd = ctx.saved_tensors
    act, ypad = ctx.cfg
    dx = ops.instnorm_bwd(x.contiguous(), mean, rstd, dy.contiguous(), dypad=ypad, act=_act(act))
    return dx, None, None


instance_norm.register_autograd(_in_backward, setup_context=_in_setup)


@torch.library.custom_op("mragan::replication_pad", mutates_args=(), device_types="cuda")
def replication_pad(x: torch.Tensor, p: int) -> torch.Tensor:
    return ops.rpad(x.contiguous(), p)


@replication_pad.register_fake
def _(x, p):
    N, D, H, W, C = x.shape
    return x.new_empty((N, D + 2 * p, H + 2 * p, W + 2 * p, C))


def _rpad_setup(ctx, inputs, output):
    ctx.p = inputs[1]


def _rpad_backward(ctx, dy):
    return ops.rpad_fold(dy.contiguous(), ctx.p), None


replication_pad.register_autograd(_rpad_backward, setup_context=_rpad_setup)


def _unit_loss_scale(name: str):
    if ops.get_loss_scale() != 1.0:
        raise RuntimeError(f"mragan::{name} backward: the process-wide loss scale is {ops.get_loss_scale()}, "
                           "expected 1 (the kernels fold it into the gradient)")


@torch.library.custom_op("mragan::l1_loss", mutates_args=(), device_types="cuda")
def l1_loss(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if a.shape != b.shape:
        raise ValueError(f"l1_loss: shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    _need_f32(a, "l1_loss: a", a.device)
    _need_f32(b, "l1_loss: b", a.device)
    loss = torch.empty((), device=a.device, dtype=torch.float32)
    ops.l1_loss(a.contiguous(), b.contiguous(), 1.0, loss, None)
    return loss


@l1_loss.register_fake
def _(a, b):
    return a.new_empty(())


def _l1_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _l1_backward(ctx, dloss):
    a, b = ctx.saved_tensors
    _unit_loss_scale("l1_loss")
    g = torch.empty(a.shape, device=a.device, dtype=torch.float32)
    slot = torch.empty((), device=a.device, dtype=torch.float32)
    ops.l1_loss(a.contiguous(), b.contiguous(), 1.0, slot, g)
    g = g * dloss
    return (g if ctx.needs_input_grad[0] else None), (-g if ctx.needs_input_grad[1] else None)


l1_loss.register_autograd(_l1_backward, setup_context=_l1_setup)


@torch.library.custom_op("mragan::gan_loss", mutates_args=(), device_types="cuda")
def gan_loss(p: torch.Tensor, target: float, lsgan: bool) -> torch.Tensor:
    _need_f32(p, "gan_loss: p", p.device)
    loss = torch.empty((), device=p.device, dtype=torch.float32)
    ops.gan_loss(p.contiguous(), target, lsgan, 1.0, loss, None)
    return loss


@gan_loss.register_fake
def _(p, target, lsgan):
    return p.new_empty(())


def _gan_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])
    ctx.cfg = (inputs[1], inputs[2])


def _gan_backward(ctx, dloss):
    (p,) = ctx.saved_tensors
    target, lsgan = ctx.cfg
    _unit_loss_scale("gan_loss")
    dp = torch.empty(p.shape, device=p.device, dtype=torch.float32)
    slot = torch.empty((), device=p.device, dtype=torch.float32)
    ops.gan_loss(p.contiguous(), target, lsgan, 1.0, slot, dp)
    return dp * dloss, None, None


gan_loss.register_autograd(_gan_backward, setup_context=_gan_setup)


@torch.library.custom_op("mragan::adam_", mutates_args=("param", "exp_avg", "exp_avg_sq"), device_types="cuda")
def adam_(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, lr: float,
          beta1: float, beta2: float, eps: float, step: int, grad_scale: float) -> None:
    """One torch.optim.Adam step (amsgrad False, weight_decay 0) in place; `step` counts from 1."""
    for t, n in ((param, "param"), (grad, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != param.numel():
            raise ValueError(f"adam_: {n} must be a contiguous float32 tensor of {param.numel()} elements")
    ops.adam(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, step, grad_scale)


@adam_.register_fake
def _(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, step, grad_scale):
    return None


OPS: List[str] = ["conv3d", "instance_norm", "replication_pad", "l1_loss", "gan_loss", "adam_"]
