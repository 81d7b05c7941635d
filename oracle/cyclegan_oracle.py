"""CPU oracle for the MRA-GAN CycleGAN hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the HIP engine in ``mra-gan_amd/``.  It is a
functional restatement, in PyTorch-CPU (fp32 or fp64), of the reference's
``CycleGANModel.optimize_parameters()`` step and everything under it:

* ResnetGenerator / ResnetBlock      (reference models/networks3D.py:173-263)
* UnetGenerator / UnetSkipConnectionBlock (reference models/networks3D.py:270-343)
* NLayerDiscriminator                (reference models/networks3D.py:381-425)
* InstanceNorm3d(affine=False, track_running_stats=True) in train mode
                                     (reference models/networks3D.py:15-24)
* GANLoss (BCE or LSGAN), L1 losses  (reference models/networks3D.py:130-150,
                                      models/cycle_gan_model.py:103-105)
* ImagePool                          (reference models/cycle_gan_model.py:8-35)
* torch.optim.Adam                   (reference models/cycle_gan_model.py:107-110)
* the step orchestration             (reference models/cycle_gan_model.py:121-240)
* deterministic init (same RNG consumption as the reference's constructors +
  init_weights, so a given torch seed yields bit-identical initial weights)
                                     (reference models/networks3D.py:44-81)

Pinning: the oracle is checked against golden fixtures produced by running the
reference itself in the build container (``tools/gen_fixtures.py`` →
``tests/golden/``; test ``tests/test_oracle_golden.py``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  The product path never does.
"""
from __future__ import annotations

import math
import random
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F
from torch.nn import init

IN_EPS = 1e-5          # nn.InstanceNorm3d default eps
IN_MOMENTUM = 0.1      # nn.InstanceNorm3d default momentum
LRELU_SLOPE = 0.2      # networks3D.py:393


# --------------------------------------------------------------------------------------
# Architecture specs (state_dict indices identical to the reference's nn.Sequential)
# --------------------------------------------------------------------------------------

def resnet_generator_layers(input_nc: int, output_nc: int, ngf: int, n_blocks: int) -> List[dict]:
    """Layer list of ResnetGenerator (networks3D.py:173-220) with the reference's
    Sequential indices as state_dict prefixes.  Each entry is one conv (+ its norm/act)."""
    layers = []
    idx = 0
    # RPad3 (idx 0) → Conv k7 (1) → IN (2) → ReLU (3)   networks3D.py:185-189
    layers.append(dict(kind="conv", name=f"model.{idx+1}", cin=input_nc, cout=ngf, k=7, s=1, p=0,
                       prepad=3, bias=True, norm=f"model.{idx+2}", act="relu"))
    idx += 4
    # 2 × [Conv k3 s2 p1 → IN → ReLU]                      networks3D.py:191-197
    for i in range(2):
        mult = 2 ** i
        layers.append(dict(kind="conv", name=f"model.{idx}", cin=ngf * mult, cout=ngf * mult * 2, k=3, s=2,
                           p=1, prepad=0, bias=True, norm=f"model.{idx+1}", act="relu"))
        idx += 3
    # ResnetBlocks                                       networks3D.py:199-201, 224-263
    dim = ngf * 4
    for b in range(n_blocks):
        pre = f"model.{idx}.conv_block"
        layers.append(dict(kind="resblock", name=f"model.{idx}", dim=dim,
                           conv1=f"{pre}.1", norm1=f"{pre}.2", conv2=f"{pre}.5", norm2=f"{pre}.6"))
        idx += 1
    # 2 × [ConvT k3 s2 p1 op1 → IN → ReLU]                 networks3D.py:203-210
    for i in range(2):
        mult = 2 ** (2 - i)
        layers.append(dict(kind="convT", name=f"model.{idx}", cin=ngf * mult, cout=ngf * mult // 2, k=3,
                           s=2, p=1, op=1, bias=True, norm=f"model.{idx+1}", act="relu"))
        idx += 3
    # RPad3 → Conv k7 (ngf → output_nc) → Tanh             networks3D.py:211-213
    layers.append(dict(kind="conv", name=f"model.{idx+1}", cin=ngf, cout=output_nc, k=7, s=1, p=0,
                       prepad=3, bias=True, norm=None, act="tanh"))
    return layers


def nlayer_discriminator_layers(input_nc: int, ndf: int, n_layers: int, use_sigmoid: bool) -> List[dict]:
    """Layer list of NLayerDiscriminator (networks3D.py:381-425)."""
    layers = [dict(kind="conv", name="model.0", cin=input_nc, cout=ndf, k=4, s=2, p=1, prepad=0,
                   bias=True, norm=None, act="lrelu")]
    idx = 2
    nf_mult = 1
    for n in range(1, n_layers):
        nf_prev, nf_mult = nf_mult, min(2 ** n, 8)
        layers.append(dict(kind="conv", name=f"model.{idx}", cin=ndf * nf_prev, cout=ndf * nf_mult, k=4, s=2,
                           p=1, prepad=0, bias=True, norm=f"model.{idx+1}", act="lrelu"))
        idx += 3
    nf_prev, nf_mult = nf_mult, min(2 ** n_layers, 8)
    layers.append(dict(kind="conv", name=f"model.{idx}", cin=ndf * nf_prev, cout=ndf * nf_mult, k=4, s=1, p=1,
                       prepad=0, bias=True, norm=f"model.{idx+1}", act="lrelu"))
    idx += 3
    layers.append(dict(kind="conv", name=f"model.{idx}", cin=ndf * nf_mult, cout=1, k=4, s=1, p=1, prepad=0,
                       bias=True, norm=None, act="sigmoid" if use_sigmoid else None))
    return layers


# --------------------------------------------------------------------------------------
# Deterministic init — consumes the global torch RNG exactly like the reference
# --------------------------------------------------------------------------------------

def _conv_param_shapes(layer: dict) -> List[Tuple[str, tuple, int]]:
    """(prefix, weight shape, fan_in for bias bound) for each conv of a layer entry."""
    if layer["kind"] == "resblock":
        d = layer["dim"]
        w = (d, d, 3, 3, 3)
        return [(layer["conv1"], w), (layer["conv2"], w)]
    k = layer["k"]
    if layer["kind"] == "convT":     # ConvTranspose3d weight is [Cin, Cout, k, k, k]
        return [(layer["name"], (layer["cin"], layer["cout"], k, k, k))]
    return [(layer["name"], (layer["cout"], layer["cin"], k, k, k))]


def _norm_entries(layer: dict) -> List[Tuple[str, int]]:
    if layer["kind"] == "resblock":
        return [(layer["norm1"], layer["dim"]), (layer["norm2"], layer["dim"])]
    if layer.get("norm"):
        return [(layer["norm"], layer["cout"])]
    return []


def init_net_state(layers: List[dict], init_gain: float = 0.02, dtype=torch.float32) -> "OrderedDict[str, torch.Tensor]":
    """Build the state_dict of a net.  RNG consumption mirrors:
    (1) nn.Conv3d / nn.ConvTranspose3d constructors (kaiming_uniform_(a=√5) on the weight,
        uniform_ on the bias) in module-construction order, then
    (2) init_weights (networks3D.py:44-65): normal_(0, gain) on every conv weight, bias = 0,
        in net.apply order (= module order for these nets)."""
    state: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    convs = []
    for layer in layers:
        for prefix, wshape in _conv_param_shapes(layer):
            w = torch.empty(wshape, dtype=torch.float32)
            init.kaiming_uniform_(w, a=math.sqrt(5))
            b = torch.empty(wshape[0] if layer["kind"] != "convT" else wshape[1], dtype=torch.float32)
            fan_in, _ = init._calculate_fan_in_and_fan_out(w)
            bound = 1.0 / math.sqrt(fan_in)
            init.uniform_(b, -bound, bound)
            convs.append((prefix, w, b))
    for prefix, w, b in convs:
        init.normal_(w, 0.0, init_gain)
        b.zero_()
    # assemble in state_dict order (module order; norms interleaved after their conv)
    conv_map = {p: (w, b) for p, w, b in convs}
    for layer in layers:
        if layer["kind"] == "resblock":
            order = [("conv", layer["conv1"]), ("norm", layer["norm1"]), ("conv", layer["conv2"]), ("norm", layer["norm2"])]
            dims = {layer["norm1"]: layer["dim"], layer["norm2"]: layer["dim"]}
        else:
            order = [("conv", layer["name"])]
            if layer.get("norm"):
                order.append(("norm", layer["norm"]))
            dims = {layer.get("norm"): layer["cout"]}
        for kind, prefix in order:
            if kind == "conv":
                w, b = conv_map[prefix]
                state[prefix + ".weight"] = w.to(dtype)
                state[prefix + ".bias"] = b.to(dtype)
            else:
                c = dims[prefix]
                state[prefix + ".running_mean"] = torch.zeros(c, dtype=dtype)
                state[prefix + ".running_var"] = torch.ones(c, dtype=dtype)
                state[prefix + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return state


# --------------------------------------------------------------------------------------
# Ops (explicit restatements of the ATen semantics the reference relies on)
# --------------------------------------------------------------------------------------

def instance_norm_train(x: torch.Tensor, state: dict, prefix: str) -> torch.Tensor:
    """nn.InstanceNorm3d(affine=False, track_running_stats=True) in train mode
    (networks3D.py:19).  y = (x − μ_nc)/√(σ²_nc,biased + eps).  Running stats:
    r ← (1−m)·r + m·mean_n(stat_n) with the UNBIASED variance; num_batches_tracked is
    left at 0 (InstanceNorm never increments it)."""
    n = x.shape[2] * x.shape[3] * x.shape[4]
    if n <= 1:
        raise ValueError(f"Expected more than 1 spatial element when training, got input size {list(x.shape)}")
    dims = (2, 3, 4)
    mean = x.mean(dim=dims, keepdim=True)
    var = ((x - mean) ** 2).mean(dim=dims, keepdim=True)
    y = (x - mean) / torch.sqrt(var + IN_EPS)
    with torch.no_grad():
        rm = state[prefix + ".running_mean"]
        rv = state[prefix + ".running_var"]
        bmean = mean.detach().reshape(x.shape[0], x.shape[1]).to(rm.dtype).mean(0)
        bvar_unb = (var.detach() * (n / (n - 1))).reshape(x.shape[0], x.shape[1]).to(rv.dtype).mean(0)
        rm.mul_(1 - IN_MOMENTUM).add_(IN_MOMENTUM * bmean)
        rv.mul_(1 - IN_MOMENTUM).add_(IN_MOMENTUM * bvar_unb)
    return y


def _act(x, act):
    if act == "relu":
        return F.relu(x)
    if act == "lrelu":
        return F.leaky_relu(x, LRELU_SLOPE)
    if act == "tanh":
        return torch.tanh(x)
    if act == "sigmoid":
        return torch.sigmoid(x)
    return x


def _rpad(x, p):
    return F.pad(x, (p,) * 6, mode="replicate") if p else x   # nn.ReplicationPad3d(p)


# --------------------------------------------------------------------------------------
# Convolution arithmetic: exact (the reference's ATen convs), or with the operands rounded to
# bf16 / fp16 where the engine's 16-bit contraction modes round them
# --------------------------------------------------------------------------------------

class ExactConv:
    """The reference's convolutions (nn.Conv3d / nn.ConvTranspose3d → ATen) in the oracle's dtype."""

    def conv3d(self, x, w, b=None, stride=1, padding=0):
        return F.conv3d(x, w, b, stride=stride, padding=padding)

    def conv_transpose3d(self, x, w, b=None, stride=1, padding=0, output_padding=0):
        return F.conv_transpose3d(x, w, b, stride=stride, padding=padding, output_padding=output_padding)


EXACT = ExactConv()


class RoundedConv:
    """The reference's convolutions with every operand rounded the way the engine's bf16 / fp16
    contraction modes round it (include/mragan_hip.h, ABI 10 — every convolution, every kernel):

      forward          y  = conv(R(x), R(W)) + b              (bias added unrounded, fp32 epilogue)
      data gradient    dx = conv_input(R(dY), R(W))
      weight gradient  dW = conv_weight(R(X), R(dY));  db = Σ dY  (unrounded, channel_sum)

    R rounds the fp32 value (the engine's tensors are fp32; an fp64 oracle value is first rounded
    to fp32) to bf16 or fp16, round-to-nearest-even, as v_cvt_pk_bf16_f32 / v_cvt_f16_f32 and the
    MFMA fragment conversion do.  Gradients enter the engine's backward multiplied by the static
    loss scale (mragan_set_loss_scale), so a gradient operand is R(s·dY)/s — an exact power-of-two
    rescaling except where fp16's range clips.  The products and sums are then evaluated in the
    oracle's dtype (fp64: "emulated", no accumulation error; fp32: the calibration twin)."""

    def __init__(self, mode: str, loss_scale: float = 1.0):
        if mode not in ("bf16", "fp16", "bf16x3"):
            raise ValueError(f"operand rounding must be 'bf16', 'fp16' or 'bf16x3', got {mode!r}")
        self.mode = mode
        self.dt = torch.float16 if mode == "fp16" else torch.bfloat16
        self.scale = float(loss_scale)

    # ---- bf16x3 (the engine's fp32-grade split mode, csrc/prec.h kPrecBf16x3) -------------------
    # Each fp32 operand v splits into hi = bf16(v), lo = bf16(v − hi) (RNE; v − hi is exact in
    # fp32) and a product a·b is a_hi·b_hi + a_hi·b_lo + a_lo·b_hi — lo·lo dropped — accumulated in
    # fp32 (three v_mfma_f32_32x32x16_bf16).  By linearity one bilinear op f (a convolution, its
    # data or weight gradient) is then f(a_hi, b_hi + b_lo) + f(a_lo, b_hi): in fp64 both terms are
    # exact sums of exact products.  Only the MFMA kernels split: the thin VALU kernels and the
    # fp32 implicit-GEMM / weight-gradient fallbacks compute exact fp32 products in this mode
    # (common.h op_round keeps the value), so each convolution takes the path the C ABI would
    # dispatch it to (capi.hip conv_common / mragan_conv3d_wgrad, conv_igemm.hip, conv_wgrad.hip).
    def split(self, t: torch.Tensor):
        f = t.detach().float()
        hi = f.to(torch.bfloat16)
        lo = (f - hi.float()).to(torch.bfloat16)
        return hi.to(t.dtype), lo.to(t.dtype)

    def x3(self, f, a, b):
        ah, al = self.split(a)
        bh, bl = self.split(b)
        return f(ah, bh + bl) + f(al, bh)

    @staticmethod
    def conv_splits(cx, ny, k, s):
        """Does conv_common (a forward- or transposed-form launch: cx input channels, ny output
        channels) run an MFMA (split) kernel?  thin_side → the 1-channel k7 MFMA kernels (thin1_x3,
        thinn_x3) or the VALU thin kernels; else the implicit-GEMM family, whose MFMA paths (brick,
        brickT, conv_igemm_x3) need cx % 16 == 0 and whose fp32 tiles take the rest."""
        if cx <= 4 or ny <= 4 or cx % 8:
            return k == 7 and s == 1 and ((cx == 1 and ny == 32) or (cx == 32 and ny == 1))
        return cx % 16 == 0

    @staticmethod
    def wgrad_splits(cd, cg, k, s):
        """Does mragan_conv3d_wgrad (dense cd channels, gathered cg) run an MFMA kernel?  thin side:
        only thin1_wgrad_x3 (k7, 32 ↔ 1 channels); else wgrad3 / wgrad3s2 / conv_wgrad_x3, all of
        which need multiples of 32 channels on both sides (the fp32 kernel takes the rest)."""
        if cd < 8 or cg < 8:
            return k == 7 and s == 1 and ((cd == 32 and cg == 1) or (cd == 1 and cg == 32))
        return cd % 32 == 0 and cg % 32 == 0

    def op(self, t: torch.Tensor) -> torch.Tensor:
        return t.detach().float().to(self.dt).to(t.dtype)

    def grad(self, g: torch.Tensor) -> torch.Tensor:
        if self.scale == 1.0:
            return self.op(g)
        return (g.detach().float() * self.scale).to(self.dt).to(g.dtype) / self.scale

    def conv3d(self, x, w, b=None, stride=1, padding=0):
        return _RoundedConvFn.apply(x, w, b, self, False, stride, padding, 0)

    def conv_transpose3d(self, x, w, b=None, stride=1, padding=0, output_padding=0):
        return _RoundedConvFn.apply(x, w, b, self, True, stride, padding, output_padding)


class _RoundedConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, rnd, transposed, stride, padding, output_padding):
        if rnd.mode == "bf16x3":
            return _X3ConvFn.forward(ctx, x, w, b, rnd, transposed, stride, padding, output_padding)
        xr, wr = rnd.op(x), rnd.op(w)
        ctx.save_for_backward(xr, wr)
        ctx.cfg = (rnd, transposed, stride, padding, output_padding, b is not None)
        y = _conv_any(xr, wr, transposed, stride, padding, output_padding)
        return y + b.view(1, -1, 1, 1, 1) if b is not None else y

    @staticmethod
    def backward(ctx, gy):
        if ctx.cfg[0].mode == "bf16x3":
            return _X3ConvFn.backward(ctx, gy)
        xr, wr = ctx.saved_tensors
        rnd, transposed, stride, padding, output_padding, has_b = ctx.cfg
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        gx = gw = gb = None
        if need_x or need_w:
            with torch.enable_grad():
                xl = xr.detach().requires_grad_(need_x)
                wl = wr.detach().requires_grad_(need_w)
                y = _conv_any(xl, wl, transposed, stride, padding, output_padding)
                want = [t for t, n in ((xl, need_x), (wl, need_w)) if n]
                got = list(torch.autograd.grad(y, want, rnd.grad(gy)))
            gx = got.pop(0) if need_x else None
            gw = got.pop(0) if need_w else None
        if has_b and ctx.needs_input_grad[2]:
            gb = gy.sum(dim=(0, 2, 3, 4))
        return gx, gw, gb, None, None, None, None, None


class _X3ConvFn:
    """The bf16x3 mode's convolution (RoundedConv.x3): forward, data gradient and weight gradient
    each split or exact as the engine dispatches it.  Shapes seen by the kernels: a Conv3d layer
    (w [cout][cin]) runs its forward as conv_common(cx = cin, ny = cout), its data gradient in the
    transposed form with (cx = cout, ny = cin) and its weight gradient with dense = dY (cout),
    gathered = X (cin); a ConvTranspose3d layer (w [cin][cout]) the mirror image, with dense = X
    (cin), gathered = dY (cout) (mragan_hip/engine.py Conv.dgrad / Conv.wgrad)."""

    @staticmethod
    def forward(ctx, x, w, b, rnd, transposed, stride, padding, output_padding):
        ctx.save_for_backward(x, w)
        ctx.cfg = (rnd, transposed, stride, padding, output_padding, b is not None)
        k = w.shape[-1]
        cin, cout = (w.shape[0], w.shape[1]) if transposed else (w.shape[1], w.shape[0])
        f = lambda a, c: _conv_any(a, c, transposed, stride, padding, output_padding)   # noqa: E731
        y = rnd.x3(f, x, w) if rnd.conv_splits(cin, cout, k, stride) else f(x, w)
        return y + b.view(1, -1, 1, 1, 1) if b is not None else y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        rnd, transposed, stride, padding, output_padding, has_b = ctx.cfg
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        k = w.shape[-1]
        cin, cout = (w.shape[0], w.shape[1]) if transposed else (w.shape[1], w.shape[0])

        def vjp(xa, wa, ga, wrt):
            with torch.enable_grad():
                xl = xa.detach().requires_grad_(wrt == "x")
                wl = wa.detach().requires_grad_(wrt == "w")
                y = _conv_any(xl, wl, transposed, stride, padding, output_padding)
                return torch.autograd.grad(y, xl if wrt == "x" else wl, ga)[0]

        gx = gw = gb = None
        if need_x:
            dgrad = lambda g, c: vjp(x, c, g, "x")                                       # noqa: E731
            gx = rnd.x3(dgrad, gy, w) if rnd.conv_splits(cout, cin, k, stride) else dgrad(gy, w)
        if need_w:
            wgrad = lambda a, g: vjp(a, w, g, "w")                                       # noqa: E731
            dense, gathered = (cin, cout) if transposed else (cout, cin)
            gw = rnd.x3(wgrad, x, gy) if rnd.wgrad_splits(dense, gathered, k, stride) else wgrad(x, gy)
        if has_b and ctx.needs_input_grad[2]:
            gb = gy.sum(dim=(0, 2, 3, 4))
        return gx, gw, gb, None, None, None, None, None


def _conv_any(x, w, transposed, stride, padding, output_padding):
    if transposed:
        return F.conv_transpose3d(x, w, None, stride=stride, padding=padding, output_padding=output_padding)
    return F.conv3d(x, w, None, stride=stride, padding=padding)


def generator_forward(state: dict, params: dict, layers: List[dict], x: torch.Tensor, conv=EXACT) -> torch.Tensor:
    """ResnetGenerator.forward (networks3D.py:219-220): the Sequential of layers."""
    h = x
    for L in layers:
        if L["kind"] == "conv":
            h = conv.conv3d(_rpad(h, L["prepad"]), params[L["name"] + ".weight"], params[L["name"] + ".bias"],
                            stride=L["s"], padding=L["p"])
            if L["norm"]:
                h = instance_norm_train(h, state, L["norm"])
            h = _act(h, L["act"])
        elif L["kind"] == "convT":
            h = conv.conv_transpose3d(h, params[L["name"] + ".weight"], params[L["name"] + ".bias"],
                                      stride=L["s"], padding=L["p"], output_padding=L["op"])
            h = instance_norm_train(h, state, L["norm"])
            h = _act(h, L["act"])
        else:  # ResnetBlock.forward: x + conv_block(x)   networks3D.py:261-263
            r = conv.conv3d(_rpad(h, 1), params[L["conv1"] + ".weight"], params[L["conv1"] + ".bias"])
            r = F.relu(instance_norm_train(r, state, L["norm1"]))
            r = conv.conv3d(_rpad(r, 1), params[L["conv2"] + ".weight"], params[L["conv2"] + ".bias"])
            r = instance_norm_train(r, state, L["norm2"])
            h = h + r
    return h


discriminator_forward = generator_forward   # same Sequential walk (networks3D.py:424-425)


def gan_loss(pred: torch.Tensor, target_is_real: bool, use_lsgan: bool) -> torch.Tensor:
    """GANLoss.__call__ (networks3D.py:130-150): MSELoss (lsgan) or BCELoss vs a constant
    target of 1/0.  BCELoss clamps each log at −100 (ATen binary_cross_entropy)."""
    t = 1.0 if target_is_real else 0.0
    if use_lsgan:
        return ((pred - t) ** 2).mean()
    return F.binary_cross_entropy(pred, torch.full_like(pred, t))


def l1_loss(a, b):
    return (a - b).abs().mean()      # nn.L1Loss (cycle_gan_model.py:104-105)


def cor_coe_loss(y_pred, y_target):
    """Cor_CoeLoss (networks3D.py:156-166): 1 − r²; computed but unused by loss_G."""
    xv = y_pred - y_pred.mean()
    yv = y_target - y_target.mean()
    r = (xv * yv).sum() / (torch.sqrt((xv ** 2).sum()) * torch.sqrt((yv ** 2).sum()))
    return 1 - r ** 2


class ImagePool:
    """ImagePool (cycle_gan_model.py:8-35).  Uses the Python `random` module."""

    def __init__(self, pool_size: int, rng: random.Random = None):
        self.pool_size = pool_size
        self.rng = rng if rng is not None else random
        self.num_imgs = 0
        self.images: List[torch.Tensor] = []

    def query(self, images: torch.Tensor) -> torch.Tensor:
        if self.pool_size == 0:
            return images
        out = []
        for image in images:
            image = image.detach().unsqueeze(0)
            if self.num_imgs < self.pool_size:
                self.num_imgs += 1
                self.images.append(image)
                out.append(image)
            else:
                if self.rng.uniform(0, 1) > 0.5:
                    rid = self.rng.randint(0, self.pool_size - 1)
                    tmp = self.images[rid].clone()
                    self.images[rid] = image
                    out.append(tmp)
                else:
                    out.append(image)
        return torch.cat(out, 0)


def adam_update(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
                lr: float, beta1: float, beta2: float = 0.999, eps: float = 1e-8) -> None:
    """torch.optim.Adam single-tensor update (amsgrad=False, weight_decay=0), as used by
    cycle_gan_model.py:107-110.  m uses lerp (torch's exact form)."""
    m.lerp_(g, 1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-step_size)


# --------------------------------------------------------------------------------------
# UnetGenerator (networks3D.py:270-343) — --netG unet_custom / unet_256
# --------------------------------------------------------------------------------------

def unet_generator_levels(input_nc: int, output_nc: int, ngf: int, num_downs: int) -> dict:
    """UnetSkipConnectionBlocks outermost → innermost (networks3D.py:276-287) with their
    state_dict prefixes.  Sequential indices (networks3D.py:316-338): outermost
    [down 0, sub 1, uprelu 2, up 3, tanh 4]; middle [downrelu 0, down 1, downnorm 2, sub 3,
    uprelu 4, up 5, upnorm 6]; innermost [downrelu 0, down 1, uprelu 2, up 3, upnorm 4]."""
    chans = [(output_nc, ngf, input_nc), (ngf, 2 * ngf, ngf), (2 * ngf, 4 * ngf, 2 * ngf), (4 * ngf, 8 * ngf, 4 * ngf)]
    chans += [(8 * ngf, 8 * ngf, 8 * ngf)] * (num_downs - 5)
    chans += [(8 * ngf, 8 * ngf, 8 * ngf)]
    levels = []
    prefix = "model"
    for i, (outer, inner, cin) in enumerate(chans):
        kind = "outer" if i == 0 else ("inner" if i == len(chans) - 1 else "mid")
        p = prefix + ".model"
        idx = {"outer": (0, None, 1, 3, None), "mid": (1, 2, 3, 5, 6), "inner": (1, None, None, 3, 4)}[kind]
        down, dnorm, sub, up, unorm = idx
        levels.append(dict(kind=kind, down=f"{p}.{down}", up=f"{p}.{up}",
                           dnorm=f"{p}.{dnorm}" if dnorm is not None else None,
                           unorm=f"{p}.{unorm}" if unorm is not None else None,
                           cin=cin, inner=inner, outer=outer, up_cin=inner if kind == "inner" else 2 * inner,
                           up_bias=kind == "outer"))
        prefix = f"{p}.{sub}"
    return dict(kind="unet", levels=levels)


def init_unet_state(spec: dict, init_gain: float = 0.02, dtype=torch.float32) -> "OrderedDict[str, torch.Tensor]":
    """RNG consumption of UnetGenerator construction + init_weights: the blocks are built
    innermost first, each drawing kaiming_uniform_ for its downconv then its upconv (+ bias for
    the outermost upconv, the only conv with a bias: use_bias compares against
    nn.InstanceNorm2d, networks3D.py:302-305); init_weights then redraws normal_(0, gain) in
    net.apply order = the downconvs outer → inner, then the upconvs inner → outer."""
    levels = spec["levels"]
    w = {}
    for lv in reversed(levels):
        wd = torch.empty((lv["inner"], lv["cin"], 4, 4, 4), dtype=torch.float32)
        init.kaiming_uniform_(wd, a=math.sqrt(5))
        wu = torch.empty((lv["up_cin"], lv["outer"], 4, 4, 4), dtype=torch.float32)
        init.kaiming_uniform_(wu, a=math.sqrt(5))
        w[lv["down"]] = [wd, None]
        w[lv["up"]] = [wu, None]
        if lv["up_bias"]:
            b = torch.empty(lv["outer"], dtype=torch.float32)
            fan_in, _ = init._calculate_fan_in_and_fan_out(wu)
            init.uniform_(b, -1.0 / math.sqrt(fan_in), 1.0 / math.sqrt(fan_in))
            w[lv["up"]][1] = b
    for key in [lv["down"] for lv in levels] + [lv["up"] for lv in reversed(levels)]:
        init.normal_(w[key][0], 0.0, init_gain)
        if w[key][1] is not None:
            w[key][1].zero_()
    state: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for key in sorted(w):
        state[key + ".weight"] = w[key][0].to(dtype)
        if w[key][1] is not None:
            state[key + ".bias"] = w[key][1].to(dtype)
    for lv in levels:
        for nk, c in ((lv["dnorm"], lv["inner"]), (lv["unorm"], lv["outer"])):
            if nk:
                state[nk + ".running_mean"] = torch.zeros(c, dtype=dtype)
                state[nk + ".running_var"] = torch.ones(c, dtype=dtype)
                state[nk + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return state


def unet_forward(state: dict, params: dict, spec: dict, x: torch.Tensor, conv=EXACT) -> torch.Tensor:
    """UnetGenerator.forward with the reference's in-place activations made explicit: a
    non-outermost block's `downrelu` (inplace) rewrites its input, so the skip half of
    torch.cat([x, model(x)], 1) is LeakyReLU(x) (networks3D.py:340-343)."""
    levels = spec["levels"]

    def block(i, h):
        lv = levels[i]
        wd, wu = params[lv["down"] + ".weight"], params[lv["up"] + ".weight"]
        if lv["kind"] == "outer":
            s = block(i + 1, conv.conv3d(h, wd, None, stride=2, padding=1))
            y = conv.conv_transpose3d(F.relu(s), wu, params[lv["up"] + ".bias"], stride=2, padding=1)
            return torch.tanh(y)
        a = F.leaky_relu(h, LRELU_SLOPE)
        d = conv.conv3d(a, wd, None, stride=2, padding=1)
        if lv["kind"] == "mid":
            r = F.relu(block(i + 1, instance_norm_train(d, state, lv["dnorm"])))
        else:
            r = F.relu(d)
        u = instance_norm_train(conv.conv_transpose3d(r, wu, None, stride=2, padding=1), state, lv["unorm"])
        return torch.cat([a, u], 1)

    return block(0, x)


# --------------------------------------------------------------------------------------
# The step
# --------------------------------------------------------------------------------------

class CycleGANOracle:
    """Functional restatement of CycleGANModel (cycle_gan_model.py:38-240) on CPU."""

    LOSS_NAMES = ['D_A', 'G_A', 'cycle_A', 'idt_A', 'D_B', 'G_B', 'cycle_B', 'idt_B']  # :68

    def __init__(self, input_nc=1, output_nc=1, ngf=32, ndf=32, n_blocks=9, n_layers_D=3, netG=None,
                 use_lsgan=False, lambda_A=10.0, lambda_B=10.0, lambda_identity=0.5,
                 lr=2e-4, beta1=0.5, pool_size=50, init_gain=0.02, dtype=torch.float32,
                 states: Dict[str, dict] = None, pool_rng: random.Random = None,
                 operand_rounding: str = None, loss_scale: float = 1.0):
        """operand_rounding: None (the reference's arithmetic) or 'bf16' / 'fp16' — every
        convolution operand rounded as the engine's 16-bit contraction modes round it
        (RoundedConv), fp16 gradients under the static `loss_scale` — or 'bf16x3', the split-bf16
        products of the engine's fp32-grade MFMA mode where its MFMA kernels run (RoundedConv.x3)."""
        self.dtype = dtype
        self.conv = EXACT if operand_rounding is None else RoundedConv(operand_rounding, loss_scale)
        self.use_lsgan = use_lsgan
        self.lambda_A, self.lambda_B, self.lambda_idt = lambda_A, lambda_B, lambda_identity
        self.lr, self.beta1 = lr, beta1
        if netG in ("unet_custom", "unet_256"):      # define_G, networks3D.py:84-102
            nd = 5 if netG == "unet_custom" else 8
            gA = unet_generator_levels(input_nc, output_nc, ngf, nd)
            gB = unet_generator_levels(output_nc, input_nc, ngf, nd)
        else:
            if netG is not None:
                n_blocks = {"resnet_9blocks": 9, "resnet_6blocks": 6}[netG]
            gA = resnet_generator_layers(input_nc, output_nc, ngf, n_blocks)
            gB = resnet_generator_layers(output_nc, input_nc, ngf, n_blocks)
        self.layers = {
            "G_A": gA,
            "G_B": gB,
            "D_A": nlayer_discriminator_layers(output_nc, ndf, n_layers_D, not use_lsgan),
            "D_B": nlayer_discriminator_layers(input_nc, ndf, n_layers_D, not use_lsgan),
        }
        if states is None:   # same construction order as CycleGANModel.initialize (:83-96)
            states = {k: (init_unet_state(self.layers[k], init_gain) if isinstance(self.layers[k], dict)
                          else init_net_state(self.layers[k], init_gain)) for k in ("G_A", "G_B", "D_A", "D_B")}
        self.state = {k: OrderedDict((n, t.clone().to(dtype) if t.is_floating_point() else t.clone())
                                     for n, t in v.items()) for k, v in states.items()}
        self.params = {k: OrderedDict((n, t) for n, t in self.state[k].items()
                                      if n.endswith(".weight") or n.endswith(".bias")) for k in self.state}
        self.adam = {k: {n: (torch.zeros_like(t), torch.zeros_like(t)) for n, t in self.params[k].items()}
                     for k in self.params}
        self.step_count = {"G": 0, "D": 0}
        self.fake_A_pool = ImagePool(pool_size, pool_rng)
        self.fake_B_pool = ImagePool(pool_size, pool_rng)
        self.grads: Dict[str, Dict[str, torch.Tensor]] = {}

    # --- helpers -------------------------------------------------------------------
    def _net(self, name, x, params):
        spec = self.layers[name]
        if isinstance(spec, dict):
            return unet_forward(self.state[name], params, spec, x, self.conv)
        return generator_forward(self.state[name], params, spec, x, self.conv)

    def _leaf_params(self, names, requires_grad):
        out = {}
        for k in names:
            out[k] = {n: t.detach().clone().requires_grad_(requires_grad) for n, t in self.params[k].items()}
        return out

    def _adam(self, nets, leaf, group):
        self.step_count[group] += 1
        step = self.step_count[group]
        for k in nets:
            for n, p in self.params[k].items():
                g = leaf[k][n].grad
                if g is None:
                    continue
                m, v = self.adam[k][n]
                adam_update(p, g.detach(), m, v, step, self.lr, self.beta1)

    # --- optimize_parameters (cycle_gan_model.py:227-240) --------------------------
    def optimize_parameters(self, real_A: torch.Tensor, real_B: torch.Tensor) -> "OrderedDict[str, float]":
        real_A = real_A.to(self.dtype)
        real_B = real_B.to(self.dtype)
        self.real_A, self.real_B = real_A, real_B
        lp = self._leaf_params(["G_A", "G_B"], True)
        dp = self._leaf_params(["D_A", "D_B"], False)       # set_requires_grad(D, False) :231
        # forward (:121-136)
        fake_B = self._net("G_A", real_A, lp["G_A"])
        rec_A = self._net("G_B", fake_B, lp["G_B"])
        fake_A = self._net("G_B", real_B, lp["G_B"])
        rec_B = self._net("G_A", fake_A, lp["G_A"])
        # backward_G (:163-225); lambda_identity <= 0: no identity pass, losses 0 (:191-193)
        if self.lambda_idt > 0:
            idt_A = self._net("G_A", real_B, lp["G_A"])
            loss_idt_A = l1_loss(idt_A, real_B) * self.lambda_B * self.lambda_idt
            idt_B = self._net("G_B", real_A, lp["G_B"])
            loss_idt_B = l1_loss(idt_B, real_A) * self.lambda_A * self.lambda_idt
        else:
            idt_A = idt_B = None
            loss_idt_A = loss_idt_B = torch.zeros((), dtype=self.dtype)
        loss_G_A = gan_loss(self._net("D_A", fake_B, dp["D_A"]), True, self.use_lsgan)
        loss_G_B = gan_loss(self._net("D_B", fake_A, dp["D_B"]), True, self.use_lsgan)
        loss_cycle_A = l1_loss(rec_A, real_A) * self.lambda_A
        loss_cycle_B = l1_loss(rec_B, real_B) * self.lambda_B
        loss_G = loss_G_A + loss_G_B + loss_cycle_A + loss_cycle_B + loss_idt_A + loss_idt_B
        loss_G.backward()
        self.grads = {k: {n: t.grad.detach().clone() for n, t in lp[k].items()} for k in ("G_A", "G_B")}
        self._adam(["G_A", "G_B"], lp, "G")
        # D phase (:236-240)
        dp = self._leaf_params(["D_A", "D_B"], True)
        fB = self.fake_B_pool.query(fake_B.detach())
        loss_D_A = 0.5 * (gan_loss(self._net("D_A", real_B, dp["D_A"]), True, self.use_lsgan)
                          + gan_loss(self._net("D_A", fB, dp["D_A"]), False, self.use_lsgan))
        loss_D_A.backward()
        fA = self.fake_A_pool.query(fake_A.detach())
        loss_D_B = 0.5 * (gan_loss(self._net("D_B", real_A, dp["D_B"]), True, self.use_lsgan)
                          + gan_loss(self._net("D_B", fA, dp["D_B"]), False, self.use_lsgan))
        loss_D_B.backward()
        self.grads.update({k: {n: t.grad.detach().clone() for n, t in dp[k].items()} for k in ("D_A", "D_B")})
        self._adam(["D_A", "D_B"], dp, "D")
        self.fake_B, self.rec_A, self.fake_A, self.rec_B = (t.detach() for t in (fake_B, rec_A, fake_A, rec_B))
        self.idt_A = idt_A.detach() if idt_A is not None else None
        self.idt_B = idt_B.detach() if idt_B is not None else None
        vals = dict(D_A=loss_D_A, G_A=loss_G_A, cycle_A=loss_cycle_A, idt_A=loss_idt_A,
                    D_B=loss_D_B, G_B=loss_G_B, cycle_B=loss_cycle_B, idt_B=loss_idt_B)
        return OrderedDict((k, float(vals[k].detach())) for k in self.LOSS_NAMES)


def synthetic_pair(shape, seed: int):
    """Synthetic inputs: A then B ~ N(0,1) fp32 from torch.Generator(seed)."""
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(shape, generator=g)
    b = torch.randn(shape, generator=g)
    return a, b


# ------------------------------------------------------------------------------------------
# Sliding-window inference (reference test.py:38-207, the array part: lines 96-186)
# ------------------------------------------------------------------------------------------

def sliding_window_starts(shape, patch, stride_inplane, stride_layer):
    """test.py:111-143: the patch start corners in the order the reference visits them
    (i over x, then j over y, then k over z; the last patch of an axis is clamped to the end)."""
    import math as _m
    px, py, pz = patch
    inum = int(_m.ceil((shape[0] - px) / float(stride_inplane))) + 1
    jnum = int(_m.ceil((shape[1] - py) / float(stride_inplane))) + 1
    knum = int(_m.ceil((shape[2] - pz) / float(stride_layer))) + 1
    out = []
    for i in range(inum):
        for j in range(jnum):
            for k in range(knum):
                istart = i * stride_inplane
                if istart + px > shape[0]:
                    istart = shape[0] - px
                jstart = j * stride_inplane
                if jstart + py > shape[1]:
                    jstart = shape[1] - py
                kstart = k * stride_layer
                if kstart + pz > shape[2]:
                    kstart = shape[2] - pz
                out.append((istart, jstart, kstart))
    return out


def sliding_window_inference(g_forward, image_np, patch, stride_inplane, stride_layer):
    """test.py:96-186 on an already normalised (0-255, Normalization :639-651), resampled and
    padded volume `image_np` [x, y, z] float32.  `g_forward(batch [1,1,px,py,pz] float32 tensor)`
    returns fake_B.  Returns the label volume [x, y, z] float32 (before the final un-padding
    crop of :180, which the caller applies with its pre-padding size)."""
    import numpy as np
    image_np = np.asarray(image_np, dtype=np.float32)
    label_np = np.zeros(image_np.shape, dtype=np.float32)
    padding = image_np.shape[2] % 2 != 0                                     # :101-108
    if padding:
        image_np = np.pad(image_np, ((0, 0), (0, 0), (0, 1)), 'edge')
        label_np = np.pad(label_np, ((0, 0), (0, 0), (0, 1)), 'edge')
    weight_np = np.zeros(label_np.shape)                                     # :113 (float64)
    px, py, pz = patch
    for (i0, j0, k0) in sliding_window_starts(image_np.shape, patch, stride_inplane, stride_layer):
        batch = image_np[i0:i0 + px, j0:j0 + py, k0:k0 + pz][np.newaxis]     # prepare_batch, bs 1
        batch = (batch - 127.5) / 127.5                                      # :150
        x = torch.from_numpy(batch[np.newaxis, :, :, :])                     # [1, 1, px, py, pz]
        pred = g_forward(x)
        pred = pred.squeeze().detach().cpu().numpy().astype(np.float32)
        pred = (pred * 127.5) + 127.5                                        # :161
        label_np[i0:i0 + px, j0:j0 + py, k0:k0 + pz] += pred[:, :, :]
        weight_np[i0:i0 + px, j0:j0 + py, k0:k0 + pz] += 1.0
    label_np = (np.float32(label_np) / np.float32(weight_np) + 0.01)        # :173
    if padding:
        label_np = label_np[:, :, 0:(label_np.shape[2] - 1)]
    return label_np


# ------------------------------------------------------------------------------------------
# Training patch sampling (reference train.py:35-52, MONAI transforms — third-party, unpinned and
# absent here: restated from MONAI's published algorithm; "parity unpinned" beyond this restatement)
# ------------------------------------------------------------------------------------------

def monai_normalize_intensity(img):
    """NormalizeIntensityd(keys=['image'], channel_wise=True): (x − mean) / std, np.std (ddof 0),
    a zero std treated as 1."""
    import numpy as np
    x = np.asarray(img, dtype=np.float32)
    mean = x.mean()
    std = x.std()
    if std == 0:
        std = 1.0
    return ((x - mean) / std).astype(np.float32)


def monai_crop_foreground(img, label):
    """CropForegroundd(keys=['image','label'], source_key='image'), select_fn x > 0, margin 0."""
    import numpy as np
    coords = np.argwhere(img > 0)
    if coords.size == 0:
        return img, label
    lo = coords.min(0)
    hi = coords.max(0) + 1
    return img[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]], label[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]]


def monai_pos_neg_crops(image, label, spatial_size, num_samples, rand_state, pos=20, neg=0):
    """RandCropByPosNegLabeld(label_key='label', spatial_size, pos, neg, num_samples): the crops of
    one volume, each (image_patch, label_patch), drawn from rand_state (np.random.RandomState)."""
    import numpy as np
    shape = label.shape
    fg = [i for i, v in enumerate(label.reshape(-1)) if v != 0]
    bg = [i for i, v in enumerate(label.reshape(-1)) if v == 0] if neg > 0 else []
    ratio = pos / float(pos + neg)
    if not fg and not bg:
        raise ValueError("No sampling location available.")
    if not fg or not bg:
        ratio = 0 if not fg else 1
    half = [s // 2 for s in spatial_size]
    end = [int(np.uint16(shape[i] + 1 - spatial_size[i] / 2.0)) for i in range(3)]
    end = [e + 1 if e == h else e for e, h in zip(end, half)]
    out = []
    for _ in range(num_samples):
        use = fg if rand_state.rand() < ratio else bg
        flat = use[rand_state.randint(len(use))]
        c = [flat // (shape[1] * shape[2]), (flat // shape[2]) % shape[1], flat % shape[2]]
        c = [min(max(c[i], half[i]), end[i] - 1) for i in range(3)]
        s0 = [c[i] - half[i] for i in range(3)]
        sl = tuple(slice(s0[i], s0[i] + spatial_size[i]) for i in range(3))
        out.append((image[sl], label[sl]))
    return out
