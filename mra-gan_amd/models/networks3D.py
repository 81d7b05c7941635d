"""Network library — drop-in for the reference's models/networks3D.py.

Same public names and signatures (get_norm_layer, get_scheduler, init_weights, init_net,
define_G, define_D, GANLoss, Cor_CoeLoss, ResnetGenerator, ResnetBlock, NLayerDiscriminator),
the same module tree and therefore the same state_dict keys (`model.1.weight`,
`model.10.conv_block.1.weight`, ...), and the same parameter-init RNG consumption, so a given
`torch.manual_seed` produces bit-identical initial weights to the reference's CPU path.

What differs is execution: the layer classes here are parameter containers; a network's
forward runs the whole network through the hand-written HIP kernels of
`mragan_hip` (NDHWC fp32, fused InstanceNorm/activation/padding), with a hand-written
backward registered as one autograd node.  There is no CPU / eager-PyTorch fallback.
"""
from __future__ import annotations

import functools
import math

import torch
import torch.nn as nn
from torch.nn import init
from torch.optim import lr_scheduler

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")   # reference networks3D.py:8


# =======================================================================================
# Layer containers (parameters + hyper-parameters; executed by the network engine)
# =======================================================================================

class _EngineOnly(nn.Module):
    def forward(self, *args, **kwargs):
        raise NotImplementedError(
            f"{type(self).__name__} is executed as part of its network by the HIP engine; "
            "call the enclosing ResnetGenerator / NLayerDiscriminator instead")


class Conv3d(_EngineOnly):
    """nn.Conv3d hyper-parameters and parameters (weight [Cout, Cin, k, k, k]).  Construction
    consumes the RNG exactly like torch.nn.Conv3d.reset_parameters."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = int(kernel_size), int(stride), int(padding)
        k = self.kernel_size
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, k, k, k))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in, _ = init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            init.uniform_(self.bias, -bound, bound)

    def extra_repr(self):
        k = self.kernel_size
        return (f"{self.in_channels}, {self.out_channels}, kernel_size=({k}, {k}, {k}), "
                f"stride=({self.stride}, {self.stride}, {self.stride}), padding=({self.padding}, {self.padding}, "
                f"{self.padding}){'' if self.bias is not None else ', bias=False'}")


class ConvTranspose3d(_EngineOnly):
    """nn.ConvTranspose3d hyper-parameters and parameters (weight [Cin, Cout, k, k, k])."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = int(kernel_size), int(stride), int(padding)
        self.output_padding = int(output_padding)
        k = self.kernel_size
        self.weight = nn.Parameter(torch.empty(in_channels, out_channels, k, k, k))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in, _ = init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            init.uniform_(self.bias, -bound, bound)

    def extra_repr(self):
        k = self.kernel_size
        return (f"{self.in_channels}, {self.out_channels}, kernel_size=({k}, {k}, {k}), "
                f"stride=({self.stride}, {self.stride}, {self.stride}), padding=({self.padding}, {self.padding}, "
                f"{self.padding}), output_padding=({self.output_padding}, {self.output_padding}, "
                f"{self.output_padding})")


class InstanceNorm3d(_EngineOnly):
    """nn.InstanceNorm3d(affine=False, track_running_stats=True) buffers."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=False, track_running_stats=True):
        super().__init__()
        if affine:
            raise NotImplementedError("InstanceNorm3d(affine=True) is not used by the reference nets")
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.affine, self.track_running_stats = affine, track_running_stats
        if track_running_stats:
            self.register_buffer("running_mean", torch.zeros(num_features))
            self.register_buffer("running_var", torch.ones(num_features))
            self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        else:
            self.running_mean = self.running_var = self.num_batches_tracked = None

    def extra_repr(self):
        return (f"{self.num_features}, eps={self.eps}, momentum={self.momentum}, affine={self.affine}, "
                f"track_running_stats={self.track_running_stats}")

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        # like torch's _NormBase: a checkpoint without num_batches_tracked (the reference's
        # load_networks strips it, base_model.py:114-127) keeps the current counter
        key = prefix + "num_batches_tracked"
        if self.track_running_stats and key not in state_dict:
            state_dict[key] = self.num_batches_tracked.clone()
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


class ReplicationPad3d(_EngineOnly):
    def __init__(self, padding):
        super().__init__()
        self.padding = int(padding)

    def extra_repr(self):
        return f"({self.padding}, {self.padding}, {self.padding}, {self.padding}, {self.padding}, {self.padding})"


class ReLU(_EngineOnly):
    act_name = "relu"

    def __init__(self, inplace=False):
        super().__init__()
        self.inplace = inplace


class LeakyReLU(_EngineOnly):
    act_name = "lrelu"

    def __init__(self, negative_slope=0.01, inplace=False):
        super().__init__()
        if negative_slope != 0.2:
            raise NotImplementedError("only LeakyReLU(0.2) (networks3D.py:393) is supported")
        self.negative_slope, self.inplace = negative_slope, inplace


class Tanh(_EngineOnly):
    act_name = "tanh"


class Sigmoid(_EngineOnly):
    act_name = "sigmoid"


class Dropout(_EngineOnly):
    def __init__(self, p=0.5):
        super().__init__()
        self.p = p


# =======================================================================================
# Helper functions (reference networks3D.py:15-81)
# =======================================================================================

def get_norm_layer(norm_type='instance'):
    if norm_type == 'batch':
        raise NotImplementedError('normalization layer [batch] is not supported by the HIP engine '
                                  '(the reference nets are trained with --norm instance)')
    elif norm_type == 'instance':
        norm_layer = functools.partial(InstanceNorm3d, affine=False, track_running_stats=True)
    elif norm_type == 'none':
        norm_layer = None
    else:
        raise NotImplementedError('normalization layer [%s] is not found' % norm_type)
    return norm_layer


def get_scheduler(optimizer, opt):
    """Same policies as the reference (networks3D.py:27-41), including its quirk of *returning*
    NotImplementedError for an unknown policy."""
    if opt.lr_policy == 'lambda':
        def lambda_rule(epoch):
            lr_l = 1.0 - max(0, epoch + 1 + opt.epoch_count - opt.niter) / float(opt.niter_decay + 1)
            return lr_l
        scheduler = lr_scheduler.LambdaLR(optimizer, lr_lambda=lambda_rule)
    elif opt.lr_policy == 'step':
        scheduler = lr_scheduler.StepLR(optimizer, step_size=opt.lr_decay_iters, gamma=0.1)
    elif opt.lr_policy == 'plateau':
        scheduler = lr_scheduler.ReduceLROnPlateau(optimizer, mode='min', factor=0.2, threshold=0.01, patience=5)
    elif opt.lr_policy == 'cosine':
        scheduler = lr_scheduler.CosineAnnealingLR(optimizer, T_max=opt.niter, eta_min=0)
    else:
        return NotImplementedError('learning rate policy [%s] is not implemented', opt.lr_policy)
    return scheduler


def init_weights(net, init_type='normal', gain=0.02):
    def init_func(m):
        classname = m.__class__.__name__
        if hasattr(m, 'weight') and (classname.find('Conv') != -1 or classname.find('Linear') != -1):
            if init_type == 'normal':
                init.normal_(m.weight.data, 0.0, gain)
            elif init_type == 'xavier':
                init.xavier_normal_(m.weight.data, gain=gain)
            elif init_type == 'kaiming':
                init.kaiming_normal_(m.weight.data, a=0, mode='fan_in')
            elif init_type == 'orthogonal':
                init.orthogonal_(m.weight.data, gain=gain)
            else:
                raise NotImplementedError('initialization method [%s] is not implemented' % init_type)
            if hasattr(m, 'bias') and m.bias is not None:
                init.constant_(m.bias.data, 0.0)

    print('initialize network with %s' % init_type)
    net.apply(init_func)


def flatten_parameters(net: nn.Module):
    """Put every parameter of `net` in one contiguous fp32 buffer (and every gradient in a
    second one) so the optimizer is a single fused kernel.  Parameters stay nn.Parameter
    objects; only their storage moves."""
    params = list(net.parameters())
    dev = params[0].device
    total = sum(p.numel() for p in params)
    flat = torch.empty(total, device=dev, dtype=torch.float32)
    gflat = torch.zeros(total, device=dev, dtype=torch.float32)
    off = 0
    for p in params:
        n = p.numel()
        flat[off:off + n].copy_(p.data.reshape(-1))
        p.data = flat[off:off + n].view_as(p)
        p.grad = gflat[off:off + n].view_as(p)
        off += n
    net._flat_param = flat
    net._flat_grad = gflat
    net._flat_ptrs = [p.data_ptr() for p in params]
    net._grad_group = None
    return flat, gflat


def group_grads(nets):
    """One contiguous gradient buffer for several flattened networks — each net's `_flat_grad` (and
    its parameters' .grad views) a slice of it, in order — so the data-parallel exchange of an
    optimizer's networks is ONE all-reduce (G_A + G_B, D_A + D_B; mragan_hip/dist.py).  Returns the
    buffer; idempotent while the grouping holds, regroups (copying the current gradients) after a
    network was re-flattened."""
    buf = getattr(nets[0], "_grad_group", None)
    if buf is not None:
        off, ok = 0, True
        for n in nets:
            k = n._flat_grad.numel()
            ok = ok and getattr(n, "_grad_group", None) is buf and n._flat_grad.data_ptr() == buf[off:off + k].data_ptr()
            off += k
        if ok and off == buf.numel():
            return buf
    total = sum(n._flat_grad.numel() for n in nets)
    buf = torch.empty(total, device=nets[0]._flat_grad.device, dtype=torch.float32)
    off = 0
    for n in nets:
        k = n._flat_grad.numel()
        buf[off:off + k].copy_(n._flat_grad)
        n._flat_grad = buf[off:off + k]
        n._grad_group = buf
        o = 0
        for p in n.parameters():
            p.grad = n._flat_grad[o:o + p.numel()].view_as(p)
            o += p.numel()
        off += k
    return buf


def ensure_flat(net: nn.Module):
    """Re-flatten if a parameter was re-assigned (e.g. net.cpu()/.cuda() or load_state_dict
    replacing storage); re-link p.grad views if an optimizer set them to None."""
    params = list(net.parameters())
    if getattr(net, "_flat_ptrs", None) != [p.data_ptr() for p in params] or \
            net._flat_param.device != params[0].device:
        flatten_parameters(net)
        return True
    g = net._flat_grad
    off = 0
    for p in params:
        n = p.numel()
        if p.grad is None or p.grad.data_ptr() != g[off:off + n].data_ptr():
            if p.grad is not None:
                g[off:off + n].copy_(p.grad.reshape(-1))
            else:
                g[off:off + n].zero_()
            p.grad = g[off:off + n].view_as(p)
        off += n
    return False


def init_net(net, init_type='normal', init_gain=0.02, gpu_ids=[]):
    """Reference networks3D.py:68-81.  Weights are drawn on the CPU generator (the reference's
    CPU path; bit-identical for a given seed), then the net moves to the HIP device and its
    parameters are flattened for the fused optimizer."""
    init_weights(net, init_type, gain=init_gain)
    net.to(device)
    if device.type == "cuda":
        flatten_parameters(net)
    return net


def define_G(input_nc, output_nc, ngf, netG, norm='batch', use_dropout=False, init_type='normal', init_gain=0.02,
             gpu_ids=[]):
    net = None
    norm_layer = get_norm_layer(norm_type=norm)
    if netG == 'resnet_9blocks':
        net = ResnetGenerator(input_nc, output_nc, ngf, norm_layer=norm_layer, use_dropout=use_dropout, n_blocks=9)
    elif netG == 'resnet_6blocks':
        net = ResnetGenerator(input_nc, output_nc, ngf, norm_layer=norm_layer, use_dropout=use_dropout, n_blocks=6)
    elif netG == 'unet_custom':
        net = UnetGenerator(input_nc, output_nc, 5, ngf, norm_layer=norm_layer, use_dropout=use_dropout)
    elif netG == 'unet_256':
        net = UnetGenerator(input_nc, output_nc, 8, ngf, norm_layer=norm_layer, use_dropout=use_dropout)
    elif netG == 'Dynet':
        raise NotImplementedError('Generator model [Dynet] needs MONAI DynUNet (out of scope, SURVEY §2 row 1)')
    else:
        raise NotImplementedError('Generator model name [%s] is not recognized' % netG)
    return init_net(net, init_type, init_gain, gpu_ids)


def define_D(input_nc, ndf, netD, n_layers_D=3, norm='batch', use_sigmoid=False, init_type='normal', init_gain=0.02,
             gpu_ids=[]):
    net = None
    norm_layer = get_norm_layer(norm_type=norm)
    if netD == 'basic':
        net = NLayerDiscriminator(input_nc, ndf, n_layers=3, norm_layer=norm_layer, use_sigmoid=use_sigmoid)
    elif netD == 'n_layers':
        net = NLayerDiscriminator(input_nc, ndf, n_layers_D, norm_layer=norm_layer, use_sigmoid=use_sigmoid)
    elif netD == 'pixel':
        raise NotImplementedError('Discriminator model [pixel] is not implemented by the HIP engine '
                                  '(not selected by any reference config)')
    else:
        raise NotImplementedError('Discriminator model name [%s] is not recognized' % net)
    return init_net(net, init_type, init_gain, gpu_ids)


# =======================================================================================
# Losses
# =======================================================================================

class GANLoss(nn.Module):
    """networks3D.py:130-150: MSE (lsgan) or BCE against a constant 1/0 target.  Calling it
    evaluates the loss value on the device with the HIP loss kernel (no autograd graph; the
    CycleGAN step computes loss gradients inside its fused backward)."""

    def __init__(self, use_lsgan=True, target_real_label=1.0, target_fake_label=0.0):
        super().__init__()
        self.register_buffer('real_label', torch.tensor(target_real_label))
        self.register_buffer('fake_label', torch.tensor(target_fake_label))
        self.use_lsgan = use_lsgan

    def get_target_tensor(self, input, target_is_real):
        target_tensor = self.real_label if target_is_real else self.fake_label
        return target_tensor.expand_as(input)

    def __call__(self, input, target_is_real):
        from mragan_hip import ops
        t = float(self.real_label if target_is_real else self.fake_label)
        out = torch.zeros(1, device=input.device, dtype=torch.float32)
        ops.gan_loss(input.contiguous().float(), t, self.use_lsgan, 1.0, out, None)
        return out[0]


def Cor_CoeLoss(y_pred, y_target):
    """networks3D.py:156-166 (1 − r²).  The reference computes it in backward_G but never adds
    it to loss_G; here it is evaluated only on demand (outside the training step)."""
    x, y = y_pred, y_target
    x_var = x - torch.mean(x)
    y_var = y - torch.mean(y)
    r_num = torch.sum(x_var * y_var)
    r_den = torch.sqrt(torch.sum(x_var ** 2)) * torch.sqrt(torch.sum(y_var ** 2))
    r = r_num / r_den
    return 1 - r ** 2


# =======================================================================================
# Networks
# =======================================================================================

class _EngineNet(nn.Module):
    """Common forward: NCDHW in/out (reference layout), NDHWC inside, one autograd node."""

    _plan = None

    def _compile(self):
        raise NotImplementedError

    @property
    def plan(self):
        if self._plan is None:
            object.__setattr__(self, "_plan", self._compile())
        return self._plan

    def mark_params_dirty(self):
        if self._plan is not None:
            self._plan.dirty = True

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self.mark_params_dirty()

    def forward(self, input):
        if not input.is_cuda:
            raise RuntimeError(f"{type(self).__name__} runs on the HIP device only (got a {input.device} tensor); "
                               "there is no CPU path")
        if not self.training:
            raise NotImplementedError("eval-mode InstanceNorm (running statistics) is not supported by the HIP engine; "
                                      "the reference never switches its nets to eval (test.py uses train-mode stats)")
        ensure_flat(self)
        x = input.float().permute(0, 2, 3, 4, 1).contiguous()
        params = tuple(self.parameters())
        y = _EngineFunction.apply(x, self, *params)
        return y.permute(0, 4, 1, 2, 3)


class _EngineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net, *params):
        from mragan_hip import engine
        plan = net.plan
        nctx = plan.forward(x)
        entries = plan.running_entries([(nctx, 0, nctx.N)])
        ctx._keep = engine.apply_running_updates(entries, x.device)
        ctx.nctx, ctx.net = nctx, net
        return nctx.out

    @staticmethod
    def backward(ctx, gout):
        net = ctx.net
        ensure_flat(net)
        need_w = any(p.requires_grad for p in net.parameters())
        dx = net.plan.backward(ctx.nctx, [gout.contiguous()], need_wgrad=need_w,
                               need_input_grad=ctx.needs_input_grad[0])
        return (dx, None) + (None,) * (len(ctx.needs_input_grad) - 2)


class ResnetGenerator(_EngineNet):
    """networks3D.py:173-220 (padding_type 'reflect' builds ReplicationPad3d, as in the reference)."""

    def __init__(self, input_nc, output_nc, ngf=64, norm_layer=InstanceNorm3d, use_dropout=False, n_blocks=6,
                 padding_type='reflect'):
        assert n_blocks >= 0
        super().__init__()
        self.input_nc, self.output_nc, self.ngf = input_nc, output_nc, ngf
        if type(norm_layer) == functools.partial:
            use_bias = norm_layer.func == InstanceNorm3d
        else:
            use_bias = norm_layer == InstanceNorm3d
        if norm_layer is None:
            raise NotImplementedError("norm='none' generator is not supported by the HIP engine")
        model = [ReplicationPad3d(3), Conv3d(input_nc, ngf, kernel_size=7, padding=0, bias=use_bias),
                 norm_layer(ngf), ReLU(True)]
        n_downsampling = 2
        for i in range(n_downsampling):
            mult = 2 ** i
            model += [Conv3d(ngf * mult, ngf * mult * 2, kernel_size=3, stride=2, padding=1, bias=use_bias),
                      norm_layer(ngf * mult * 2), ReLU(True)]
        mult = 2 ** n_downsampling
        for i in range(n_blocks):
            model += [ResnetBlock(ngf * mult, padding_type=padding_type, norm_layer=norm_layer,
                                  use_dropout=use_dropout, use_bias=use_bias)]
        for i in range(n_downsampling):
            mult = 2 ** (n_downsampling - i)
            model += [ConvTranspose3d(ngf * mult, int(ngf * mult / 2), kernel_size=3, stride=2, padding=1,
                                      output_padding=1, bias=use_bias),
                      norm_layer(int(ngf * mult / 2)), ReLU(True)]
        model += [ReplicationPad3d(3)]
        model += [Conv3d(ngf, output_nc, kernel_size=7, padding=0)]
        model += [Tanh()]
        self.model = nn.Sequential(*model)

    def _compile(self):
        from mragan_hip.engine import compile_resnet_generator
        return compile_resnet_generator(self)


class ResnetBlock(nn.Module):
    """networks3D.py:224-263.  Executed as one fused stage by the generator's engine."""

    def __init__(self, dim, padding_type, norm_layer, use_dropout, use_bias):
        super().__init__()
        self.conv_block = self.build_conv_block(dim, padding_type, norm_layer, use_dropout, use_bias)

    def build_conv_block(self, dim, padding_type, norm_layer, use_dropout, use_bias):
        conv_block = []
        if padding_type not in ('reflect', 'replicate'):
            if padding_type == 'zero':
                raise NotImplementedError("padding_type 'zero' is not used by the reference generator")
            raise NotImplementedError('padding [%s] is not implemented' % padding_type)
        conv_block += [ReplicationPad3d(1)]
        conv_block += [Conv3d(dim, dim, kernel_size=3, padding=0, bias=use_bias), norm_layer(dim), ReLU(True)]
        if use_dropout:
            conv_block += [Dropout(0.5)]
        conv_block += [ReplicationPad3d(1)]
        conv_block += [Conv3d(dim, dim, kernel_size=3, padding=0, bias=use_bias), norm_layer(dim)]
        return nn.Sequential(*conv_block)

    def forward(self, x):
        raise NotImplementedError("ResnetBlock runs inside its ResnetGenerator's HIP engine")


class NLayerDiscriminator(_EngineNet):
    """networks3D.py:381-425 (PatchGAN)."""

    def __init__(self, input_nc, ndf=64, n_layers=3, norm_layer=InstanceNorm3d, use_sigmoid=False):
        super().__init__()
        if norm_layer is None:
            raise NotImplementedError("norm='none' discriminator is not supported by the HIP engine")
        if type(norm_layer) == functools.partial:
            use_bias = norm_layer.func == InstanceNorm3d
        else:
            use_bias = norm_layer == InstanceNorm3d
        kw, padw = 4, 1
        sequence = [Conv3d(input_nc, ndf, kernel_size=kw, stride=2, padding=padw), LeakyReLU(0.2, True)]
        nf_mult = 1
        for n in range(1, n_layers):
            nf_mult_prev = nf_mult
            nf_mult = min(2 ** n, 8)
            sequence += [Conv3d(ndf * nf_mult_prev, ndf * nf_mult, kernel_size=kw, stride=2, padding=padw,
                                bias=use_bias),
                         norm_layer(ndf * nf_mult), LeakyReLU(0.2, True)]
        nf_mult_prev = nf_mult
        nf_mult = min(2 ** n_layers, 8)
        sequence += [Conv3d(ndf * nf_mult_prev, ndf * nf_mult, kernel_size=kw, stride=1, padding=padw, bias=use_bias),
                     norm_layer(ndf * nf_mult), LeakyReLU(0.2, True)]
        sequence += [Conv3d(ndf * nf_mult, 1, kernel_size=kw, stride=1, padding=padw)]
        if use_sigmoid:
            sequence += [Sigmoid()]
        self.input_nc = input_nc
        self.model = nn.Sequential(*sequence)

    def _compile(self):
        from mragan_hip.engine import compile_nlayer_discriminator
        return compile_nlayer_discriminator(self)


class UnetGenerator(_EngineNet):
    """networks3D.py:270-293.  `num_downs` stride-2 k4 convolutions; the innermost block is
    built first, so parameter init consumes the RNG innermost-out like the reference, and
    the nested `model.model.1.model.3...` state_dict keys are identical."""

    def __init__(self, input_nc, output_nc, num_downs, ngf=64, norm_layer=InstanceNorm3d, use_dropout=False):
        super().__init__()
        if num_downs < 5:
            raise ValueError("UnetGenerator needs num_downs >= 5 (networks3D.py:278-283)")
        if norm_layer is None:
            raise NotImplementedError("norm='none' generator is not supported by the HIP engine")
        self.input_nc, self.output_nc, self.ngf, self.num_downs = input_nc, output_nc, ngf, num_downs
        blk = UnetSkipConnectionBlock(ngf * 8, ngf * 8, submodule=None, norm_layer=norm_layer, innermost=True)
        for _ in range(num_downs - 5):
            blk = UnetSkipConnectionBlock(ngf * 8, ngf * 8, submodule=blk, norm_layer=norm_layer,
                                          use_dropout=use_dropout)
        for outer, inner in ((ngf * 4, ngf * 8), (ngf * 2, ngf * 4), (ngf, ngf * 2)):
            blk = UnetSkipConnectionBlock(outer, inner, submodule=blk, norm_layer=norm_layer)
        self.model = UnetSkipConnectionBlock(output_nc, ngf, input_nc=input_nc, submodule=blk, outermost=True,
                                             norm_layer=norm_layer)

    def _compile(self):
        from mragan_hip.engine import compile_unet_generator
        return compile_unet_generator(self)


class UnetSkipConnectionBlock(nn.Module):
    """networks3D.py:298-343: X → [down → submodule → up] → cat(X, ·) (outermost: no cat).
    The reference's in-place LeakyReLU/ReLU also rewrite the skip tensor; the engine
    reproduces that (the skip carries LeakyReLU(X)).  Executed by the generator's engine."""

    def __init__(self, outer_nc, inner_nc, input_nc=None, submodule=None, outermost=False, innermost=False,
                 norm_layer=InstanceNorm3d, use_dropout=False):
        super().__init__()
        self.outermost, self.innermost = outermost, innermost
        if type(norm_layer) == functools.partial:
            use_bias = norm_layer.func == nn.InstanceNorm2d      # False for the 3-D norms (reference quirk)
        else:
            use_bias = norm_layer == nn.InstanceNorm2d
        if input_nc is None:
            input_nc = outer_nc
        downconv = Conv3d(input_nc, inner_nc, kernel_size=4, stride=2, padding=1, bias=use_bias)
        downrelu, uprelu = LeakyReLU(0.2, True), ReLU(True)
        downnorm, upnorm = norm_layer(inner_nc), norm_layer(outer_nc)
        if outermost:
            upconv = ConvTranspose3d(inner_nc * 2, outer_nc, kernel_size=4, stride=2, padding=1)
            seq = [downconv, submodule, uprelu, upconv, Tanh()]
        elif innermost:
            upconv = ConvTranspose3d(inner_nc, outer_nc, kernel_size=4, stride=2, padding=1, bias=use_bias)
            seq = [downrelu, downconv, uprelu, upconv, upnorm]
        else:
            upconv = ConvTranspose3d(inner_nc * 2, outer_nc, kernel_size=4, stride=2, padding=1, bias=use_bias)
            seq = [downrelu, downconv, downnorm, submodule, uprelu, upconv, upnorm]
            if use_dropout:
                seq.append(Dropout(0.5))
        self.model = nn.Sequential(*seq)

    def forward(self, x):
        raise NotImplementedError("UnetSkipConnectionBlock runs inside its UnetGenerator's HIP engine")
