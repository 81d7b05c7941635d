"""Explicit forward/backward plans for the CycleGAN networks on the HIP kernel library.

The reference runs ResnetGenerator / NLayerDiscriminator through torch.nn + autograd
(networks3D.py:173-263, 381-425).  Here each network is compiled once into a list of
*stages* (conv or transposed conv → InstanceNorm → activation, or a whole ResnetBlock) and
run by hand-written forward and backward passes on NDHWC fp32 tensors:

* the ReplicationPad3d in front of a conv is produced by the previous stage's InstanceNorm
  kernel writing a padded output (no separate pad pass), and folded back inside the next
  InstanceNorm-backward kernel;
* conv biases that feed an InstanceNorm are mathematically cancelled by it (affine=False), so
  they are not added in the forward and their gradient is exactly 0 (the reference's fp32
  gradient for them is round-off noise); they still enter the running_mean;
* weight gradients are written straight into the net's flat gradient buffer (torch layout),
  so the optimizer is one fused kernel per buffer.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import ops
from ._lib import call

# A/B switch: MRAGAN_NO_IN_STATS=1 runs the ResnetBlock InstanceNorms with their own statistics
# pass instead of the brick conv's epilogue partials
_NO_IN_STATS = bool(int(__import__("os").environ.get("MRAGAN_NO_IN_STATS", "0") or "0"))
_NO_HEAD_STATS = __import__("os").environ.get("MRAGAN_NO_HEAD_STATS") is not None   # A/B: head dgrad without IN statistics
_NO_S2_STATS = __import__("os").environ.get("MRAGAN_NO_S2_STATS") is not None       # A/B: stride-2 dgrads without them
# A/B: a ResnetBlock's second-IN backward statistics from the next block's conv1 data gradient (ABI 18)
_NO_SKIP_STATS = __import__("os").environ.get("MRAGAN_NO_SKIP_STATS") is not None
# A/B: skip statistics only up to this batch (the N = 4 data gradient runs the 8-wave brick, whose
# statistics epilogue costs ≈ 5 µs, r05ba)
_SKIP_STATS_MAXN = int(__import__("os").environ.get("MRAGAN_SKIP_STATS_MAXN", "0") or "0")
# conv2's data gradient where the split runs: plain (split) + IN1's statistics pass, not the
# backward-statistics brick (128³ step 29.10 / 29.02 vs 29.52 / 29.30 ms, r05bi); A/B switch
_IN1_STATS_BIG = __import__("os").environ.get("MRAGAN_IN1_STATS_BIG") is not None


def _dgrad_split(N, D, H, W, C):
    """Scheduling hint, not a correctness rule: where conv_igemm.hip full_dgrad_split_applicable
    runs the plain ResnetBlock data gradient as interior brick + shell pass (N ≥ 2 at 24³ / 32³,
    multiples of 8 from 24; faster than any whole-grid brick there, and than the backward-statistics
    brick plus the saved statistics pass: 128³ step 29.07 / 29.10 ms with it against 29.40 / 29.44
    with the statistics brick, r05bg), the engine asks for the plain data gradient and runs the
    statistics pass.  Both passes read the pre-split weights (ABI 19), so a disagreement with the C
    rule would cost time, never correctness — and there is none: the library's rule is queried
    (mragan_conv3d_dgrad_split, which also honours MRAGAN_DGRAD_SPLIT).  The skip
    statistics (ABI 18) are used below 32³ only: at 1 × 32³ too the statistics brick (K-split, large
    grid) costs about what the statistics pass saves (r05bh: 29.12 / 29.22 vs 29.08 / 29.07 ms)."""
    return ops.dgrad_split(N, D, H, W, C, C)
# A/B switch: MRAGAN_NO_OP16=1 keeps the ResnetBlock tensors fp32 in the bf16 / fp16 modes (no
# 16-bit operand planes, ABI 11)
_NO_OP16 = bool(int(__import__("os").environ.get("MRAGAN_NO_OP16", "0") or "0"))
# A/B switch: MRAGAN_NO_S2_PLANES keeps the stem / down1 InstanceNorm outputs in fp32 (no ABI 14 planes)
_NO_S2_PLANES = __import__("os").environ.get("MRAGAN_NO_S2_PLANES") is not None
# brickT on planes (G up2's input, G down1's dY only as planes): MRAGAN_BRICKT_PLANES=0 turns it off
_BRICKT_PLANES = __import__("os").environ.get("MRAGAN_BRICKT_PLANES", "1") != "0"
# ABI 17: the k7 layers' 32-channel operands (the head input, the stem IN backward's dx) only as planes
# in the one-plane modes; MRAGAN_NO_K7_PLANES=1 keeps them fp32 (A/B)
_NO_K7_PLANES = __import__("os").environ.get("MRAGAN_NO_K7_PLANES") is not None
# ABI 15: InstanceNorm statistics finalized in the producing brick's launch (MRAGAN_NO_IN_TICKETS: off)
_IN_FIN = ops.in_tickets_enabled()
# A/B switch: MRAGAN_FP32_PACKS=1 refreshes the fp32 packs of the brick convs in every mode
_FP32_PACKS = (bool(int(__import__("os").environ.get("MRAGAN_FP32_PACKS", "0") or "0"))
               # the library's A/B switches that send those convs to the fp32-pack kernels
               or any(v in __import__("os").environ for v in ("MRAGAN_NO_BRICK", "MRAGAN_BRICK_STAGED")))

IN_MOMENTUM = 0.1
# A/B switch: MRAGAN_NO_WGRAD_DEFER=1 runs each pass's ResnetBlock weight gradients in that pass (no
# first-pass + cycle-pass pairing, NetPlan.backward wgrad_defer / wgrad_pair)
_NO_WGRAD_DEFER = __import__("os").environ.get("MRAGAN_NO_WGRAD_DEFER") is not None


# --------------------------------------------------------------------------------------
# Layers
# --------------------------------------------------------------------------------------

class ConvLayer:
    """A Conv3d (forward form) or ConvTranspose3d (transposed form) with packed weights."""

    def __init__(self, module, transposed: bool):
        self.m = module
        self.transposed = transposed
        self.k = module.kernel_size
        self.s = module.stride
        self.p = module.padding
        self.op = getattr(module, "output_padding", 0)
        self.cin = module.in_channels
        self.cout = module.out_channels
        self._wp_fwd: Optional[torch.Tensor] = None     # fp32 packs [t][Cout][Cin] / [t][Cin][Cout]
        self._wp_bwd: Optional[torch.Tensor] = None
        self.ws_fwd: Optional[torch.Tensor] = None      # bf16x3 pre-split copies (brick convs only)
        self.ws_bwd: Optional[torch.Tensor] = None
        self.fp32_stale = False                         # the fp32 packs were not refreshed (packs())

    # The fp32 packs as the kernels may see them: None while stale (ABI 19 — the library then refuses
    # every kernel that would read them, instead of computing with old weights; r05final2's garbage
    # 128³ gradients were a stale pack read by the interior + shell data gradient's shell pass, which
    # now stages the pre-split copy like the interior brick)
    @property
    def wp_fwd(self) -> Optional[torch.Tensor]:
        return None if self.fp32_stale else self._wp_fwd

    @property
    def wp_bwd(self) -> Optional[torch.Tensor]:
        return None if self.fp32_stale else self._wp_bwd

    @staticmethod
    def _splittable(k, s, ny, C):
        # the bf16x3 brick kernel's shapes (conv_brick_applicable): k3 s1, C % 32, ny % 64
        return k == 3 and s == 1 and C % 32 == 0 and ny % 64 == 0

    def packs(self):
        """The two packs of this layer as (src, A, B, T, transpose_ab, dst) (buffers allocated)."""
        w = self.m.weight.data
        T = self.k ** 3
        if self._wp_fwd is None or self._wp_fwd.device != w.device:
            self._wp_fwd = torch.empty(w.numel(), device=w.device, dtype=torch.float32)
            self._wp_bwd = torch.empty(w.numel(), device=w.device, dtype=torch.float32)
        if not self.transposed:     # torch [Cout][Cin][t]
            out = [(w, self.cout, self.cin, T, False, self._wp_fwd),     # [t][Cout][Cin]
                   (w, self.cout, self.cin, T, True, self._wp_bwd)]      # [t][Cin][Cout]
        else:
            out = [(w, self.cin, self.cout, T, True, self._wp_fwd),      # torch [Cin][Cout][t] → [t][Cout][Cin]
                   (w, self.cin, self.cout, T, False, self._wp_bwd)]     # [t][Cin][Cout]
        # pre-split 16-bit fragment copies for the brick kernel, refreshed by the same pack launch
        # (tr 2|3: bf16 hi/lo — the bf16x3 and bf16 modes; tr 4|5: fp16 — the fp16 mode)
        (_, A, B, _, tf, _), (_, _, _, _, tb, _) = out
        prec = ops.get_conv_precision()
        base = 4 if prec == "fp16" else 2
        # (+ the k3 s2 p1 down convs' forward: the stride-2 brick reads the same fragment copy, round 6)
        split_f = (self._splittable(self.k, self.s, self.cout, self.cin)
                   or (self.k == 3 and self.s == 2 and self.p == 1 and not self.transposed and self.cin % 32 == 0
                       and self.cout % 64 == 0))
        split_b = self._splittable(self.k, self.s, self.cin, self.cout)
        if split_f:
            if self.ws_fwd is None or self.ws_fwd.device != w.device:
                self.ws_fwd = torch.empty(w.numel(), device=w.device, dtype=torch.float32)
            out.append((w, A, B, T, base + int(tf), self.ws_fwd))
        if split_b:
            if self.ws_bwd is None or self.ws_bwd.device != w.device:
                self.ws_bwd = torch.empty(w.numel(), device=w.device, dtype=torch.float32)
            out.append((w, A, B, T, base + int(tb), self.ws_bwd))
        self.fp32_stale = False
        if prec != "f32" and split_f and split_b and not self.transposed and not _FP32_PACKS:
            # the MFMA-mode kernels of a k3 s1 ResnetBlock conv (the bricks both ways, the interior +
            # shell data gradient) read only its pre-split copies: the two fp32 packs are not
            # refreshed (the repack moves half the bytes; a mode switch repacks, ensure_packed) and
            # are not handed to the library while stale (wp_fwd / wp_bwd are None)
            self.fp32_stale = True
            out = out[2:]
        return out

    def repack(self):
        for src, A, B, T, tr, dst in self.packs():
            ops.pack_weight(src, A, B, T, tr, dst)

    def out_spatial(self, d, h, w):
        if self.transposed:
            f = lambda n: ops.convT_out_size(n, self.k, self.s, self.p, self.op)
        else:
            f = lambda n: ops.conv_out_size(n, self.k, self.s, self.p)
        return f(d), f(h), f(w)

    def forward(self, x, bias=None, act=None):
        N, D, H, W, _ = x.shape
        return ops.conv3d(x, self.wp_fwd, self.cout, self.k, self.s, self.p, self.out_spatial(D, H, W),
                          bias=bias, act=act, transposed=self.transposed, wsplit=self.ws_fwd)

    def forward_in_stats(self, x):
        """forward() of a bias-free conv feeding an InstanceNorm; in the MFMA modes the brick
        kernel (k3 s1), the implicit GEMM (no K split), brickT (32-channel ConvTranspose3d) and the
        stem's thin1 kernel (k7, 1 → 32) also leave the IN statistics partials.
        Returns (y, part, chunks); chunks = 0 when no partials were produced."""
        # G stem (thin1 ring kernel): one input channel, or two in the one-plane modes (nc = 2)
        thin1 = ((self.cin == 1 or (self.cin == 2 and ops.get_conv_precision() in ("bf16", "fp16")))
                 and self.k == 7 and self.s == 1 and not self.transposed)
        if _NO_IN_STATS or ops.get_conv_precision() == "f32" or (min(self.cin, self.cout) < 8 and not thin1):
            return self.forward(x), None, 0
        N, D, H, W, _ = x.shape
        osp = self.out_spatial(D, H, W)
        part = ops.in_partials_buffer(N, osp, self.cout, x.device)
        y, chunks = ops.conv3d_in_stats(x, self.wp_fwd, self.cout, self.k, self.s, self.p, osp, self.ws_fwd, part,
                                        transposed=self.transposed)
        return y, part, chunks

    def forward_in_stats_op16(self, x16):
        """forward_in_stats on the operand plane of the input (brick kernel, 16-bit modes)."""
        N, D, H, W, _ = x16.shape
        osp = self.out_spatial(D, H, W)
        part = None if _NO_IN_STATS else ops.in_partials_buffer(N, osp, self.cout, x16.device)
        y, chunks = ops.conv3d_op16(x16, self.wp_fwd, self.cout, self.k, self.s, self.p, osp, self.ws_fwd, part,
                                    transposed=self.transposed)
        return y, part, chunks

    def forward_in_stats_op16_fin(self, x16):
        """forward_in_stats_op16 → (y, part, chunks, stats): stats = (mean, rstd) when the conv's
        launch finalized them (ABI 15; then instnorm_fwd_op16(stats=…)), else None."""
        if not _IN_FIN or _NO_IN_STATS:
            return self.forward_in_stats_op16(x16) + (None,)
        N, D, H, W, _ = x16.shape
        osp = self.out_spatial(D, H, W)
        part = ops.in_partials_buffer(N, osp, self.cout, x16.device)
        y, chunks, stats = ops.conv3d_op16(x16, self.wp_fwd, self.cout, self.k, self.s, self.p, osp, self.ws_fwd, part,
                                           fin=True)
        return y, part, chunks, stats

    def dgrad_op16(self, dy16, in_spatial):
        """dgrad from the operand plane of dy (brick kernel, 16-bit modes)."""
        return ops.conv3d_op16(dy16, self.wp_bwd, self.cin, self.k, self.s, self.p, in_spatial, self.ws_bwd,
                               transposed=not self.transposed)[0]

    def dgrad_op16_in_stats(self, dy16, norm_x, mean, rstd, act):
        """dgrad_op16 (whole-grid, k3 s1 p0) that also leaves the backward-statistics partials of
        the InstanceNorm(+act) that produced this conv's input (norm_x its pre-norm input).
        Returns (dz, part, chunks, coef); chunks = 0: no partials; coef: that IN backward's
        coefficients when the launch finalized them (ABI 15), else None."""
        if _NO_IN_STATS:
            N, D, H, W, _ = dy16.shape
            return self.dgrad_op16(dy16, (D + 2, H + 2, W + 2)), None, 0, None
        N, D, H, W, _ = dy16.shape
        part = ops.in_partials_buffer(N, (D + 2, H + 2, W + 2), self.cin, dy16.device)
        if _IN_FIN:
            dz, chunks, coef = ops.conv3d_op16_dgrad_in_stats(dy16, self.wp_bwd, self.cin, self.ws_bwd, norm_x, mean,
                                                              rstd, act, part, fin=True)
            return dz, part, chunks, coef
        dz, chunks = ops.conv3d_op16_dgrad_in_stats(dy16, self.wp_bwd, self.cin, self.ws_bwd, norm_x, mean, rstd, act,
                                                    part)
        return dz, part, chunks, None

    def dgrad_op16_in_stats_add(self, dy16, norm_x, mean, rstd, act, add, fin=True):
        """dgrad_op16_in_stats for an InstanceNorm whose backward input is fold(dz) + add (ABI 18):
        conv1 of ResnetBlock i+1, whose input gradient meets block i+1's output gradient G (the
        skip path) at block i's second IN.  Returns (dz, part, chunks, coef) as dgrad_op16_in_stats;
        fin=False when the consumer cannot take finalized coefficients (coef is then None)."""
        N, D, H, W, _ = dy16.shape
        part = ops.in_partials_buffer(N, (D + 2, H + 2, W + 2), self.cin, dy16.device)
        if _IN_FIN and fin:
            dz, chunks, coef = ops.conv3d_op16_dgrad_in_stats(dy16, self.wp_bwd, self.cin, self.ws_bwd, norm_x, mean,
                                                              rstd, act, part, fin=True, x_add=add)
            return dz, part, chunks, coef
        dz, chunks = ops.conv3d_op16_dgrad_in_stats(dy16, self.wp_bwd, self.cin, self.ws_bwd, norm_x, mean, rstd, act,
                                                    part, x_add=add)
        return dz, part, chunks, None

    def wgrad_op16(self, x16, dy16, accumulate=True):
        """wgrad of a forward-form conv from the operand planes of X and dY (wgrad3, 16-bit modes)."""
        ops.conv3d_wgrad_op16(dy16, x16, self.k, self.s, self.p, self.m.weight.grad, accumulate)

    def op16_ok(self, W, H=None):
        """Can this k3 s1 conv run on operand planes (brick both ways, wgrad3) at output width W?
        (wgrad3's row segments: 16 voxels, or 24 with whole rows per 8-segment stage — H % 8 == 0)"""
        seg_ok = W % 16 == 0 or (W == 24 and (H is None or H % 8 == 0))
        return (not self.transposed and self.k == 3 and self.s == 1 and self.ws_fwd is not None
                and self.ws_bwd is not None and self.cin % 64 == 0 and self.cout % 64 == 0 and seg_ok)

    def dgrad(self, dy, in_spatial):
        """Gradient w.r.t. this layer's input (shape = input spatial dims, Cin channels)."""
        return ops.conv3d(dy, self.wp_bwd, self.cin, self.k, self.s, self.p, in_spatial,
                          transposed=not self.transposed, wsplit=self.ws_bwd)

    def dgrad_in_stats_ok(self):
        """The G head (ngf → 1, k7 p0; ngf → 2 in the one-plane modes): its data gradient runs the
        thin1 ring kernel in the MFMA modes, whose epilogue can leave the backward statistics of the
        InstanceNorm in front of it (ABI 12)."""
        prec = ops.get_conv_precision()
        return (not _NO_IN_STATS and not _NO_HEAD_STATS and prec != "f32" and not self.transposed
                and (self.cout == 1 or (self.cout == 2 and prec in ("bf16", "fp16")))
                and self.k == 7 and self.s == 1 and self.p == 0)

    def dgrad_in_stats(self, dy, in_spatial, norm_x, mean, rstd, act, fold_pad):
        """dgrad() that also leaves the backward-statistics partials of the IN(+act) whose output,
        replication-padded by fold_pad, was this conv's input.  Returns (dz, part, chunks)."""
        part = ops.in_partials_buffer(dy.shape[0], in_spatial, self.cin, dy.device)
        dz, chunks = ops.conv3d_dgrad_in_stats(dy, self.wp_bwd, self.cin, self.k, norm_x, mean, rstd, act, fold_pad,
                                               part)
        return dz, part, chunks

    def dgrad_bwd_stats_ok(self):
        """Stride-2 layers: their data gradient runs the 16-bit-MFMA implicit GEMM, whose epilogue
        can leave the backward statistics of the (unpadded) InstanceNorm in front (ABI 12)."""
        return (not _NO_IN_STATS and not _NO_S2_STATS and ops.get_conv_precision() != "f32" and self.s == 2
                and min(self.cin, self.cout) >= 8)

    def dgrad_bwd_stats(self, dy, in_spatial, norm_x, mean, rstd, act):
        """dgrad() that also leaves the backward-statistics partials of the IN(+act) whose output
        was this conv's input.  Returns (dz, part, chunks)."""
        part = ops.in_partials_buffer(dy.shape[0], in_spatial, self.cin, dy.device)
        dz, chunks = ops.conv3d_bwd_stats(dy, self.wp_bwd, self.cin, self.k, self.s, self.p, in_spatial, self.ws_bwd,
                                          norm_x, mean, rstd, act, part, transposed=not self.transposed)
        return dz, part, chunks

    def wgrad_g16(self, x16, dy, accumulate=True):
        """wgrad of a forward-form conv whose input exists only as its operand plane: the k3 s2 convs
        (ABI 14) and the G head (k7, 32 → nc; ABI 17)."""
        if self.k == 7:
            ops.conv3d_wgrad_thin_op16(dy, x16, self.k, self.s, self.p, self.m.weight.grad, accumulate)
        else:
            ops.conv3d_wgrad_g16(dy, x16, self.k, self.s, self.p, self.m.weight.grad, accumulate)

    def k7_wide16_ok(self):
        """A k7 s1 layer between nc (1, 2) and 32 channels whose 32-channel operand can be its 16-bit
        operand plane in every kernel that reads it (thinn_x3, thin1 weight gradient; ABI 17)."""
        return (not _NO_K7_PLANES and ops.get_conv_precision() in ("bf16", "fp16") and not self.transposed
                and self.k == 7 and self.s == 1
                and ((self.cin == 32 and self.cout in (1, 2)) or (self.cout == 32 and self.cin in (1, 2))))

    def s2_plane_ok(self, W_in):
        """A forward-form k3 s2 p1 conv (G down1 / down2) that can read its input of width W_in as
        an operand plane: the implicit GEMM (Cin % 32) forward and wgrad3s2 (Cout % 64, coarse row
        segments of 16 voxels) weight gradient."""
        return (not self.transposed and self.k == 3 and self.s == 2 and self.p == 1 and self.cin % 32 == 0
                and self.cout % 64 == 0 and W_in % 32 == 0)

    def transposed_plane_bwd_ok(self, W_in):
        """A ConvTranspose3d k3 s2 p1 (G up1 / up2) whose backward can run on the plane of its output
        gradient: the data gradient is a forward-form implicit GEMM over Cout (% 32) input channels,
        the weight gradient wgrad3s2 with the plane as its gathered operand (Cin % 64 dense
        channels, coarse rows of 16: the input width W_in % 16)."""
        return (self.transposed and self.k == 3 and self.s == 2 and self.p == 1 and self.cout % 32 == 0
                and (self.cout == 32 or self.cout % 64 == 0) and self.cin % 64 == 0 and W_in % 16 == 0)

    def wgrad(self, x, dy, accumulate=True):
        g = self.m.weight.grad
        if not self.transposed:
            ops.conv3d_wgrad(dy, x, self.k, self.s, self.p, g, accumulate)     # dW[Cout][Cin][t]
        else:
            ops.conv3d_wgrad(x, dy, self.k, self.s, self.p, g, accumulate)     # dW[Cin][Cout][t]


@dataclass
class Stage:
    kind: str                       # "conv" | "block"
    conv: Optional[ConvLayer] = None
    norm: object = None             # InstanceNorm3d container or None
    act: Optional[str] = None
    prepad: int = 0                 # ReplicationPad3d applied to this stage's input
    use_bias: bool = False          # bias actually added (no norm after the conv)
    # block
    conv1: Optional[ConvLayer] = None
    norm1: object = None
    conv2: Optional[ConvLayer] = None
    norm2: object = None


@dataclass
class StageCtx:
    inp: torch.Tensor = None        # stage input (padded by prepad)
    h: torch.Tensor = None          # conv output
    mean: torch.Tensor = None
    rstd: torch.Tensor = None
    out: torch.Tensor = None        # stage output as produced (padded by next prepad)
    h1: torch.Tensor = None
    mean1: torch.Tensor = None
    rstd1: torch.Tensor = None
    z1: torch.Tensor = None         # block: relu(IN(h1)) padded by 1 (its operand plane on the op16 path)
    inp16: torch.Tensor = None      # block on the op16 path: the operand plane of inp


@dataclass
class NetCtx:
    N: int
    spatial: tuple
    stages: List[StageCtx] = field(default_factory=list)
    out: torch.Tensor = None


# --------------------------------------------------------------------------------------
# Network plan
# --------------------------------------------------------------------------------------

class NetPlan:
    """Stage list compiled from a ResnetGenerator / NLayerDiscriminator module tree."""

    def __init__(self, stages: List[Stage], in_channels: int, out_channels: int):
        self.stages = stages
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.dirty = True

    # ---- parameters --------------------------------------------------------------------
    def conv_layers(self):
        for st in self.stages:
            if st.kind == "block":
                yield st.conv1
                yield st.conv2
            else:
                yield st.conv

    def repack(self):
        """Every conv layer's two packs in one launch (after each optimizer step)."""
        if not hasattr(self, "_pack_table"):
            self._pack_table = ops.PackTable()
        self._packed_prec = ops.get_conv_precision()
        self._pack_table.run([p for c in self.conv_layers() for p in c.packs()])
        self.dirty = False

    def ensure_packed(self):
        # the pre-split fragment copies depend on the precision mode (fp16 vs bf16 words)
        if self.dirty or getattr(self, "_packed_prec", None) != ops.get_conv_precision():
            self.repack()

    def norms_in_order(self):
        for st in self.stages:
            if st.kind == "block":
                yield st, st.norm1, st.conv1
                yield st, st.norm2, st.conv2
            elif st.norm is not None:
                yield st, st.norm, st.conv

    # ---- forward -----------------------------------------------------------------------
    def _next_prepad(self, i):
        if i + 1 >= len(self.stages):
            return 0
        nxt = self.stages[i + 1]
        return 1 if nxt.kind == "block" else nxt.prepad

    def forward(self, x: torch.Tensor) -> NetCtx:
        """x: NDHWC [N, D, H, W, in_channels].  Returns the context holding every tensor the
        backward needs; ctx.out is the network output (NDHWC)."""
        self.ensure_packed()
        N, D, H, W, Cin = x.shape
        if Cin != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {Cin}")
        ctx = NetCtx(N=N, spatial=(D, H, W))
        first = self.stages[0]
        cur = ops.rpad(x, first.prepad) if first.prepad else x
        cur16 = None            # operand plane of cur (16-bit modes, ResnetBlock inputs)
        op16 = self._op16_active()
        for i, st in enumerate(self.stages):
            sc = StageCtx(inp=cur, inp16=cur16)
            ypad = self._next_prepad(i)
            # a ResnetBlock next: its input's operand plane beside the fp32 tensor (the skip add)
            want16 = op16 and i + 1 < len(self.stages) and self.stages[i + 1].kind == "block"
            # a ConvTranspose3d with a norm next (G up1): it reads its input's plane too (round 4)
            nxt_ = self.stages[i + 1] if i + 1 < len(self.stages) else None
            up16 = (op16 and not _NO_S2_PLANES and ypad == 0 and nxt_ is not None and nxt_.kind != "block"
                    and nxt_.norm is not None and not nxt_.prepad and nxt_.conv.transposed and nxt_.conv.cin % 32 == 0)
            out16 = None
            if st.kind == "block":
                if cur16 is not None:
                    # 16-bit operand planes (ABI 11): conv1 reads the block input's plane, IN1 writes
                    # only the plane of relu(IN(h1)) (conv2's operand), IN2 both copies of the output
                    # ABI 15: where the brick's launch finalizes the statistics, the IN is its apply pass alone
                    sc.h1, part, chunks, stats = st.conv1.forward_in_stats_op16_fin(cur16)
                    _, sc.z1, sc.mean1, sc.rstd1 = ops.instnorm_fwd_op16(sc.h1, act="relu", ypad=1, part=part,
                                                                          chunks=chunks, stats=stats)
                    if want16:
                        sc.h, part, chunks, stats = st.conv2.forward_in_stats_op16_fin(sc.z1)
                        sc.out, out16, sc.mean, sc.rstd = ops.instnorm_fwd_op16(sc.h, act=None, ypad=ypad, resid=cur,
                                                                                rpad=1, part=part, chunks=chunks,
                                                                                want_f32=True, stats=stats)
                    elif up16:
                        # the last block before G up1: its output's plane feeds up1's implicit GEMM, the
                        # fp32 copy up1's weight gradient
                        sc.h, part, chunks, stats = st.conv2.forward_in_stats_op16_fin(sc.z1)
                        sc.out, out16, sc.mean, sc.rstd = ops.instnorm_fwd_op16(sc.h, act=None, ypad=ypad, resid=cur,
                                                                                rpad=1, part=part, chunks=chunks,
                                                                                want_f32=True, stats=stats)
                    else:
                        sc.h, part, chunks = st.conv2.forward_in_stats_op16(sc.z1)
                        sc.out, sc.mean, sc.rstd = ops.instnorm_fwd(sc.h, act=None, ypad=ypad, resid=cur, rpad=1,
                                                                    part=part, chunks=chunks)
                else:
                    # the brick conv accumulates its InstanceNorm's statistics in its epilogue
                    sc.h1, part, chunks = st.conv1.forward_in_stats(cur)
                    sc.z1, sc.mean1, sc.rstd1 = ops.instnorm_fwd(sc.h1, act="relu", ypad=1, part=part, chunks=chunks)
                    sc.h, part, chunks = st.conv2.forward_in_stats(sc.z1)
                    sc.out, sc.mean, sc.rstd = ops.instnorm_fwd(sc.h, act=None, ypad=ypad, resid=cur, rpad=1, part=part,
                                                                chunks=chunks)
            else:
                bias = st.conv.m.bias if (st.use_bias and st.conv.m.bias is not None) else None
                if st.norm is not None:
                    # the conv's epilogue leaves the norm's statistics partials where it can
                    if cur is None or (cur16 is not None and st.conv.transposed):
                        # the input exists only as its plane (only16 below), or also as one (up16)
                        sc.h, part, chunks = st.conv.forward_in_stats_op16(cur16)
                    else:
                        sc.h, part, chunks = st.conv.forward_in_stats(cur)
                    # a stride-2 forward conv next (G down1 / down2): this norm's output only as its
                    # plane — that conv and its weight gradient are its only readers (ABI 14)
                    nxt = self.stages[i + 1] if i + 1 < len(self.stages) else None
                    # the G head next (k7, 32 → nc, ABI 17): its input only as the plane — the head's
                    # forward (thinn_x3) and weight gradient are its only readers
                    head16 = (op16 and nxt is not None and nxt.kind != "block" and nxt.norm is None
                              and nxt.prepad == ypad and nxt.conv.cin == 32 and nxt.conv.k7_wide16_ok())
                    # — or a 32-output-channel ConvTranspose3d next (G up2: brickT reads the plane, its
                    # weight gradient takes both operands as planes)
                    only16 = head16 or (op16 and not _NO_S2_PLANES and ypad == 0 and nxt is not None and nxt.kind != "block"
                              and nxt.norm is not None and not nxt.prepad
                              and (nxt.conv.s2_plane_ok(sc.h.shape[3])
                                   or (_BRICKT_PLANES and nxt.conv.transposed and nxt.conv.cout == 32
                                       and nxt.conv.transposed_plane_bwd_ok(sc.h.shape[3]))))
                    if only16:
                        _, out16, sc.mean, sc.rstd = ops.instnorm_fwd_op16(sc.h, act=st.act, ypad=ypad, part=part,
                                                                           chunks=chunks)
                    elif want16 and self._op16_blocks_ok(sc.h.shape[3], sc.h.shape[2]):
                        sc.out, out16, sc.mean, sc.rstd = ops.instnorm_fwd_op16(sc.h, act=st.act, ypad=ypad,
                                                                                part=part, chunks=chunks,
                                                                                want_f32=True)
                    else:
                        sc.out, sc.mean, sc.rstd = ops.instnorm_fwd(sc.h, act=st.act, ypad=ypad, part=part,
                                                                    chunks=chunks)
                else:
                    if cur is None:
                        # the G head on its input's plane (ABI 17)
                        c = st.conv
                        sc.h = ops.conv3d_thin_op16(cur16, c.wp_fwd, c.cout, c.k, c.s, c.p, c.out_spatial(*cur16.shape[1:4]),
                                                    bias=bias, act=st.act)
                    else:
                        sc.h = st.conv.forward(cur, bias=bias, act=st.act)     # activated output
                    sc.out = ops.rpad(sc.h, ypad) if ypad else sc.h
            ctx.stages.append(sc)
            cur, cur16 = sc.out, out16
        ctx.out = cur
        return ctx

    def _in_bwd_plane_paths(self, st, sc):
        """(plane_bwd, plane_bwd_fwd, stem16): which 16-bit-plane backward a non-block stage with an
        InstanceNorm takes (all False otherwise) — its IN backward then writes dY only as the plane
        (and can take coefficients finalized in the producing launch).
        plane_bwd — G up1 / up2 (ABI 16): the data gradient (forward-form implicit GEMM) and the
        weight gradient (its gathered operand) read the plane;
        plane_bwd_fwd — G down1 / down2 (inputs only planes already): the weight gradient reads both
        planes, the data gradient (transposed implicit GEMM, or brickT for down1's 32 output
        channels) dY's;
        stem16 — the G stem (k7, nc → 32; ABI 17): its weight and data gradient (thinn_x3) read it."""
        if st.kind == "block" or st.norm is None:
            return False, False, False
        conv = st.conv
        op16 = self._op16_active()
        x_any = sc.inp if sc.inp is not None else sc.inp16
        plane_bwd = (x_any is not None and conv.transposed_plane_bwd_ok(x_any.shape[3])
                     and op16 and not _NO_S2_PLANES and not st.use_bias)
        plane_bwd_fwd = (sc.inp is None and sc.inp16 is not None and not st.use_bias
                         and not conv.transposed and conv.s2_plane_ok(sc.inp16.shape[3])
                         and (conv.cin != 32 or _BRICKT_PLANES) and op16 and not _NO_S2_PLANES)
        stem16 = (not plane_bwd and not plane_bwd_fwd and sc.inp is not None and op16 and conv.cout == 32
                  and conv.k7_wide16_ok())
        return plane_bwd, plane_bwd_fwd, stem16

    def _op16_active(self):
        """16-bit operand planes for the ResnetBlock section: bf16 / fp16 mode, not switched off."""
        return not _NO_OP16 and ops.op16_dtype() is not None

    def _op16_blocks_ok(self, W, H=None):
        """Every ResnetBlock conv can run on operand planes at block width W (height H)."""
        return all(st.conv1.op16_ok(W, H) and st.conv2.op16_ok(W, H) for st in self.stages if st.kind == "block")

    # ---- backward ----------------------------------------------------------------------
    def backward(self, ctx: NetCtx, dout: List[Optional[torch.Tensor]], need_wgrad: bool = True,
                 need_input_grad: bool = False, dx_out: Optional[torch.Tensor] = None,
                 dx_add: Optional[torch.Tensor] = None, wgrad_defer: Optional[dict] = None,
                 wgrad_pair: Optional[dict] = None) -> Optional[torch.Tensor]:
        """dout: up to 3 gradient sources w.r.t. ctx.out (summed).  Weight gradients are
        accumulated into the parameters' flat grad buffers.  Returns dL/dx (NDHWC) when
        need_input_grad (written to dx_out, plus dx_add if given).

        wgrad_defer / wgrad_pair (ABI 19): the reference accumulates a generator's weight gradient
        over its first pass and its cycle pass in one loss_G.backward() (cycle_gan_model.py:163-225).
        A pass given `wgrad_defer` (a dict) leaves the operand planes of its ResnetBlock weight
        gradients there instead of launching them; the other pass of the same network, given that
        dict as `wgrad_pair`, runs each of those convs' weight gradient once over both passes'
        instances (mragan_conv3d_wgrad_op16_pair: one launch + one reduce instead of two each).
        The caller keeps the dict's tensors alive until both passes' work is joined."""
        if _NO_WGRAD_DEFER:
            wgrad_defer = None

        def block_wgrad(conv, x16, dy16, key):
            if wgrad_defer is not None:
                wgrad_defer[key] = (conv, x16, dy16)
                return
            other = wgrad_pair.pop(key, None) if wgrad_pair is not None else None
            if other is not None:
                ops.conv3d_wgrad_op16_pair(dy16, x16, other[2], other[1], conv.k, conv.s, conv.p, conv.m.weight.grad,
                                           True)
            else:
                conv.wgrad_op16(x16, dy16)
        g, gpad, gadd = None, 0, None
        # (part, chunks, coef): backward statistics of the next IN from a data-gradient epilogue; coef =
        # its coefficients when that launch finalized them (ABI 15), else None
        bstats = None
        last = len(self.stages) - 1
        for i in range(last, -1, -1):
            st, sc = self.stages[i], ctx.stages[i]
            want_dgrad = i > 0 or need_input_grad
            if st.kind == "block" and sc.inp16 is not None:
                # 16-bit operand planes: the IN backwards write dY only as planes (the convs' sole use)
                skip = bstats if (bstats is not None and gpad == 1 and gadd is not None) else None
                own = bstats if (bstats is not None and gpad == 0 and gadd is None) else None
                bstats = None
                if gpad == 0 and gadd is None:
                    G = g
                    if own is not None:      # statistics from G up1's data-gradient epilogue
                        dh2 = ops.instnorm_bwd_partials_op16(sc.h, sc.mean, sc.rstd, G, 0, None, None, *own[:2],
                                                             coef=own[2])
                    else:
                        dh2 = ops.instnorm_bwd_op16(sc.h, sc.mean, sc.rstd, G, 0, None, act=None)
                elif skip is not None:
                    # statistics from the next block's conv1 data-gradient epilogue (ABI 18)
                    G = torch.empty(sc.h.shape, device=sc.h.device, dtype=torch.float32)
                    dh2 = ops.instnorm_bwd_partials_op16(sc.h, sc.mean, sc.rstd, g, gpad, gadd, None, skip[0], skip[1],
                                                         g_out=G, coef=skip[2])
                else:
                    G = torch.empty(sc.h.shape, device=sc.h.device, dtype=torch.float32)
                    dh2 = ops.instnorm_bwd_op16(sc.h, sc.mean, sc.rstd, g, gpad, gadd, act=None, g_out=G)
                if need_wgrad:
                    block_wgrad(st.conv2, sc.z1, dh2, (i, 2))
                # conv2's data gradient also accumulates IN1's backward statistics (ABI 11)
                if not _IN1_STATS_BIG and _dgrad_split(*dh2.shape):
                    dz1, part, chunks, coef = st.conv2.dgrad_op16(dh2, sc.z1.shape[1:4]), None, 0, None
                else:
                    dz1, part, chunks, coef = st.conv2.dgrad_op16_in_stats(dh2, sc.h1, sc.mean1, sc.rstd1, "relu")
                if chunks:
                    dh1 = ops.instnorm_bwd_partials_op16(sc.h1, sc.mean1, sc.rstd1, dz1, 1, None, "relu", part, chunks,
                                                         coef=coef)
                else:
                    dh1 = ops.instnorm_bwd_op16(sc.h1, sc.mean1, sc.rstd1, dz1, 1, None, act="relu")
                if need_wgrad:
                    block_wgrad(st.conv1, sc.inp16, dh1, (i, 1))
                nxt = self.stages[i - 1] if i > 0 else None
                nsc = ctx.stages[i - 1] if i > 0 else None
                # the IN in front: the previous block's IN2 (no activation), or G down2's IN + ReLU
                skip_in = nxt is not None and (
                    (nxt.kind == "block" and nsc.inp16 is not None)
                    or (nxt.kind != "block" and nxt.norm is not None and nsc.h is not None
                        and tuple(nsc.h.shape) == tuple(G.shape)))
                # (measured below 32³ only, DESIGN §4: gated on the voxel count, so a 16 × 64 × 64 block
                # takes the statistics pass like a 32³ one — ADVICE r05)
                if (skip_in and not _NO_IN_STATS and not _NO_SKIP_STATS
                        and dh1.shape[1] * dh1.shape[2] * dh1.shape[3] < 32 ** 3
                        and not _dgrad_split(*dh1.shape)
                        and (_SKIP_STATS_MAXN <= 0 or dh1.shape[0] <= _SKIP_STATS_MAXN)):
                    # conv1's data gradient also accumulates that IN's backward statistics, with this
                    # block's output gradient G joining at the skip (ABI 18)
                    act_in = None if nxt.kind == "block" else nxt.act
                    # finalized coefficients only for a consumer with an apply-only entry (the plane
                    # IN backwards): the fp32 one reduces the partials itself
                    fin = nxt.kind == "block" or any(self._in_bwd_plane_paths(nxt, nsc))
                    g, part, chunks, coef = st.conv1.dgrad_op16_in_stats_add(dh1, nsc.h, nsc.mean, nsc.rstd, act_in, G,
                                                                             fin=fin)
                    bstats = (part, chunks, coef) if chunks else None
                else:
                    g = st.conv1.dgrad_op16(dh1, sc.inp.shape[1:4])
                gpad, gadd = 1, G
                continue
            if st.kind == "block":
                if gpad == 0 and gadd is None:
                    G = g
                    dh2 = ops.instnorm_bwd(sc.h, sc.mean, sc.rstd, G, 0, None, act=None)
                else:
                    # the block-output gradient G = fold(g) + skip gradient is needed again below
                    # (the skip path): the IN backward writes it in the same pass
                    G = torch.empty(sc.h.shape, device=sc.h.device, dtype=torch.float32)
                    dh2 = ops.instnorm_bwd(sc.h, sc.mean, sc.rstd, g, gpad, gadd, act=None, g_out=G)
                if need_wgrad:
                    st.conv2.wgrad(sc.z1, dh2)
                dz1 = st.conv2.dgrad(dh2, sc.z1.shape[1:4])
                dh1 = ops.instnorm_bwd(sc.h1, sc.mean1, sc.rstd1, dz1, 1, None, act="relu")
                if need_wgrad:
                    st.conv1.wgrad(sc.inp, dh1)
                g = st.conv1.dgrad(dh1, sc.inp.shape[1:4])
                gpad, gadd = 1, G
                continue
            conv = st.conv
            x_any = sc.inp if sc.inp is not None else sc.inp16
            plane_bwd, plane_bwd_fwd, stem16 = self._in_bwd_plane_paths(st, sc)
            dh16 = None
            if plane_bwd or plane_bwd_fwd:
                if bstats is not None:
                    dh16 = ops.instnorm_bwd_partials_op16(sc.h, sc.mean, sc.rstd, g, gpad, gadd, st.act, *bstats[:2],
                                                          coef=bstats[2])
                else:
                    dh16 = ops.instnorm_bwd_op16(sc.h, sc.mean, sc.rstd, g, gpad, gadd, act=st.act)
                in_spatial = x_any.shape[1:4]
                if need_wgrad and plane_bwd and sc.inp is not None:
                    ops.conv3d_wgrad_g16(sc.inp, dh16, conv.k, conv.s, conv.p, conv.m.weight.grad, True)
                elif need_wgrad and plane_bwd:       # G up2 on up1's plane: both operands planes
                    ops.conv3d_wgrad_op16(sc.inp16, dh16, conv.k, conv.s, conv.p, conv.m.weight.grad, True)
                elif need_wgrad:
                    ops.conv3d_wgrad_op16(dh16, sc.inp16, conv.k, conv.s, conv.p, conv.m.weight.grad, True)
                bstats = None
                if want_dgrad:
                    nxt = self.stages[i - 1] if i > 0 else None
                    # the IN in front: a down / up conv's IN(+act), or (G up1) the last ResnetBlock's
                    # IN2 — no activation, no fold, its output gradient is this data gradient alone
                    blk_in = (nxt is not None and nxt.kind == "block" and ctx.stages[i - 1].inp16 is not None
                              and not _NO_SKIP_STATS and tuple(ctx.stages[i - 1].h.shape[1:4]) == tuple(in_spatial))
                    in_ok = blk_in or (nxt is not None and nxt.kind != "block" and nxt.norm is not None)
                    if in_ok and not st.prepad and conv.dgrad_bwd_stats_ok():
                        nsc = ctx.stages[i - 1]
                        part = ops.in_partials_buffer(dh16.shape[0], in_spatial, conv.cin, dh16.device)
                        g, bchunks = ops.conv3d_op16_bwd_stats(dh16, conv.wp_bwd, conv.cin, conv.k, conv.s, conv.p,
                                                               in_spatial, nsc.h, nsc.mean, nsc.rstd,
                                                               None if blk_in else nxt.act, part,
                                                               transposed=not conv.transposed)
                        bstats = (part, bchunks, None) if bchunks else None
                    else:
                        g = ops.conv3d_op16(dh16, conv.wp_bwd, conv.cin, conv.k, conv.s, conv.p, in_spatial, None,
                                            transposed=not conv.transposed)[0]
                    gpad, gadd = st.prepad, None
                continue
            if stem16:
                # the G stem (k7, nc → 32; ABI 17): its IN backward writes dx only as the plane — the
                # stem's weight gradient and data gradient (thinn_x3) are its only readers
                if bstats is not None:
                    dh16 = ops.instnorm_bwd_partials_op16(sc.h, sc.mean, sc.rstd, g, gpad, gadd, st.act, *bstats[:2],
                                                          coef=bstats[2])
                else:
                    dh16 = ops.instnorm_bwd_op16(sc.h, sc.mean, sc.rstd, g, gpad, gadd, act=st.act)
                bstats = None
                if need_wgrad:
                    ops.conv3d_wgrad_thin_op16(dh16, sc.inp, conv.k, conv.s, conv.p, conv.m.weight.grad, True)
                if want_dgrad:
                    g = ops.conv3d_thin_op16(dh16, conv.wp_bwd, conv.cin, conv.k, conv.s, conv.p, sc.inp.shape[1:4],
                                             transposed=True)
                    gpad, gadd = st.prepad, None
                continue
            if st.norm is not None:
                if bstats is not None:
                    # (no coefficients were asked for: this entry reduces the partials itself)
                    dh = ops.instnorm_bwd_partials(sc.h, sc.mean, sc.rstd, g, gpad, gadd, st.act, *bstats[:2])
                else:
                    dh = ops.instnorm_bwd(sc.h, sc.mean, sc.rstd, g, gpad, gadd, act=st.act)
            else:
                if i == last:
                    srcs = [t for t in dout if t is not None]
                elif gpad:
                    srcs = [ops.rpad_fold(g, gpad, add=gadd)]
                else:
                    srcs = [g, gadd]
                dh = torch.empty(sc.h.shape, device=sc.h.device, dtype=torch.float32)
                ops.act_bwd(sc.h, srcs, st.act, dh)
            in_spatial = (sc.inp if sc.inp is not None else sc.inp16).shape[1:4]
            if need_wgrad:
                if sc.inp is None:
                    conv.wgrad_g16(sc.inp16, dh)        # the input exists only as its plane
                else:
                    conv.wgrad(sc.inp, dh)
                if st.use_bias and conv.m.bias is not None:
                    ops.channel_sum(dh, conv.m.bias.grad, accumulate=True)
            bstats = None
            if want_dgrad:
                nxt = self.stages[i - 1] if i > 0 else None
                if (nxt is not None and nxt.kind != "block" and nxt.norm is not None and st.prepad
                        and conv.dgrad_in_stats_ok()):
                    # the G head: its data gradient also accumulates the last up-conv IN's backward
                    # statistics (the pad-3 statistics pass over dz and x goes)
                    nsc = ctx.stages[i - 1]
                    g, bpart, bchunks = conv.dgrad_in_stats(dh, in_spatial, nsc.h, nsc.mean, nsc.rstd, nxt.act,
                                                            st.prepad)
                    bstats = (bpart, bchunks, None) if bchunks else None
                elif (nxt is not None and nxt.kind != "block" and nxt.norm is not None and not st.prepad
                        and conv.dgrad_bwd_stats_ok()):
                    # stride-2 layers: the data gradient's epilogue accumulates the next IN's
                    # backward statistics (no fold: that IN's output is this conv's input)
                    nsc = ctx.stages[i - 1]
                    g, bpart, bchunks = conv.dgrad_bwd_stats(dh, in_spatial, nsc.h, nsc.mean, nsc.rstd, nxt.act)
                    bstats = (bpart, bchunks, None) if bchunks else None
                else:
                    g = conv.dgrad(dh, in_spatial)
                gpad, gadd = st.prepad, None
        if wgrad_pair:
            # deferred weight gradients this pass had no partner for (its blocks took another path)
            for conv, x16, dy16 in wgrad_pair.values():
                conv.wgrad_op16(x16, dy16)
            wgrad_pair.clear()
        if not need_input_grad:
            return None
        first = self.stages[0]
        if first.prepad:
            return ops.rpad_fold(g, first.prepad, add=dx_add, out=dx_out)
        if dx_add is not None or dx_out is not None:
            out = dx_out if dx_out is not None else torch.empty_like(g)
            ops.act_bwd(None, [g, dx_add], None, out)
            return out
        return g

    # ---- running statistics ------------------------------------------------------------
    def running_entries(self, segments):
        """segments: list of (NetCtx, row0, count) in the reference's call order.  Returns
        (norm, bias, C, S, [(mean_ptr, rstd_ptr, count)]) per IN layer."""
        entries = []
        si = 0
        layer_list = list(self.norms_in_order())
        for li, (st, norm, conv) in enumerate(layer_list):
            segs = []
            for ctx, row0, count in segments:
                sc, which = _locate(self, ctx, li)
                mean = sc.mean1 if which == 1 else sc.mean
                rstd = sc.rstd1 if which == 1 else sc.rstd
                h = sc.h1 if which == 1 else sc.h
                C_ = mean.shape[1]
                S = h.shape[1] * h.shape[2] * h.shape[3]
                segs.append((mean.data_ptr() + 4 * row0 * C_, rstd.data_ptr() + 4 * row0 * C_, count))
            bias = conv.m.bias
            entries.append((norm, bias, conv.cout, S, segs))
            si += 1
        return entries


def _locate(plan: NetPlan, ctx: NetCtx, norm_index: int):
    """Map the n-th InstanceNorm of the plan to (StageCtx, 1 for a block's first IN else 2/0)."""
    k = 0
    for st, sc in zip(plan.stages, ctx.stages):
        if st.kind == "block":
            if k == norm_index:
                return sc, 1
            if k + 1 == norm_index:
                return sc, 2
            k += 2
        elif st.norm is not None:
            if k == norm_index:
                return sc, 0
            k += 1
    raise IndexError(norm_index)


class _Seg(C.Structure):
    _fields_ = [("mean", C.c_void_p), ("rstd", C.c_void_p), ("count", C.c_int32), ("_pad", C.c_int32)]


class _Entry(C.Structure):
    _fields_ = [("rm", C.c_void_p), ("rv", C.c_void_p), ("bias", C.c_void_p), ("C", C.c_int32),
                ("nseg", C.c_int32), ("S", C.c_int64), ("seg", _Seg * 8)]


def apply_running_updates(entries, device):
    """Launch the running-stat update for a list of entries from NetPlan.running_entries."""
    if not entries:
        return
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("running-statistics update inside a HIP graph capture: launch it outside the graph "
                           "with a table from running_table()")
    dev = running_table(entries, device)
    launch_running_update(dev, len(entries))
    return dev   # keep alive until the stream consumed it (caller holds the reference)


def running_table(entries, device):
    """Device copy of the update table for `entries` (pointers only: reusable for as long as
    the tensors it points to live, e.g. across replays of a captured step)."""
    arr = (_Entry * len(entries))()
    for e, (norm, bias, C_, S, segs) in zip(arr, entries):
        if len(segs) > 8:
            raise ValueError("more than 8 IN calls per step for one layer")
        e.rm = norm.running_mean.data_ptr()
        e.rv = norm.running_var.data_ptr()
        e.bias = bias.data_ptr() if bias is not None else None
        e.C = C_
        e.nseg = len(segs)
        e.S = S
        for j, (mp, rp, cnt) in enumerate(segs):
            e.seg[j].mean = mp
            e.seg[j].rstd = rp
            e.seg[j].count = cnt
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.pin_memory().to(device, non_blocking=True)


def launch_running_update(table, n):
    call("mragan_instnorm_running_update", table.data_ptr(), n, C.c_float(IN_MOMENTUM),
         torch.cuda.current_stream().cuda_stream)


# --------------------------------------------------------------------------------------
# Plan compilation from the module trees in models/networks3D.py
# --------------------------------------------------------------------------------------

def compile_resnet_generator(net) -> NetPlan:
    from models import networks3D as N3
    stages: List[Stage] = []
    pending_pad = 0
    for m in net.model:
        if isinstance(m, N3.ReplicationPad3d):
            pending_pad = m.padding
        elif isinstance(m, N3.Conv3d):
            stages.append(Stage(kind="conv", conv=ConvLayer(m, False), prepad=pending_pad))
            pending_pad = 0
        elif isinstance(m, N3.ConvTranspose3d):
            stages.append(Stage(kind="conv", conv=ConvLayer(m, True), prepad=pending_pad))
            pending_pad = 0
        elif isinstance(m, N3.InstanceNorm3d):
            stages[-1].norm = m
        elif isinstance(m, (N3.ReLU, N3.LeakyReLU, N3.Tanh, N3.Sigmoid)):
            stages[-1].act = m.act_name
        elif isinstance(m, N3.ResnetBlock):
            cb = list(m.conv_block)
            convs = [c for c in cb if isinstance(c, N3.Conv3d)]
            norms = [c for c in cb if isinstance(c, N3.InstanceNorm3d)]
            if len(convs) != 2 or len(norms) != 2:
                raise NotImplementedError("ResnetBlock without two conv+InstanceNorm pairs")
            stages.append(Stage(kind="block", conv1=ConvLayer(convs[0], False), norm1=norms[0],
                                conv2=ConvLayer(convs[1], False), norm2=norms[1]))
        elif isinstance(m, N3.Dropout):
            raise NotImplementedError("dropout inside the generator is not supported by the HIP engine")
        else:
            raise NotImplementedError(f"generator layer {type(m).__name__} not supported by the HIP engine")
    for st in stages:
        if st.kind == "conv":
            st.use_bias = st.norm is None
    return NetPlan(stages, net.input_nc, net.output_nc)


def compile_nlayer_discriminator(net) -> NetPlan:
    from models import networks3D as N3
    stages: List[Stage] = []
    for m in net.model:
        if isinstance(m, N3.Conv3d):
            stages.append(Stage(kind="conv", conv=ConvLayer(m, False)))
        elif isinstance(m, N3.InstanceNorm3d):
            stages[-1].norm = m
        elif isinstance(m, (N3.ReLU, N3.LeakyReLU, N3.Tanh, N3.Sigmoid)):
            stages[-1].act = m.act_name
        else:
            raise NotImplementedError(f"discriminator layer {type(m).__name__} not supported by the HIP engine")
    for st in stages:
        st.use_bias = st.norm is None
    return NetPlan(stages, stages[0].conv.cin, stages[-1].conv.cout)


# --------------------------------------------------------------------------------------
# UnetGenerator (networks3D.py:270-343)
# --------------------------------------------------------------------------------------

@dataclass
class UnetLevel:
    """One UnetSkipConnectionBlock: `down` = Conv3d k4 s2 p1, `up` = ConvTranspose3d k4 s2 p1.
    kind "outer" (no norms, up has bias + Tanh), "mid" (down → IN, up → IN) or "inner"
    (down without norm, up → IN)."""
    kind: str
    down: ConvLayer
    up: ConvLayer
    down_norm: object = None
    up_norm: object = None


@dataclass
class UnetLevelCtx:
    inp: torch.Tensor = None        # level input: the image (outer) or LeakyReLU(x) = the skip tensor
    h: torch.Tensor = None          # down-conv output (mid: pre-IN; inner: ReLU'd)
    dmean: torch.Tensor = None
    drstd: torch.Tensor = None
    nxt: torch.Tensor = None        # input of the next level (LeakyReLU applied), outer/mid only
    r: torch.Tensor = None          # up-conv input: ReLU(cat(skip, sub)) (inner: ReLU(h))
    g: torch.Tensor = None          # up-conv output (pre-IN; outer: Tanh output)
    umean: torch.Tensor = None
    urstd: torch.Tensor = None
    ru: torch.Tensor = None         # ReLU(IN(g)): the sub-block half of the parent's cat, ReLU'd


class UnetPlan:
    """Explicit forward/backward of a UnetGenerator on NDHWC tensors.

    The reference's in-place activations define what every tensor holds
    (networks3D.py:318-343): a block's `downrelu` (LeakyReLU, inplace) rewrites its input x,
    which is also the tensor `torch.cat([x, model(x)], 1)` keeps as the skip, and the parent's
    `uprelu` (ReLU, inplace) acts on the concatenation.  So, level by level:

        a_{L+1} = LeakyReLU(IN(conv_down_L(a_L)))      (outer level: no IN, a_1 = LReLU(conv(x)))
        r_L     = cat(ReLU(a_{L+1}), ReLU(u_{L+1}))    u = IN(conv_up(r)) of the level below
        inner:  r = ReLU(conv_down(a));  u = IN(conv_up(r))
        outer:  out = Tanh(conv_up(r_0) + b)

    Activations are fused into the producing conv / InstanceNorm kernel; the concatenation
    and its backward are `channel_concat` / `channel_split`."""

    def __init__(self, levels: List[UnetLevel], in_channels: int, out_channels: int):
        self.levels = levels
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.dirty = True

    def conv_layers(self):
        for lv in self.levels:
            yield lv.down
            yield lv.up

    def repack(self):
        """Every conv layer's two packs in one launch (after each optimizer step)."""
        if not hasattr(self, "_pack_table"):
            self._pack_table = ops.PackTable()
        self._packed_prec = ops.get_conv_precision()
        self._pack_table.run([p for c in self.conv_layers() for p in c.packs()])
        self.dirty = False

    def ensure_packed(self):
        if self.dirty or getattr(self, "_packed_prec", None) != ops.get_conv_precision():
            self.repack()

    def _norms(self):
        """(norm, conv, ctx getter) for every InstanceNorm, in module order."""
        out = []
        for i, lv in enumerate(self.levels):
            if lv.down_norm is not None:
                out.append((lv.down_norm, lv.down, i, "down"))
            if lv.up_norm is not None:
                out.append((lv.up_norm, lv.up, i, "up"))
        return out

    @staticmethod
    def _check_spatial(x_shape, levels):
        """The reference fails on these inputs too: a conv with an empty output, or an
        InstanceNorm over a single voxel (torch's message)."""
        d, h, w = x_shape[1:4]
        for lv in levels:
            d, h, w = lv.down.out_spatial(d, h, w)
            if min(d, h, w) < 1:
                raise RuntimeError("UnetGenerator: input too small for its number of downsamplings "
                                   f"(a Conv3d k4 s2 output would be {d}x{h}x{w})")
            if lv.down_norm is not None and d * h * w == 1:
                raise ValueError("Expected more than 1 spatial element when training, got input size "
                                 f"[{x_shape[0]}, {lv.down.cout}, 1, 1, 1]")

    def forward(self, x: torch.Tensor) -> NetCtx:
        self.ensure_packed()
        N, D, H, W, Cin = x.shape
        if Cin != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {Cin}")
        self._check_spatial(x.shape, self.levels)
        ctx = NetCtx(N=N, spatial=(D, H, W))
        cur = x
        for lv in self.levels:                      # encoder
            lc = UnetLevelCtx(inp=cur)
            sp = lv.down.out_spatial(*cur.shape[1:4])
            if lv.kind == "outer":
                lc.nxt = lv.down.forward(cur, act="lrelu")
            elif lv.kind == "mid":
                lc.h = lv.down.forward(cur)
                lc.nxt, lc.dmean, lc.drstd = ops.instnorm_fwd(lc.h, act="lrelu")
            else:
                lc.h = lv.down.forward(cur, act="relu")
                lc.r = lc.h
            assert tuple(sp) == tuple((lc.nxt if lc.nxt is not None else lc.h).shape[1:4])
            ctx.stages.append(lc)
            cur = lc.nxt
        for i in range(len(self.levels) - 1, -1, -1):   # decoder
            lv, lc = self.levels[i], ctx.stages[i]
            if lv.kind != "inner":
                below = ctx.stages[i + 1]
                lc.r = ops.channel_concat(below.inp, "relu", below.ru, None)
            lc.g = lv.up.forward(lc.r, bias=lv.up.m.bias if lv.kind == "outer" else None,
                                 act="tanh" if lv.kind == "outer" else None)
            if lv.kind != "outer":
                lc.ru, lc.umean, lc.urstd = ops.instnorm_fwd(lc.g, act="relu")
        ctx.out = ctx.stages[0].g
        return ctx

    def backward(self, ctx: NetCtx, dout: List[Optional[torch.Tensor]], need_wgrad: bool = True,
                 need_input_grad: bool = False, dx_out: Optional[torch.Tensor] = None,
                 dx_add: Optional[torch.Tensor] = None, wgrad_defer: Optional[dict] = None,
                 wgrad_pair: Optional[dict] = None) -> Optional[torch.Tensor]:
        """Same contract as NetPlan.backward (no ResnetBlocks: wgrad_defer / wgrad_pair stay empty,
        every weight gradient runs in its pass)."""
        n = len(self.levels)
        skip = [None] * (n + 1)        # gradient w.r.t. level i's input through the skip half of the cat
        du = [None] * (n + 1)          # gradient w.r.t. ReLU(u_i) (raw, the IN backward applies ReLU')
        for i, (lv, lc) in enumerate(zip(self.levels, ctx.stages)):    # decoder, top-down
            if lv.kind == "outer":
                srcs = [t for t in dout if t is not None]
                dg = torch.empty_like(lc.g)
                ops.act_bwd(lc.g, srcs, "tanh", dg)
                if need_wgrad and lv.up.m.bias is not None:
                    ops.channel_sum(dg, lv.up.m.bias.grad, accumulate=True)
            else:
                dg = ops.instnorm_bwd(lc.g, lc.umean, lc.urstd, du[i], 0, None, act="relu")
            if need_wgrad:
                lv.up.wgrad(lc.r, dg)
            dr = lv.up.dgrad(dg, lc.r.shape[1:4])
            if lv.kind == "inner":
                dh = torch.empty_like(lc.h)
                ops.act_bwd(lc.h, [dr], "relu", dh)
                ctx_inner_dh = dh
            else:
                below = ctx.stages[i + 1]
                skip[i + 1], du[i + 1] = ops.channel_split(dr, below.inp.shape[4], below.inp, "relu", None, None)
        g_in = None                    # gradient w.r.t. the current level's input through its down conv
        for i in range(n - 1, -1, -1):                                  # encoder, bottom-up
            lv, lc = self.levels[i], ctx.stages[i]
            if lv.kind == "inner":
                dh = ctx_inner_dh
            elif lv.kind == "mid":
                dh = ops.instnorm_bwd(lc.h, lc.dmean, lc.drstd, g_in, 0, skip[i + 1], act="lrelu")
            else:
                dh = torch.empty_like(lc.nxt)
                ops.act_bwd(lc.nxt, [g_in, skip[i + 1]], "lrelu", dh)
            if need_wgrad:
                lv.down.wgrad(lc.inp, dh)
            if i > 0 or need_input_grad:
                g_in = lv.down.dgrad(dh, lc.inp.shape[1:4])
        if not need_input_grad:
            return None
        if dx_add is not None or dx_out is not None:
            out = dx_out if dx_out is not None else torch.empty_like(g_in)
            ops.act_bwd(None, [g_in, dx_add], None, out)
            return out
        return g_in

    def running_entries(self, segments):
        entries = []
        for norm, conv, i, which in self._norms():
            segs = []
            for ctx, row0, count in segments:
                lc = ctx.stages[i]
                mean, rstd, h = (lc.dmean, lc.drstd, lc.h) if which == "down" else (lc.umean, lc.urstd, lc.g)
                C_ = mean.shape[1]
                S = h.shape[1] * h.shape[2] * h.shape[3]
                segs.append((mean.data_ptr() + 4 * row0 * C_, rstd.data_ptr() + 4 * row0 * C_, count))
            entries.append((norm, conv.m.bias, conv.cout, S, segs))
        return entries


def compile_unet_generator(net) -> UnetPlan:
    from models import networks3D as N3
    levels: List[UnetLevel] = []
    blk = net.model
    while blk is not None:
        seq = list(blk.model)
        if any(isinstance(m, N3.Dropout) for m in seq):
            raise NotImplementedError("dropout inside the generator is not supported by the HIP engine")
        down = next(m for m in seq if isinstance(m, N3.Conv3d))
        up = next(m for m in seq if isinstance(m, N3.ConvTranspose3d))
        norms = [m for m in seq if isinstance(m, N3.InstanceNorm3d)]
        kind = "outer" if blk.outermost else ("inner" if blk.innermost else "mid")
        lv = UnetLevel(kind=kind, down=ConvLayer(down, False), up=ConvLayer(up, True))
        if kind == "mid":
            lv.down_norm, lv.up_norm = norms
        elif kind == "inner":
            lv.up_norm = norms[0]
        levels.append(lv)
        sub = [m for m in seq if isinstance(m, N3.UnetSkipConnectionBlock)]
        blk = sub[0] if sub else None
    if levels[0].kind != "outer" or levels[-1].kind != "inner":
        raise NotImplementedError("UnetGenerator must run outermost → innermost")
    return UnetPlan(levels, net.input_nc, net.output_nc)
