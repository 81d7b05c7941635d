"""Per-kernel parity: every HIP entry point (through the C ABI) against a float64 PyTorch-CPU
evaluation of the same op.  Tolerances are relative L2 errors; fp32 kernels reach ~1e-6, the
gate is 1e-5 (SURVEY §8c per-op gate)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 1e-5


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def ndhwc(t):          # NCDHW → NDHWC contiguous
    return t.permute(0, 2, 3, 4, 1).contiguous()


def ncdhw(t):
    return t.permute(0, 4, 1, 2, 3)


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mragan_hip import ops as _ops
    # a model built in another test file (fp16: loss scale 1024) leaves the process-wide state set
    _ops.set_conv_precision("f32")
    _ops.set_loss_scale(1.0)
    return _ops


def pack(ops, w, transposed_layer, for_dgrad):
    """Pack a torch-layout weight the way engine.ConvLayer does."""
    w = w.float().cuda().contiguous()
    k = w.shape[2]
    out = torch.empty(w.numel(), device="cuda")
    A, B = w.shape[0], w.shape[1]
    tr = (not transposed_layer) == for_dgrad
    ops.pack_weight(w, A, B, k ** 3, tr, out)
    return out


CONV_CASES = [
    # N, cin, cout, S, k, s, p     (generic MFMA path: cin % 8 == 0, cout > 4)
    (2, 32, 64, 12, 3, 2, 1),
    (1, 64, 128, 8, 3, 2, 1),
    (2, 128, 128, 6, 3, 1, 0),
    (1, 32, 64, 10, 4, 2, 1),
    (2, 128, 256, 5, 4, 1, 1),
    (1, 8, 16, 9, 3, 2, 1),
    (3, 16, 24, 7, 3, 1, 1),
    (1, 24, 40, 6, 4, 2, 1),
    (2, 64, 128, 13, 3, 1, 1),      # k3 s1 halo-brick path (conv_brick.hip), zero pad, 2 chunks
    # thin paths
    (2, 1, 32, 14, 7, 1, 0),
    (1, 2, 32, 12, 7, 1, 0),
    (2, 32, 1, 14, 7, 1, 0),
    (1, 32, 2, 12, 7, 1, 0),
    (2, 1, 32, 16, 4, 2, 1),
    (1, 2, 16, 12, 4, 2, 1),
    (2, 256, 1, 7, 4, 1, 1),
    (1, 64, 1, 6, 4, 1, 1),
    (4, 512, 1, 7, 4, 1, 1),        # D last at 64³ (thin_dot)
    (2, 256, 1, 15, 4, 1, 1),       # D last at 128³ (ndf 32: 5,488 outputs, thin_dot — was thin_n, 535 µs)
    (1, 64, 2, 6, 4, 1, 1),
    # ngf = 4 generators (thin_k with a cut weight slice: cin ≤ 4, k7, few output channels)
    (1, 4, 1, 12, 7, 1, 0),
    (1, 4, 2, 11, 7, 1, 0),
    (1, 4, 4, 10, 7, 1, 0),
    # large enough for the row-sweep thin_n kernel (fwd: ≥ 4096 output voxels; dgrad likewise)
    (1, 32, 1, 22, 7, 1, 0),
    (1, 16, 2, 21, 7, 1, 0),
    (1, 8, 1, 20, 4, 1, 1),
    (2, 2, 32, 20, 7, 1, 0),
    # nc = 2 stem / head at sizes past one 16×16 tile (thin1 ring with two channels, thinn with two
    # output channels in the one-plane modes)
    (2, 2, 32, 23, 7, 1, 0),
    (1, 32, 2, 23, 7, 1, 0),
    # UnetGenerator downconvs (k4 s2 p1): stem nc→ngf, down to a 1³ innermost output
    (2, 1, 8, 16, 4, 2, 1),
    (1, 64, 64, 2, 4, 2, 1),
    (2, 16, 32, 8, 4, 2, 1),
]


@pytest.mark.parametrize("N,cin,cout,S,k,s,p", CONV_CASES)
@pytest.mark.parametrize("act", [None, "lrelu", "tanh", "sigmoid"])
def test_conv3d_fwd(ops, N, cin, cout, S, k, s, p, act):
    g = torch.Generator().manual_seed(N * 1000 + cin * 7 + cout)
    x = torch.randn(N, cin, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(cout, generator=g, dtype=torch.float64)
    ref = F.conv3d(x, w, b, stride=s, padding=p)
    if act == "lrelu":
        ref = F.leaky_relu(ref, 0.2)
    elif act == "tanh":
        ref = torch.tanh(ref)
    elif act == "sigmoid":
        ref = torch.sigmoid(ref)
    wp = pack(ops, w, False, False)
    out = ops.conv3d(ndhwc(x.float()).cuda(), wp, cout, k, s, p, ref.shape[2:], bias=b.float().cuda(), act=act)
    assert rel(ncdhw(out), ref) < TOL


@pytest.mark.parametrize("N,cin,cout,S,k,s,p", CONV_CASES)
def test_conv3d_dgrad(ops, N, cin, cout, S, k, s, p):
    """Input gradient of a forward conv = transposed-form kernel with the dgrad packing."""
    g = torch.Generator().manual_seed(7 + N * 100 + cin + cout)
    x = torch.randn(N, cin, S, S + 1, S + 2, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) * 0.1
    y = F.conv3d(x, w, stride=s, padding=p)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (dx_ref,) = torch.autograd.grad(y, x, dy)
    wp = pack(ops, w, False, True)
    dx = ops.conv3d(ndhwc(dy.float()).cuda(), wp, cin, k, s, p, x.shape[2:], transposed=True)
    assert rel(ncdhw(dx), dx_ref) < TOL


@pytest.mark.parametrize("N,cin,cout,S,k,s,p", CONV_CASES)
def test_conv3d_wgrad(ops, N, cin, cout, S, k, s, p):
    g = torch.Generator().manual_seed(11 + N * 10 + cin + cout)
    x = torch.randn(N, cin, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = (torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    y = F.conv3d(x, w, stride=s, padding=p)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (dw_ref,) = torch.autograd.grad(y, w, dy)
    dw = torch.full((cout, cin, k, k, k), 3.0, device="cuda")
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), k, s, p, dw, accumulate=False)
    assert rel(dw, dw_ref) < TOL
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), k, s, p, dw, accumulate=True)
    assert rel(dw, 2 * dw_ref) < TOL


CONVT_CASES = [
    # N, cin, cout, S, k, s, p, op
    (2, 128, 64, 6, 3, 2, 1, 1),
    (1, 64, 32, 8, 3, 2, 1, 1),
    (1, 16, 8, 5, 3, 2, 1, 1),
    (2, 32, 16, 4, 4, 2, 1, 0),
    (1, 24, 32, 5, 3, 1, 1, 0),
    # UnetGenerator upconvs (k4 s2 p1): innermost 1³ → 2³, middle, outermost 2ngf → nc (thin)
    (2, 64, 64, 1, 4, 2, 1, 0),
    (1, 128, 32, 4, 4, 2, 1, 0),
    (2, 16, 1, 8, 4, 2, 1, 0),
    (1, 16, 2, 6, 4, 2, 1, 0),
    # thin_n_class8 (≤ 4 outputs, ≤ 32 contraction channels, ceil(k/s) = 2): the D-first
    # data-gradient shape (32 → 1, k4 s2 p1), partial lane groups, k3 s2 with output padding, 4
    # outputs; 64 / 40 channels take thin_n_class
    (2, 32, 1, 9, 4, 2, 1, 0),
    (1, 24, 3, 4, 3, 2, 1, 1),
    (2, 8, 4, 5, 4, 2, 1, 0),
    (1, 64, 2, 5, 4, 2, 1, 0),
    (1, 40, 3, 4, 3, 2, 1, 1),
]


@pytest.mark.parametrize("N,cin,cout,S,k,s,p,op", CONVT_CASES)
def test_conv_transpose3d_fwd_dgrad_wgrad(ops, N, cin, cout, S, k, s, p, op):
    g = torch.Generator().manual_seed(N + cin + 3 * cout)
    x = torch.randn(N, cin, S, S + 1, S, generator=g, dtype=torch.float64, requires_grad=True)
    w = (torch.randn(cin, cout, k, k, k, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    y = F.conv_transpose3d(x, w, stride=s, padding=p, output_padding=op)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dx_ref, dw_ref = torch.autograd.grad(y, (x, w), dy)
    xg = ndhwc(x.detach().float()).cuda()
    out = ops.conv3d(xg, pack(ops, w.detach(), True, False), cout, k, s, p, y.shape[2:], transposed=True)
    assert rel(ncdhw(out), y.detach()) < TOL
    dx = ops.conv3d(ndhwc(dy.float()).cuda(), pack(ops, w.detach(), True, True), cin, k, s, p, x.shape[2:])
    assert rel(ncdhw(dx), dx_ref) < TOL
    dw = torch.empty(cin, cout, k, k, k, device="cuda")
    ops.conv3d_wgrad(xg, ndhwc(dy.float()).cuda(), k, s, p, dw, accumulate=False)
    assert rel(dw, dw_ref) < TOL


X3_TOL = 2e-5     # bf16x3: ≤ 3·2⁻¹⁸ relative per product, random → ~5e-6 rel-L2 measured scale
# bf16 / fp16: every operand is rounded once (RNE) and the products of the rounded operands are
# exact in fp32, so the kernel must equal the fp64 convolution of the ROUNDED operands up to fp32
# accumulation order (~1e-6 rel-L2): same gate as bf16x3.  The unrounded fp64 result is a further
# check that the rounding happened (unit roundoff 2⁻⁸ / 2⁻¹¹ moves a long random sum by ≥ 1e-3 /
# 1e-4 rel-L2).
MODE_TOL = {"bf16x3": X3_TOL, "bf16": X3_TOL, "fp16": X3_TOL}
ROUNDED_MIN_DIFF = {"bf16": 1e-3, "fp16": 1e-4}


def xtol():
    from mragan_hip import ops
    return MODE_TOL[ops.get_conv_precision()]


def R(t):
    """An operand as the current contraction mode feeds it to the products: bf16 / fp16 round
    (RNE) the fp32 value, the fp32-grade modes keep it (include/mragan_hip.h, ABI 10)."""
    from mragan_hip import ops
    mode = ops.get_conv_precision()
    t32 = t.detach().float()
    if mode == "bf16":
        return t32.to(torch.bfloat16).double()
    if mode == "fp16":
        return t32.to(torch.float16).double()
    return t32.double()


def check_rounded(got, ref_rounded, ref_exact):
    """got vs the fp64 result on rounded operands; in bf16 / fp16 also far from the unrounded one."""
    from mragan_hip import ops
    mode = ops.get_conv_precision()
    assert rel(got, ref_rounded) < MODE_TOL[mode]
    if mode in ROUNDED_MIN_DIFF:
        assert rel(got, ref_exact) > ROUNDED_MIN_DIFF[mode], "operands were not rounded"

@pytest.mark.parametrize("N,cin,cout,S,k", [(2, 64, 1, 8, 4), (1, 64, 2, 5, 4), (1, 48, 1, 6, 4), (1, 64, 1, 7, 3)])
def test_thin_class8_wide_modes(x3, N, cin, cout, S, k):
    """The UNet outermost upconv shape (2·ngf = 64 → nc, ConvTranspose3d k4 s2 p1; networks3D.py
    UnetSkipConnectionBlock outermost) on thin_n_class8 with two channel quads per lane in the MFMA
    modes (round 4; it took 262 µs per launch on thin_n_class): the fp64 result on the mode's
    rounded operands."""
    ops = x3
    g = torch.Generator().manual_seed(N * 3 + cin + cout + S)
    x = torch.randn(N, cin, S, S + 1, S, generator=g, dtype=torch.float64)
    w = torch.randn(cin, cout, k, k, k, generator=g, dtype=torch.float64) * 0.1
    op = 1 if k == 3 else 0
    y = F.conv_transpose3d(x, w, stride=2, padding=1, output_padding=op)
    y_r = F.conv_transpose3d(R(x), R(w), stride=2, padding=1, output_padding=op)
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, True, False), cout, k, 2, 1, y.shape[2:], transposed=True)
    check_rounded(ncdhw(out), y_r, y)


@pytest.mark.parametrize("N,cin,cout,dims,act,bias", [
    (2, 64, 1, (8, 8, 8), "tanh", True),        # UNet outermost upconv (2·ngf → nc, + bias, Tanh)
    (1, 64, 2, (5, 6, 7), "tanh", True),        # nc = 2, partial output bricks
    (2, 32, 1, (9, 8, 10), None, False),        # D-first data gradient shape (ndf → nc)
    (1, 32, 2, (4, 4, 4), None, False),
    (2, 64, 1, (2, 2, 3), None, True),          # smaller than one brick: most of the halo is padding
])
def test_up4_mfma(x3, N, cin, cout, dims, act, bias):
    """ConvTranspose3d k4 s2 p1 to ≤ 2 channels (conv_up4.hip, the one-plane modes' MFMA path;
    bf16x3 keeps thin_n_tile8): the fp64 transposed convolution of the mode's rounded operands,
    bias and activation after."""
    ops = x3
    g = torch.Generator().manual_seed(N * 5 + cin + cout + sum(dims))
    x = torch.randn(N, cin, *dims, generator=g, dtype=torch.float64)
    w = torch.randn(cin, cout, 4, 4, 4, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(cout, generator=g, dtype=torch.float64) if bias else None
    f = {None: lambda t: t, "tanh": torch.tanh}[act]
    y = f(F.conv_transpose3d(x, w, b, stride=2, padding=1))
    y_r = f(F.conv_transpose3d(R(x), R(w), b, stride=2, padding=1))
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, True, False), cout, 4, 2, 1, y.shape[2:],
                     bias=b.float().cuda() if bias else None, act=act, transposed=True)
    check_rounded(ncdhw(out), y_r, y)


@pytest.mark.parametrize("N,cin,cout,dims,act,bias", [
    (2, 1, 32, (16, 16, 32), "lrelu", True),    # PatchGAN first layer / UNet outermost downconv
    (1, 2, 32, (10, 18, 22), "lrelu", True),    # nc = 2, partial output bricks
    (1, 1, 64, (12, 10, 8), None, False),       # UNet outermost upconv's data gradient (1 → 2·ngf)
    (2, 2, 64, (4, 6, 2), None, True),          # smaller than one brick
])
def test_down4_mfma(x3, N, cin, cout, dims, act, bias):
    """Conv3d k4 s2 p1 from 1-2 channels (conv_down4.hip, the one-plane modes' MFMA path; bf16x3
    keeps thin_k): the fp64 convolution of the mode's rounded operands, bias and activation after."""
    ops = x3
    g = torch.Generator().manual_seed(N * 3 + cin + cout + sum(dims))
    x = torch.randn(N, cin, *dims, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, 4, 4, 4, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(cout, generator=g, dtype=torch.float64) if bias else None
    f = {None: lambda t: t, "lrelu": lambda t: F.leaky_relu(t, 0.2)}[act]
    y = f(F.conv3d(x, w, b, stride=2, padding=1))
    y_r = f(F.conv3d(R(x), R(w), b, stride=2, padding=1))
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, False, False), cout, 4, 2, 1, y.shape[2:],
                     bias=b.float().cuda() if bias else None, act=act)
    check_rounded(ncdhw(out), y_r, y)


X3_CASES = [
    # N, cin, cout, S, k, s, p   (every tile shape of conv_igemm_x3.hip's dispatch)
    (2, 128, 128, 6, 3, 1, 0),
    (8, 128, 128, 18, 3, 1, 0),     # 128x128 tiles
    (4, 128, 128, 16, 3, 1, 0),     # 128x64 tiles
    (2, 32, 64, 12, 3, 2, 1),
    (4, 64, 128, 16, 3, 2, 1),
    (2, 128, 256, 5, 4, 1, 1),
    (3, 16, 24, 7, 3, 1, 1),        # BK = 16
    (2, 64, 32, 20, 4, 2, 1),       # ny = 32 tiles
    (4, 64, 128, 16, 4, 2, 1),      # PatchGAN layer 3 shape: split-K + deterministic reduce
    (4, 128, 256, 8, 4, 1, 1),      # PatchGAN layer 4 shape: split-K
]


@pytest.fixture(params=["bf16x3", "bf16", "fp16"])
def x3(ops, request):
    """Every MFMA kernel in each of its three 16-bit operand modes (prec.h)."""
    ops.set_conv_precision(request.param)
    assert ops.get_conv_precision() == request.param
    yield ops
    ops.set_conv_precision("f32")


@pytest.mark.parametrize("N,cin,cout,S,k,s,p", X3_CASES)
def test_conv3d_bf16x3_fwd_dgrad(x3, N, cin, cout, S, k, s, p):
    ops = x3
    g = torch.Generator().manual_seed(5 + N * 100 + cin + cout)
    x = torch.randn(N, cin, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(cout, generator=g, dtype=torch.float64)
    y = F.conv3d(x, w, b, stride=s, padding=p)
    yr = F.conv3d(R(x), R(w), b.float().double(), stride=s, padding=p)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dx_ref = torch.nn.grad.conv3d_input(x.shape, w, dy, stride=s, padding=p)
    dx_rnd = torch.nn.grad.conv3d_input(x.shape, R(w), R(dy), stride=s, padding=p)
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, False, False), cout, k, s, p, y.shape[2:],
                     bias=b.float().cuda(), act="lrelu")
    check_rounded(ncdhw(out), F.leaky_relu(yr, 0.2), F.leaky_relu(y, 0.2))
    dx = ops.conv3d(ndhwc(dy.float()).cuda(), pack(ops, w, False, True), cin, k, s, p, x.shape[2:], transposed=True)
    check_rounded(ncdhw(dx), dx_rnd, dx_ref)


def test_splitk_in_launch_reduce_bit_identical(ops, tmp_path):
    """Round 6, opt-in (MRAGAN_SK_FUSE=1, run in a child process): the implicit GEMM's split-K
    slices reduce in the launch (the last slice of a tile, by ticket, sums the slabs in slice order)
    — bit-identical to the separate conv_splitk_reduce launch of the default path, in every mode,
    on the PatchGAN and UNet split-K shapes (forward with bias + LeakyReLU, and the transposed k4 s2
    form); its InstanceNorm partials match the statistics pass."""
    import os
    import subprocess
    import sys
    g = torch.Generator().manual_seed(606)
    cases = []
    for prec in ("bf16x3", "bf16", "fp16"):
        for N, cin, cout, S, k, s, p, tr, act in [(4, 64, 128, 16, 4, 2, 1, False, "lrelu"),   # PatchGAN layer 3
                                                  (4, 128, 256, 8, 4, 1, 1, False, "lrelu"),   # PatchGAN layer 4
                                                  (1, 256, 256, 8, 4, 2, 1, False, "none"),    # UNet inner down
                                                  (2, 128, 64, 8, 4, 2, 1, True, "none")]:     # UNet up (convT)
            x = torch.randn(N, S, S, S, cin, generator=g)
            if tr:
                w = pack(ops, torch.randn(cin, cout, k, k, k, generator=g, dtype=torch.float64) * 0.05, True, False)
                o = ops.convT_out_size(S, k, s, p, 0)
            else:
                w = pack(ops, torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) * 0.05, False, False)
                o = ops.conv_out_size(S, k, s, p)
            b = torch.randn(cout, generator=g) if act != "none" else None
            cases.append(dict(prec=prec, x=x, w=w.cpu(), b=b, cout=cout, k=k, s=s, p=p, osp=[o, o, o], act=act, tr=tr,
                              stats=(act == "none" and not tr)))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _splitk_child
    mine = _splitk_child.run(ops, cases)
    fin, fout = tmp_path / "in.pt", tmp_path / "out.pt"
    torch.save(cases, fin)
    env = dict(os.environ, MRAGAN_SK_FUSE="1")
    subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "_splitk_child.py"),
                    str(fin), str(fout)], env=env, check=True, timeout=300)
    fused = torch.load(fout, weights_only=True)
    assert len(fused) == len(mine)
    i = 0
    for c in cases:
        a, b = mine[i], fused[i]
        assert torch.isfinite(a).all()
        assert torch.equal(a, b), (c["prec"], c["x"].shape, c["cout"], c["tr"])
        i += 1
        if c["stats"]:
            assert float(fused[i]) > 0 and float(mine[i]) == 0       # partials only from the fused launch
            ops.set_conv_precision(c["prec"])
            _, m_ref, r_ref = ops.instnorm_fwd(a.cuda(), act="lrelu", ypad=1)   # statistics pass
            ops.set_conv_precision("f32")
            assert rel(fused[i + 1], m_ref) < 1e-6 and rel(fused[i + 2], r_ref) < 1e-6
            i += 3


@pytest.mark.parametrize("N,cin,cout,S,k,s,p", X3_CASES + [(2, 32, 32, 9, 3, 1, 1), (1, 64, 256, 6, 4, 1, 1),
                                                   (2, 64, 32, 10, 3, 2, 1), (3, 32, 64, 11, 3, 2, 1),
                                                   # one split (the UNet's inner layers)
                                                   (1, 256, 256, 4, 4, 2, 1), (2, 128, 64, 5, 4, 2, 1),
                                                   (1, 96, 160, 3, 3, 1, 1)])
def test_conv3d_bf16x3_wgrad(x3, N, cin, cout, S, k, s, p):
    ops = x3
    g = torch.Generator().manual_seed(13 + N * 10 + cin + cout)
    x = torch.randn(N, cin, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) * 0.1
    y = F.conv3d(x, w, stride=s, padding=p)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dw_ref = torch.nn.grad.conv3d_weight(x, w.shape, dy, stride=s, padding=p)
    dw_rnd = torch.nn.grad.conv3d_weight(R(x), w.shape, R(dy), stride=s, padding=p)
    dw = torch.full((cout, cin, k, k, k), 3.0, device="cuda")
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), k, s, p, dw, accumulate=False)
    check_rounded(dw, dw_rnd, dw_ref)
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), k, s, p, dw, accumulate=True)
    check_rounded(dw, 2 * dw_rnd, 2 * dw_ref)


@pytest.mark.parametrize("N,cin,cout,dims", [(1, 32, 64, (8, 10, 32)), (2, 64, 128, (6, 4, 64)), (1, 32, 128, (4, 2, 32)),
                                             (3, 64, 64, (2, 6, 32)),
                                             # aligned stages (whole coarse rows per 8-segment stage)
                                             (1, 32, 64, (4, 16, 32)), (2, 64, 128, (4, 8, 64)),
                                             (1, 32, 64, (6, 16, 64)),
                                             # 8-voxel segments (coarse w 8 / 24: one-plane modes)
                                             (1, 32, 64, (8, 6, 16)), (2, 64, 128, (16, 16, 16)),
                                             (1, 32, 64, (4, 6, 48))])
def test_wgrad_s2_three_tap(x3, N, cin, cout, dims):
    """Weight gradients of the k3 s2 p1 down convs (networks3D.py:192-197) and of the transposed
    up convs (op 1, networks3D.py:203-210) on the 3-kw-tap even/odd-phase kernel
    (conv_wgrad3s2_x3.hip: even fine grid, coarse w a multiple of 16; 32- and 64-channel G tiles,
    several split-K slabs and D tiles), vs fp64."""
    ops = x3
    g = torch.Generator().manual_seed(17 + N + cin + cout)
    x = torch.randn(N, cin, *dims, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g, dtype=torch.float64) * 0.1
    y = F.conv3d(x, w, stride=2, padding=1)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dw_ref = torch.nn.grad.conv3d_weight(x, w.shape, dy, stride=2, padding=1)
    dw_rnd = torch.nn.grad.conv3d_weight(R(x), w.shape, R(dy), stride=2, padding=1)
    dw = torch.full((cout, cin, 3, 3, 3), 3.0, device="cuda")
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), 3, 2, 1, dw, accumulate=False)
    check_rounded(dw, dw_rnd, dw_ref)
    # transposed: ConvTranspose3d(cout → cin) on the coarse grid of y, output padding 1
    xt = torch.randn(y.shape, generator=g, dtype=torch.float64)
    wt = (torch.randn(cout, cin, 3, 3, 3, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    yt = F.conv_transpose3d(xt, wt, stride=2, padding=1, output_padding=1)
    assert tuple(yt.shape[2:]) == tuple(dims)
    dyt = torch.randn(yt.shape, generator=g, dtype=torch.float64)
    (dwt_ref,) = torch.autograd.grad(yt, wt, dyt)
    xr = R(xt).requires_grad_()
    wr = R(wt).requires_grad_()
    (dwt_rnd,) = torch.autograd.grad(F.conv_transpose3d(xr, wr, stride=2, padding=1, output_padding=1), wr, R(dyt))
    dwt = torch.zeros((cout, cin, 3, 3, 3), device="cuda")
    ops.conv3d_wgrad(ndhwc(xt.float()).cuda(), ndhwc(dyt.float()).cuda(), 3, 2, 1, dwt, accumulate=False)
    check_rounded(dwt, dwt_rnd, dwt_ref)


@pytest.mark.parametrize("N,cin,cout,dims", [(1, 32, 64, (8, 10, 32)), (2, 64, 128, (6, 4, 64)), (1, 32, 128, (4, 2, 32)),
                                             # aligned stages (whole coarse rows per 8-segment stage)
                                             (1, 32, 64, (4, 16, 32)), (2, 64, 128, (4, 8, 64)),
                                             (1, 32, 64, (6, 16, 64)),
                                             # 8-voxel segments (coarse w 8 / 24)
                                             (1, 32, 64, (8, 6, 16)), (2, 64, 128, (16, 16, 16)),
                                             (1, 32, 64, (4, 6, 48))])
def test_wgrad_s2_four_tap(x3, N, cin, cout, dims):
    """Weight gradients of the k4 s2 p1 convs (PatchGAN layers 2-3, networks3D.py:389-400; the
    UNet's down convs) and of the k4 s2 p1 transposed up convs (networks3D.py:300-330) on the
    4-kw-tap even/odd-phase kernel (conv_wgrad3s2_x3.hip, KW 4, one-plane modes: 34 staged fine
    positions, fine row / voxel 2H / 2W read as zeros), vs fp64; bf16x3 keeps the generic kernel."""
    ops = x3
    g = torch.Generator().manual_seed(29 + N + cin + cout)
    x = torch.randn(N, cin, *dims, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, 4, 4, 4, generator=g, dtype=torch.float64) * 0.1
    y = F.conv3d(x, w, stride=2, padding=1)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dw_ref = torch.nn.grad.conv3d_weight(x, w.shape, dy, stride=2, padding=1)
    dw_rnd = torch.nn.grad.conv3d_weight(R(x), w.shape, R(dy), stride=2, padding=1)
    dw = torch.full((cout, cin, 4, 4, 4), 3.0, device="cuda")
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), 4, 2, 1, dw, accumulate=False)
    check_rounded(dw, dw_rnd, dw_ref)
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), 4, 2, 1, dw, accumulate=True)
    check_rounded(dw, 2 * dw_rnd, 2 * dw_ref)
    # transposed: ConvTranspose3d(cout → cin, k4 s2 p1) on the coarse grid of y
    xt = torch.randn(y.shape, generator=g, dtype=torch.float64)
    wt = (torch.randn(cout, cin, 4, 4, 4, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    yt = F.conv_transpose3d(xt, wt, stride=2, padding=1)
    assert tuple(yt.shape[2:]) == tuple(dims)
    dyt = torch.randn(yt.shape, generator=g, dtype=torch.float64)
    (dwt_ref,) = torch.autograd.grad(yt, wt, dyt)
    wr = R(wt).requires_grad_()
    (dwt_rnd,) = torch.autograd.grad(F.conv_transpose3d(R(xt), wr, stride=2, padding=1), wr, R(dyt))
    dwt = torch.zeros((cout, cin, 4, 4, 4), device="cuda")
    ops.conv3d_wgrad(ndhwc(xt.float()).cuda(), ndhwc(dyt.float()).cuda(), 4, 2, 1, dwt, accumulate=False)
    check_rounded(dwt, dwt_rnd, dwt_ref)


@pytest.mark.parametrize("N,cin,cout,dims,transposed", [
    (1, 256, 256, (4, 4, 4), False), (2, 256, 256, (4, 4, 4), False),     # UNet innermost down: M = N·2³
    (1, 256, 256, (4, 4, 4), True), (2, 256, 256, (4, 4, 4), True),       # innermost up (2³ → 4³)
    (1, 128, 512, (8, 8, 8), True), (1, 128, 256, (8, 8, 8), False),     # M = 64, the threshold
    (2, 128, 512, (8, 8, 8), True),                                        # M = 128: the split-K path
    (1, 20, 48, (4, 6, 2), False), (3, 48, 20, (2, 4, 6), True)])         # ragged dims, 20-wide tiles
def test_wgrad_short_contraction(x3, N, cin, cout, dims, transposed):
    """Weight gradients whose contraction is a few voxels (conv_wgrad.hip wgrad_small_kernel in the
    one-plane modes: the UNet's innermost k4 s2 layers, networks3D.py:300-330) — torch-layout
    output, no slab, accumulate on and off — vs the fp64 result on the mode's rounded operands."""
    ops = x3
    g = torch.Generator().manual_seed(41 + N + cin + 3 * cout + int(transposed))
    if not transposed:
        x = torch.randn(N, cin, *dims, generator=g, dtype=torch.float64)
        w = torch.randn(cout, cin, 4, 4, 4, generator=g, dtype=torch.float64) * 0.1
        dy = torch.randn(F.conv3d(x, w, stride=2, padding=1).shape, generator=g, dtype=torch.float64)
        ref = torch.nn.grad.conv3d_weight(x, w.shape, dy, stride=2, padding=1)
        rnd = torch.nn.grad.conv3d_weight(R(x), w.shape, R(dy), stride=2, padding=1)
        dense, gathered = ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda()
    else:
        # ConvTranspose3d(cin → cout) on the coarse grid `dims` / 2: D = its input, G = dY
        xt = torch.randn(N, cin, *[d // 2 for d in dims], generator=g, dtype=torch.float64)
        wt = (torch.randn(cin, cout, 4, 4, 4, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
        yt = F.conv_transpose3d(xt, wt, stride=2, padding=1)
        assert tuple(yt.shape[2:]) == tuple(dims)
        dyt = torch.randn(yt.shape, generator=g, dtype=torch.float64)
        (ref,) = torch.autograd.grad(yt, wt, dyt)
        wr = R(wt).requires_grad_()
        (rnd,) = torch.autograd.grad(F.conv_transpose3d(R(xt), wr, stride=2, padding=1), wr, R(dyt))
        dense, gathered = ndhwc(xt.float()).cuda(), ndhwc(dyt.float()).cuda()
    dw = torch.full(tuple(ref.shape), 3.0, device="cuda")
    ops.conv3d_wgrad(dense, gathered, 4, 2, 1, dw, accumulate=False)
    check_rounded(dw, rnd, ref)
    ops.conv3d_wgrad(dense, gathered, 4, 2, 1, dw, accumulate=True)
    check_rounded(dw, 2 * rnd, 2 * ref)


@pytest.mark.parametrize("N,cin,cout,S,k,s,p,op", CONVT_CASES)
def test_conv_transpose3d_bf16x3(x3, N, cin, cout, S, k, s, p, op):
    ops = x3
    g = torch.Generator().manual_seed(N + cin + 3 * cout)
    x = torch.randn(N, cin, S, S + 1, S, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(cin, cout, k, k, k, generator=g, dtype=torch.float64) * 0.1
    y = F.conv_transpose3d(x, w, stride=s, padding=p, output_padding=op)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (dx_ref,) = torch.autograd.grad(y, x, dy)
    xr = R(x).requires_grad_()
    yr = F.conv_transpose3d(xr, R(w), stride=s, padding=p, output_padding=op)
    (dx_rnd,) = torch.autograd.grad(F.conv_transpose3d(xr, R(w), stride=s, padding=p, output_padding=op), xr, R(dy))
    out = ops.conv3d(ndhwc(x.detach().float()).cuda(), pack(ops, w, True, False), cout, k, s, p, y.shape[2:],
                     transposed=True)
    check_rounded(ncdhw(out), yr.detach(), y.detach())
    dx = ops.conv3d(ndhwc(dy.float()).cuda(), pack(ops, w, True, True), cin, k, s, p, x.shape[2:])
    check_rounded(ncdhw(dx), dx_rnd, dx_ref)


@pytest.mark.parametrize("N,cin,cout,S,k,s,p", CONV_CASES)
def test_conv_all_paths_rounding(x3, N, cin, cout, S, k, s, p):
    """Every dispatch path — the thin VALU kernels of the image-channel layers and the fp32
    fallbacks included — rounds its operands in the bf16 / fp16 modes exactly like the MFMA
    kernels (ABI 10): forward, data gradient and weight gradient each equal the fp64 convolution
    of the rounded operands up to fp32 accumulation order."""
    ops = x3
    g = torch.Generator().manual_seed(23 + N * 1000 + cin * 7 + cout)
    x = torch.randn(N, cin, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(cout, generator=g, dtype=torch.float64)
    y = F.conv3d(x, w, b.float().double(), stride=s, padding=p)
    yr = F.conv3d(R(x), R(w), b.float().double(), stride=s, padding=p)
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, False, False), cout, k, s, p, y.shape[2:],
                     bias=b.float().cuda())
    check_rounded(ncdhw(out), yr, y)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dx = ops.conv3d(ndhwc(dy.float()).cuda(), pack(ops, w, False, True), cin, k, s, p, x.shape[2:], transposed=True)
    check_rounded(ncdhw(dx), torch.nn.grad.conv3d_input(x.shape, R(w), R(dy), stride=s, padding=p),
                  torch.nn.grad.conv3d_input(x.shape, w, dy, stride=s, padding=p))
    dw = torch.zeros((cout, cin, k, k, k), device="cuda")
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), k, s, p, dw, accumulate=False)
    check_rounded(dw, torch.nn.grad.conv3d_weight(R(x), w.shape, R(dy), stride=s, padding=p),
                  torch.nn.grad.conv3d_weight(x, w.shape, dy, stride=s, padding=p))


def test_conv_precision_modes(ops):
    assert ops.get_conv_precision() == "f32"
    with pytest.raises(ValueError):
        ops.set_conv_precision("fp8")
    for m in ("bf16x3", "bf16", "fp16", "f32"):
        ops.set_conv_precision(m)
        assert ops.get_conv_precision() == m
    assert ops.get_loss_scale() == 1.0


def _in_ref(x, act):
    m = x.mean(dim=(2, 3, 4), keepdim=True)
    v = ((x - m) ** 2).mean(dim=(2, 3, 4), keepdim=True)
    y = (x - m) / torch.sqrt(v + 1e-5)
    if act == "relu":
        y = F.relu(y)
    elif act == "lrelu":
        y = F.leaky_relu(y, 0.2)
    return y


@pytest.mark.parametrize("N,C,S", [(2, 32, 9), (1, 128, 6), (3, 8, 5), (1, 256, 3), (2, 24, 6), (5, 4, 7), (1, 32, 40),
                                   (2, 128, 15), (2, 256, 7), (1, 12, 5)])
@pytest.mark.parametrize("act", [None, "relu", "lrelu"])
@pytest.mark.parametrize("ypad", [0, 1, 3])
def test_instnorm_fwd(ops, N, C, S, act, ypad):
    g = torch.Generator().manual_seed(N * C + S)
    x = torch.randn(N, C, S, S + 1, S + 2, generator=g, dtype=torch.float64) * 3 + 1.5
    resid = torch.randn(N, C, S, S + 1, S + 2, generator=g, dtype=torch.float64) if act is None else None
    ref = _in_ref(x, act)
    if resid is not None:
        ref = ref + resid
    ref = F.pad(ref, (ypad,) * 6, mode="replicate") if ypad else ref
    rg = None
    if resid is not None:
        rg = ndhwc(F.pad(resid, (1,) * 6, mode="replicate").float()).cuda()
    out, mean, rstd = ops.instnorm_fwd(ndhwc(x.float()).cuda(), act=act, ypad=ypad, resid=rg, rpad=1)
    assert rel(ncdhw(out), ref) < TOL
    assert rel(mean, x.mean(dim=(2, 3, 4))) < 1e-6


@pytest.mark.parametrize("N,C,S", [(2, 32, 7), (1, 128, 5), (2, 8, 6), (2, 24, 5), (1, 32, 33), (2, 128, 15), (2, 256, 7),
                                   (1, 12, 5)])
@pytest.mark.parametrize("act", [None, "relu", "lrelu"])
@pytest.mark.parametrize("dypad", [0, 1, 3])
@pytest.mark.parametrize("with_add", [False, True])
def test_instnorm_bwd(ops, N, C, S, act, dypad, with_add):
    g = torch.Generator().manual_seed(N + C + S + dypad)
    x = (torch.randn(N, C, S, S + 1, S, generator=g, dtype=torch.float64) * 2 - 0.5).requires_grad_()
    y = _in_ref(x, act)
    yp = F.pad(y, (dypad,) * 6, mode="replicate") if dypad else y
    dyp = torch.randn(yp.shape, generator=g, dtype=torch.float64)
    add = torch.randn(y.shape, generator=g, dtype=torch.float64) if with_add else None
    loss = (yp * dyp).sum() + ((y * add).sum() if with_add else 0)
    (dx_ref,) = torch.autograd.grad(loss, x)
    xg = ndhwc(x.detach().float()).cuda()
    _, mean, rstd = ops.instnorm_fwd(xg, act=act)
    dx = ops.instnorm_bwd(xg, mean, rstd, ndhwc(dyp.float()).cuda(), dypad,
                          ndhwc(add.float()).cuda() if with_add else None, act=act)
    assert rel(ncdhw(dx), dx_ref) < 5e-5


@pytest.mark.parametrize("C,dypad,act", [(128, 1, None), (32, 3, "relu"), (8, 0, "lrelu")])
def test_instnorm_bwd_g_out(ops, C, dypad, act):
    """mragan_instnorm_bwd_g: dx as mragan_instnorm_bwd, and g_out = fold(dy) + dy_add (the
    ResnetBlock input gradient that replaces a separate rpad_fold pass) equal to rpad_fold's."""
    g = torch.Generator().manual_seed(C + dypad)
    x = torch.randn(2, C, 5, 6, 7, generator=g, dtype=torch.float64)
    xg = ndhwc(x.float()).cuda()
    _, mean, rstd = ops.instnorm_fwd(xg, act=act)
    dyp = ndhwc(torch.randn(2, C, 5 + 2 * dypad, 6 + 2 * dypad, 7 + 2 * dypad, generator=g).float()).cuda()
    add = ndhwc(torch.randn(2, C, 5, 6, 7, generator=g).float()).cuda()
    dx_ref = ops.instnorm_bwd(xg, mean, rstd, dyp, dypad, add, act=act)
    G = torch.full_like(xg, float("nan"))
    dx = ops.instnorm_bwd(xg, mean, rstd, dyp, dypad, add, act=act, g_out=G)
    assert torch.equal(dx, dx_ref)
    G_ref = ops.rpad_fold(dyp, dypad, add=add) if dypad else dyp + add
    assert rel(G, G_ref) < 1e-6          # border voxels: the same terms summed in another order


@pytest.mark.parametrize("N,C,S", [(2, 128, 16), (1, 64, 9), (3, 64, 7)])
def test_brick_in_stats_partials(x3, N, C, S):
    """ABI 9: the brick conv's epilogue InstanceNorm partials (mragan_conv3d_presplit_in_stats)
    feed mragan_instnorm_fwd_partials; output, mean / rstd and the normalised tensor match the
    statistics-pass path (partial bricks included: 9³ and 7³ outputs leave padding rows)."""
    ops = x3
    g = torch.Generator().manual_seed(N * 7 + C + S)
    x = torch.randn(N, C, S + 2, S + 3, S + 2, generator=g, dtype=torch.float64)
    w = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    xg = ndhwc(x.float()).cuda()
    wp = pack(ops, w, False, False)
    wsplit = torch.empty(wp.numel(), device="cuda", dtype=torch.float32)
    ops.pack_weight(w.float().cuda().contiguous(), C, C, 27, 4 if ops.get_conv_precision() == "fp16" else 2, wsplit)
    osp = (S, S + 1, S)
    y_ref = ops.conv3d(xg, wp, C, 3, 1, 0, osp, wsplit=wsplit)
    part = ops.in_partials_buffer(N, osp, C, "cuda")
    y, chunks = ops.conv3d_in_stats(xg, wp, C, 3, 1, 0, osp, wsplit, part)
    assert chunks > 0
    assert torch.equal(y, y_ref)
    z_ref, m_ref, r_ref = ops.instnorm_fwd(y_ref, act="relu", ypad=1)
    z, m, r = ops.instnorm_fwd(y, act="relu", ypad=1, part=part, chunks=chunks)
    assert rel(m, m_ref) < 1e-6 and rel(r, r_ref) < 1e-6
    assert rel(z, z_ref) < 1e-6


@pytest.fixture(params=["bf16", "fp16"])
def op16(ops, request):
    """The two modes with 16-bit operand planes (ABI 11)."""
    ops.set_conv_precision(request.param)
    yield ops
    ops.set_conv_precision("f32")


def _presplit(ops, w, C_in, C_out, transposed_pack):
    wsplit = torch.empty(w.numel(), device="cuda", dtype=torch.float32)
    base = 4 if ops.get_conv_precision() == "fp16" else 2
    ops.pack_weight(w.float().cuda().contiguous(), C_out, C_in, 27, base + int(transposed_pack), wsplit)
    return wsplit


@pytest.mark.parametrize("N,C,S,ypad,act,resid", [(2, 128, 16, 1, "relu", False), (1, 64, 9, 1, None, True),
                                                  (3, 64, 7, 0, "relu", True)])
def test_op16_instnorm_fwd_planes(op16, N, C, S, ypad, act, resid):
    """ABI 11: the InstanceNorm forward's operand plane is exactly its fp32 output rounded RNE to
    the mode's 16-bit type (torch's .to() rounds RNE); the fp32 copy is bit-identical to the fp32
    entry's; the statistics-pass and the brick-partials forms both."""
    ops = op16
    g = torch.Generator().manual_seed(N + C + S)
    x = ndhwc(torch.randn(N, C, S, S + 1, S, generator=g).float()).cuda()
    r = ndhwc(torch.randn(N, C, S + 2, S + 3, S + 2, generator=g).float()).cuda() if resid else None
    y_ref, m_ref, s_ref = ops.instnorm_fwd(x, act=act, ypad=ypad, resid=r, rpad=1 if resid else 0)
    y, y16, m, rs = ops.instnorm_fwd_op16(x, act=act, ypad=ypad, resid=r, rpad=1 if resid else 0, want_f32=True)
    assert torch.equal(y, y_ref) and torch.equal(m, m_ref) and torch.equal(rs, s_ref)
    assert y16.dtype == ops.op16_dtype() and torch.equal(y16, y_ref.to(ops.op16_dtype()))
    none, y16b, _, _ = ops.instnorm_fwd_op16(x, act=act, ypad=ypad, resid=r, rpad=1 if resid else 0)
    assert none is None and torch.equal(y16b, y16)


@pytest.mark.parametrize("C,dypad,act,with_g", [(128, 1, None, True), (128, 1, "relu", False), (64, 0, "relu", False)])
def test_op16_instnorm_bwd_plane(op16, C, dypad, act, with_g):
    """ABI 11: the InstanceNorm backward's dx plane = its fp32 dx rounded RNE; g_out unchanged."""
    ops = op16
    g = torch.Generator().manual_seed(C + dypad)
    N, S = 2, 9
    x = ndhwc(torch.randn(N, C, S, S, S + 1, generator=g).float()).cuda()
    _, mean, rstd = ops.instnorm_fwd(x, act=act)
    dy = ndhwc(torch.randn(N, C, S + 2 * dypad, S + 2 * dypad, S + 1 + 2 * dypad, generator=g).float()).cuda()
    add = ndhwc(torch.randn(N, C, S, S, S + 1, generator=g).float()).cuda()
    G_ref = torch.empty_like(x)
    dx_ref = ops.instnorm_bwd(x, mean, rstd, dy, dypad, add, act=act, g_out=G_ref)
    G = torch.full_like(x, float("nan")) if with_g else None
    dx16 = ops.instnorm_bwd_op16(x, mean, rstd, dy, dypad, add, act=act, g_out=G)
    assert torch.equal(dx16, dx_ref.to(ops.op16_dtype()))
    if with_g:
        assert torch.equal(G, G_ref)


@pytest.mark.parametrize("N,C,S,W", [(2, 128, 16, 16), (1, 64, 9, 16), (1, 128, 5, 32), (1, 128, 8, 24), (2, 64, 8, 24)])
def test_op16_brick_conv_and_wgrad(op16, N, C, S, W):
    """ABI 11: the brick forward (with its InstanceNorm partials), the whole-grid data gradient and
    the k3 s1 weight gradient on operand planes equal the same kernels on the fp32 tensors in the
    same mode bit for bit (the fp32 path rounds each operand to the very words the planes hold)."""
    ops = op16
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N * 11 + C + S)
    x = ndhwc(torch.randn(N, C, S + 2, S + 2, W + 2, generator=g).float()).cuda()     # padded block input
    w = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp_f, wp_b = pack(ops, w, False, False), pack(ops, w, False, True)
    ws_f, ws_b = _presplit(ops, w, C, C, False), _presplit(ops, w, C, C, True)
    osp = (S, S, W)
    part_ref = ops.in_partials_buffer(N, osp, C, "cuda")
    y_ref, ch_ref = ops.conv3d_in_stats(x, wp_f, C, 3, 1, 0, osp, ws_f, part_ref)
    part = ops.in_partials_buffer(N, osp, C, "cuda")
    y, ch = ops.conv3d_op16(x.to(dt), wp_f, C, 3, 1, 0, osp, ws_f, part)
    assert ch == ch_ref > 0
    assert torch.equal(y, y_ref)
    n = N * ch * C * 2
    assert torch.equal(part[:n], part_ref[:n])
    dy = ndhwc(torch.randn(N, C, S, S, W, generator=g).float()).cuda()
    dx_ref = ops.conv3d(dy, wp_b, C, 3, 1, 0, (S + 2, S + 2, W + 2), transposed=True, wsplit=ws_b)
    dx, _ = ops.conv3d_op16(dy.to(dt), wp_b, C, 3, 1, 0, (S + 2, S + 2, W + 2), ws_b, transposed=True)
    assert torch.equal(dx, dx_ref)
    gw_ref = torch.empty(C * C * 27, device="cuda")
    ops.conv3d_wgrad(dy, x, 3, 1, 0, gw_ref, False)
    gw = torch.full_like(gw_ref, float("nan"))
    ops.conv3d_wgrad_op16(dy.to(dt), x.to(dt), 3, 1, 0, gw, False)
    if W % 16 == 0:
        assert torch.equal(gw, gw_ref)
    else:   # 24-wide rows: wgrad3's 24-voxel segments (planes only) vs the generic kernel on fp32
        assert rel(gw, gw_ref) < 2e-5
    # and against fp64 on the rounded operands (the mode's definition)
    gw64 = F.conv3d(ncdhw(x.to(dt).double().cpu()).transpose(0, 1), ncdhw(dy.to(dt).double().cpu()).transpose(0, 1))
    assert rel(gw.view(C, C, 3, 3, 3), gw64.transpose(0, 1)) < 2e-5


@pytest.mark.parametrize("N1,N2,C,S,W", [(4, 2, 128, 16, 16), (2, 1, 128, 24, 24), (1, 1, 64, 8, 32),
                                          (2, 2, 128, 5, 16)])
def test_op16_wgrad_pair(op16, N1, N2, C, S, W):
    """ABI 19: one ResnetBlock weight gradient over two instance sets (a generator's first and cycle
    pass) is bit-identical to the same kernel over the two sets concatenated in one tensor (same
    segments, splits and reduce order) where the aligned plane path takes both (16³, 24³, 32-wide);
    otherwise (5-row planes: unaligned stages) it is the two accumulating passes, bit for bit; and
    it equals fp64 on the rounded operands."""
    ops = op16
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N1 * 7 + N2 + C + S)
    x = ndhwc(torch.randn(N1 + N2, C, S + 2, S + 2, W + 2, generator=g).float()).cuda().to(dt)
    dy = ndhwc(torch.randn(N1 + N2, C, S, S, W, generator=g).float()).cuda().to(dt)
    xa, xb = x[:N1].clone(), x[N1:].clone()              # separate allocations, as the two passes'
    da, db = dy[:N1].clone(), dy[N1:].clone()
    gw = torch.full((C * C * 27,), float("nan"), device="cuda")
    ops.conv3d_wgrad_op16_pair(da, xa, db, xb, 3, 1, 0, gw, False)
    nsw = W // (16 if W % 16 == 0 else 24)                # row segments per w-row (wgrad3 w3_segw)
    aligned = S % (8 // nsw) == 0                         # whole rows per 8-segment stage
    ref = torch.empty_like(gw)
    if aligned:
        ops.conv3d_wgrad_op16(dy, x, 3, 1, 0, ref, False)
    else:
        ops.conv3d_wgrad_op16(da, xa, 3, 1, 0, ref, False)
        ops.conv3d_wgrad_op16(db, xb, 3, 1, 0, ref, True)
    torch.cuda.synchronize()
    assert torch.equal(gw, ref)
    gw64 = F.conv3d(ncdhw(x.double().cpu()).transpose(0, 1), ncdhw(dy.double().cpu()).transpose(0, 1))
    assert rel(gw.view(C, C, 3, 3, 3), gw64.transpose(0, 1)) < 2e-5


@pytest.mark.parametrize("N,S,C", [(2, 32, 128), (1, 32, 128), (4, 24, 128), (2, 24, 64), (2, 16, 128)])
def test_op16_res_dgrad_interior_shell(op16, N, S, C):
    """The ResnetBlock whole-grid data gradient for N ≥ 2 at 24³ / 32³ runs as the interior brick (the
    "same" conv written one voxel in) plus the shell pass (mragan_conv3d_dgrad_split; 1 × 32³ and
    16³ keep the whole-grid brick): fp64 on the rounded operands, and bit-identical between the plane
    and the fp32 input.  ABI 19: both passes read only the pre-split weights — the fp32 pack filled
    with NaN changes nothing, and with no fp32 pack at all (NULL) the result is the same bits."""
    ops = op16
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N * 3 + S + C)
    w = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp_b, ws_b = pack(ops, w, False, True), _presplit(ops, w, C, C, True)
    wp_nan = torch.full_like(wp_b, float("nan"))
    dy = ndhwc(torch.randn(N, C, S, S, S, generator=g).float()).cuda()
    osp = (S + 2,) * 3
    assert ops.dgrad_split(N, S, S, S, C, C) == (N >= 2 and S >= 24)
    dx, _ = ops.conv3d_op16(dy.to(dt), wp_nan, C, 3, 1, 0, osp, ws_b, transposed=True)
    dx_null, _ = ops.conv3d_op16(dy.to(dt), None, C, 3, 1, 0, osp, ws_b, transposed=True)
    dx_fresh, _ = ops.conv3d_op16(dy.to(dt), wp_b, C, 3, 1, 0, osp, ws_b, transposed=True)
    dx32 = ops.conv3d(dy, wp_nan, C, 3, 1, 0, osp, transposed=True, wsplit=ws_b)
    assert torch.isfinite(dx).all()
    assert torch.equal(dx, dx_null) and torch.equal(dx, dx_fresh)
    assert torch.equal(dx, dx32)
    ref = F.conv_transpose3d(ncdhw(dy.to(dt).double().cpu()), w.float().to(dt).double())
    assert rel(ncdhw(dx.double().cpu()), ref) < 2e-5


def test_null_fp32_pack_refused(op16):
    """ABI 19: a kernel that needs the fp32 pack refuses a NULL one (the caller's pack is stale)
    instead of computing with whatever the buffer holds: a k3 s1 conv with 32 output channels (no
    brick shape: the implicit GEMM, which reads the fp32 pack)."""
    from mragan_hip._lib import MraganError
    ops = op16
    C = 32
    w = torch.randn(C, C, 3, 3, 3, dtype=torch.float64) * 0.05
    ws = _presplit(ops, w, C, C, False)
    x = ndhwc(torch.randn(1, C, 8, 8, 8).float()).cuda()
    with pytest.raises(MraganError, match="fp32 weight pack"):
        ops.conv3d(x, None, C, 3, 1, 1, (8, 8, 8), wsplit=ws)
        torch.cuda.synchronize()


@pytest.mark.parametrize("N,S,act,fin", [(4, 16, None, True), (2, 16, None, True), (2, 16, None, False),
                                          (1, 32, None, True), (2, 16, "relu", True)])
def test_op16_dgrad_skip_statistics(op16, N, S, act, fin):
    """ABI 18: conv1's data gradient of ResnetBlock i+1 leaves the backward statistics of block i's
    second InstanceNorm, whose input gradient is fold(dz) + G (G: block i+1's output gradient, the
    skip path): dz bit-identical to the plain data gradient (fp32 noise where the statistics brick
    differs), G written by the IN backward bit-identical, dx within fp64 summation-order noise of the
    statistics-pass IN backward on the same dz — for the
    8-wave brick (N = 4), the K-split brick with and without in-launch finalize, the large grid."""
    ops = op16
    dt = ops.op16_dtype()
    C = 128
    g = torch.Generator().manual_seed(N * 13 + S)
    w = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp_b, ws_b = pack(ops, w, False, True), _presplit(ops, w, C, C, True)
    h = ndhwc(torch.randn(N, C, S, S, S, generator=g).float()).cuda()          # block i's conv2 output
    _, m, r = ops.instnorm_fwd(h, act=act)
    dh1 = ndhwc(torch.randn(N, C, S, S, S, generator=g).float()).cuda().to(dt)  # block i+1's IN1 dx plane
    G1 = ndhwc(torch.randn(N, C, S, S, S, generator=g).float()).cuda()         # block i+1's output gradient
    dz_ref, _ = ops.conv3d_op16(dh1, wp_b, C, 3, 1, 0, (S + 2,) * 3, ws_b, transposed=True)
    part = ops.in_partials_buffer(N, (S + 2,) * 3, C, "cuda")
    res = ops.conv3d_op16_dgrad_in_stats(dh1, wp_b, C, ws_b, h, m, r, act, part, fin=fin, x_add=G1)
    dz, chunks = res[0], res[1]
    coef = res[2] if fin else None
    assert chunks > 0
    # the plain data gradient of a large grid may run another brick (summation order): same to fp32 noise
    assert torch.equal(dz, dz_ref) if N * S ** 3 < 32768 else rel(dz, dz_ref) < 1e-6
    G_ref = torch.empty_like(h)
    dx_ref = ops.instnorm_bwd_op16(h, m, r, dz, 1, G1, act=act, g_out=G_ref)
    G = torch.full_like(h, float("nan"))
    dx = ops.instnorm_bwd_partials_op16(h, m, r, dz, 1, G1, act, part, chunks, g_out=G, coef=coef)
    assert torch.equal(G, G_ref)
    assert torch.isfinite(dx.float()).all()
    assert (dx != dx_ref).float().mean().item() < 1e-3        # only round-half cases of ~1e-7 shifts
    assert rel(dx, dx_ref) < 1e-5


@pytest.mark.parametrize("N,S", [(2, 16), (4, 16), (1, 12)])
def test_in_launch_finalize(op16, N, S):
    """ABI 15: the bricks' last block per (instance, column tile) finalizes the InstanceNorm
    statistics (ticket counters, write-through partials; the K-split brick, and since round 6 the
    8-wave brick of the 18³ data gradient at N = 4): the conv output and partials are
    bit-identical to the non-finalizing launch, μ / rstd and the backward coefficients agree with the
    finalize kernel to fp64 summation-order noise, and repeated launches (tickets reset by the last
    block) give bit-identical results."""
    ops = op16
    dt = ops.op16_dtype()
    C = 128
    g = torch.Generator().manual_seed(N * 5 + S)
    x16 = ndhwc(torch.randn(N, C, S + 2, S + 2, S + 2, generator=g).float()).cuda().to(dt)
    w = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp_f, wp_b = pack(ops, w, False, False), pack(ops, w, False, True)
    ws_f, ws_b = _presplit(ops, w, C, C, False), _presplit(ops, w, C, C, True)
    osp = (S, S, S)
    part_ref = ops.in_partials_buffer(N, osp, C, "cuda")
    y_ref, ch_ref = ops.conv3d_op16(x16, wp_f, C, 3, 1, 0, osp, ws_f, part_ref)
    _, z_ref, m_ref, r_ref = ops.instnorm_fwd_op16(y_ref, act="relu", ypad=1, part=part_ref, chunks=ch_ref)
    runs = []
    for _ in range(3):
        part = ops.in_partials_buffer(N, osp, C, "cuda")
        y, ch, stats = ops.conv3d_op16(x16, wp_f, C, 3, 1, 0, osp, ws_f, part, fin=True)
        runs.append((y, ch, stats))
    y, ch, stats = runs[0]
    assert ch == ch_ref > 0 and stats is not None, "the K-split brick did not finalize in-launch"
    assert torch.equal(y, y_ref)
    n = N * ch * C * 2
    assert torch.equal(part[:n], part_ref[:n])
    m, r = stats
    assert rel(m, m_ref) < 1e-6 and rel(r, r_ref) < 1e-6
    for yy, cc, ss in runs[1:]:
        assert torch.equal(yy, y) and torch.equal(ss[0], m) and torch.equal(ss[1], r)
    _, z, _, _ = ops.instnorm_fwd_op16(y, act="relu", ypad=1, stats=stats)
    assert (z != z_ref).float().mean().item() < 1e-3          # only round-half cases of ~1e-7 shifts
    # the data gradient with the backward coefficients of IN1 (the step's conv2 data gradient)
    dh2 = ndhwc(torch.randn(N, C, S, S, S, generator=g).float()).cuda().to(dt)
    pb_ref = ops.in_partials_buffer(N, (S + 2,) * 3, C, "cuda")
    dz_ref, cb_ref = ops.conv3d_op16_dgrad_in_stats(dh2, wp_b, C, ws_b, y, m, r, "relu", pb_ref)
    pb = ops.in_partials_buffer(N, (S + 2,) * 3, C, "cuda")
    dz, cb, coef = ops.conv3d_op16_dgrad_in_stats(dh2, wp_b, C, ws_b, y, m, r, "relu", pb, fin=True)
    assert torch.equal(dz, dz_ref) and cb == cb_ref > 0
    ref = ops.instnorm_bwd_partials_op16(y, m, r, dz_ref, 1, None, "relu", pb_ref, cb_ref)
    # the 8-wave brick (the 18³ data gradient at N = 4) finalizes in-launch too since round 6
    assert coef is not None, "the data gradient did not finalize in-launch"
    got = ops.instnorm_bwd_partials_op16(y, m, r, dz, 1, None, "relu", pb, cb, coef=coef)
    assert (got != ref).float().mean().item() < 1e-3


@pytest.mark.parametrize("N,cin,cout,dims", [(2, 32, 64, (32, 32, 32)), (1, 64, 128, (16, 16, 32)),
                                              (1, 32, 64, (8, 12, 64))])
def test_op16_stride2_conv_and_wgrad(op16, N, cin, cout, dims):
    """ABI 14: G down1 / down2 (Conv3d k3 s2 p1) on the operand plane of their input — the implicit
    GEMM's 16-bit A tiles (forward, with its InstanceNorm partials) and wgrad3s2's 16-bit gathered
    operand — equal the same kernels on the fp32 tensor in the same mode bit for bit."""
    ops = op16
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N * 7 + cin + cout + dims[2])
    D, H, W = dims
    x16 = ndhwc(torch.randn(N, cin, D, H, W, generator=g).float()).cuda().to(dt)
    x = x16.float()
    w = torch.randn(cout, cin, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp_f = pack(ops, w, False, False)
    osp = (D // 2, H // 2, W // 2)
    part_ref = ops.in_partials_buffer(N, osp, cout, "cuda")
    y_ref, ch_ref = ops.conv3d_in_stats(x, wp_f, cout, 3, 2, 1, osp, None, part_ref)
    part = ops.in_partials_buffer(N, osp, cout, "cuda")
    y, ch = ops.conv3d_op16(x16, wp_f, cout, 3, 2, 1, osp, None, part)
    assert ch == ch_ref
    assert torch.equal(y, y_ref)
    n = N * ch * cout * 2
    assert torch.equal(part[:n], part_ref[:n])
    dy = ndhwc(torch.randn(N, cout, *osp, generator=g).float()).cuda()
    gw_ref = torch.empty(cout * cin * 27, device="cuda")
    ops.conv3d_wgrad(dy, x, 3, 2, 1, gw_ref, False)
    gw = torch.full_like(gw_ref, float("nan"))
    ops.conv3d_wgrad_g16(dy, x16, 3, 2, 1, gw, False)
    assert torch.equal(gw, gw_ref)
    # ABI 16: both operands as planes (G down2's weight gradient: dY exists only as its plane)
    if cout % 64 == 0 and dims[2] // 2 % 16 == 0:
        gw2 = torch.full_like(gw_ref, float("nan"))
        ops.conv3d_wgrad_op16(dy.to(dt), x16, 3, 2, 1, gw2, False)
        assert torch.equal(gw2, gw_ref)
    # and against fp64 on the rounded operands (the mode's definition)
    gw64 = torch.nn.grad.conv3d_weight(ncdhw(x.double().cpu()), (cout, cin, 3, 3, 3),
                                       ncdhw(dy.to(dt).double().cpu()), stride=2, padding=1)
    assert rel(gw.view(cout, cin, 3, 3, 3), gw64) < 2e-5


S2_DEFAULT = [(2, 64, 128, (32, 32, 32)), (4, 64, 128, (32, 32, 32)), (2, 64, 128, (24, 24, 24)),
              (1, 64, 64, (14, 30, 10)), (1, 96, 128, (20, 18, 26))]
S2_FORCED = [(4, 32, 64, (64, 64, 64)), (1, 32, 64, (20, 18, 26)), (2, 32, 128, (16, 16, 16))]


@pytest.mark.parametrize("N,cin,cout,dims", S2_DEFAULT)
def test_stride2_brick(op16, N, cin, cout, dims):
    """Round 6: G down2 (Conv3d k3 s2 p1, networks3D.py:191-197) on the brick
    kernel's stride-2 form (conv_brick_x3.hip S = 2: LDS halo with even / odd w halves, the pre-split
    weights) — see stride2_brick_case."""
    stride2_brick_case(op16, N, cin, cout, dims)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_stride2_brick_forced_down1(prec):
    """The 32-input-channel form (G down1, on the implicit GEMM by default) forced onto the stride-2
    brick (MRAGAN_BRICK_S2_VAR, read once per process: a child process), every variant."""
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "from mragan_hip import ops\nimport test_kernels_gpu as t\nops.set_conv_precision(%r)\n"
            "for c in t.S2_FORCED: t.stride2_brick_case(ops, *c)\nprint('ok')\n"
            % (here, os.path.join(os.path.dirname(here), "mra-gan_amd"), prec))
    for var in ("1", "2", "4", "5"):
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, MRAGAN_BRICK_S2_VAR=var),
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (var, r.stdout[-2000:], r.stderr[-3000:])


def stride2_brick_case(ops, N, cin, cout, dims):
    """The operand-plane input and the fp32 input give the same bits (output and InstanceNorm
    partials); against the fp64 convolution of the rounded operands to 2e-5, the partials against the
    output's own sums; ragged volumes (partial bricks) included."""
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N * 13 + cin + cout + dims[2])
    D, H, W = dims
    x16 = ndhwc(torch.randn(N, cin, D, H, W, generator=g).float()).cuda().to(dt)
    x = x16.float()
    w = torch.randn(cout, cin, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp_f = pack(ops, w, False, False)
    ws = _presplit(ops, w, cin, cout, False)
    osp = tuple((d + 1) // 2 for d in dims)
    part16 = ops.in_partials_buffer(N, osp, cout, "cuda")
    # no fp32 pack: only the brick can run (the implicit GEMM refuses without one, ABI 19)
    y16, ch16 = ops.conv3d_op16(x16, None, cout, 3, 2, 1, osp, ws, part16)
    part32 = ops.in_partials_buffer(N, osp, cout, "cuda")
    y32, ch32 = ops.conv3d_in_stats(x, None, cout, 3, 2, 1, osp, ws, part32)
    assert ch16 == ch32 and ch16 > 0
    assert torch.equal(y16, y32)
    n = N * ch16 * cout * 2
    assert torch.equal(part16[:n], part32[:n])
    sums = part16[:n].view(N, ch16, cout, 2).sum(1)
    yd = y16.double()
    assert rel(sums[..., 0], yd.sum((1, 2, 3))) < 1e-9
    assert rel(sums[..., 1], (yd * yd).sum((1, 2, 3))) < 1e-9
    # the implicit GEMM on the same rounded operands (no pre-split copy: the pre-round-6 dispatch)
    y_ig, _ = ops.conv3d_op16(x16, wp_f, cout, 3, 2, 1, osp, None, None)
    assert rel(y16, y_ig) < 1e-6
    if D * H * W <= 40 ** 3:
        ref = F.conv3d(ncdhw(x.double().cpu()), R(w.float()), stride=2, padding=1)
        assert rel(ncdhw(y16.double().cpu()), ref) < 2e-5


@pytest.mark.parametrize("N,nc,S,W", [(2, 1, 20, 20), (1, 2, 17, 23), (1, 1, 64, 64)])
def test_k7_planes_bit_identical(op16, N, nc, S, W):
    """ABI 17: the k7 layers on the 16-bit operand plane of their 32-channel operand — the G head
    forward (thinn_x3 on the RPad3 input's plane, + bias, Tanh), the G stem data gradient (thinn_x3,
    transposed form, on the plane of the IN backward's dx) and both weight gradients (thin1 wgrad,
    the 32-channel side a plane) — equal the same kernels on the fp32 tensor in the same mode bit for
    bit, and the fp64 convolution of the rounded operands to 2e-5."""
    ops = op16
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N * 11 + nc + S + W)
    Sp, Wp = S + 6, W + 6
    # head: 32 → nc on the padded input
    x16 = ndhwc(torch.randn(N, 32, Sp, Sp, Wp, generator=g).float()).cuda().to(dt)
    x = x16.float()
    w_head = torch.randn(nc, 32, 7, 7, 7, generator=g, dtype=torch.float64) * 0.02
    b = torch.randn(nc, generator=g).float().cuda()
    wp = pack(ops, w_head, False, False)
    y_ref = ops.conv3d(x, wp, nc, 7, 1, 0, (S, S, W), bias=b, act="tanh")
    y = ops.conv3d_thin_op16(x16, wp, nc, 7, 1, 0, (S, S, W), bias=b, act="tanh")
    assert torch.equal(y, y_ref)
    y64 = torch.tanh(F.conv3d(ncdhw(x.double().cpu()), R(w_head), b.double().cpu()))
    assert rel(ncdhw(y), y64) < 2e-5
    # head weight gradient: dense = dz (nc channels, fp32), gathered = the input plane
    dz = ndhwc(torch.randn(N, nc, S, S, W, generator=g).float()).cuda()
    gw_ref = torch.empty(nc * 32 * 343, device="cuda")
    ops.conv3d_wgrad(dz, x, 7, 1, 0, gw_ref, False)
    gw = torch.full_like(gw_ref, float("nan"))
    ops.conv3d_wgrad_thin_op16(dz, x16, 7, 1, 0, gw, False)
    assert torch.equal(gw, gw_ref)
    # stem: nc → 32; its data gradient and weight gradient from the plane of dx (dense, 32 channels)
    dh16 = ndhwc(torch.randn(N, 32, S, S, W, generator=g).float()).cuda().to(dt)
    dh = dh16.float()
    w_stem = torch.randn(32, nc, 7, 7, 7, generator=g, dtype=torch.float64) * 0.02
    wb = pack(ops, w_stem, False, True)
    gx_ref = ops.conv3d(dh, wb, nc, 7, 1, 0, (Sp, Sp, Wp), transposed=True)
    gx = ops.conv3d_thin_op16(dh16, wb, nc, 7, 1, 0, (Sp, Sp, Wp), transposed=True)
    assert torch.equal(gx, gx_ref)
    xs = ndhwc(torch.randn(N, nc, Sp, Sp, Wp, generator=g).float()).cuda()
    gws_ref = torch.empty(32 * nc * 343, device="cuda")
    ops.conv3d_wgrad(dh, xs, 7, 1, 0, gws_ref, False)
    gws = torch.full_like(gws_ref, float("nan"))
    ops.conv3d_wgrad_thin_op16(dh16, xs, 7, 1, 0, gws, False, )
    assert torch.equal(gws, gws_ref)
    gw64 = torch.nn.grad.conv3d_weight(R(ncdhw(xs.double().cpu())), (32, nc, 7, 7, 7), ncdhw(dh.double().cpu()))
    assert rel(gws.view(32, nc, 7, 7, 7), gw64) < 2e-5


def test_k7_planes_rejected(op16):
    """conv3d_thin_op16 takes only the 32 → nc k7 shapes, wgrad_thin_op16 only nc ↔ 32 k7."""
    ops = op16
    dt = ops.op16_dtype()
    x16 = torch.zeros(1, 10, 10, 10, 64, device="cuda", dtype=dt)
    with pytest.raises(RuntimeError):
        ops.conv3d_thin_op16(x16, torch.zeros(343 * 64, device="cuda"), 1, 7, 1, 0, (4, 4, 4))
    with pytest.raises(RuntimeError):
        ops.conv3d_wgrad_thin_op16(torch.zeros(1, 4, 4, 4, 1, device="cuda"), x16, 7, 1, 0,
                                   torch.zeros(64 * 343, device="cuda"), False)


@pytest.mark.parametrize("N,cin,cout,S,act", [(2, 32, 64, 32, "relu"), (1, 64, 128, 16, "relu"), (2, 32, 64, 16, "lrelu")])
def test_op16_stride2_dgrad_backward_statistics(op16, N, cin, cout, S, act):
    """ABI 16: the data gradient of G up2 / up1 (a forward-form k3 s2 conv over the plane of the IN
    backward's dx) with the backward statistics of the IN in front: output and partials bit-identical
    to the fp32-input form of the same mode."""
    ops = op16
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N * 23 + cin + cout + S)
    x16 = ndhwc(torch.randn(N, cin, S, S, S, generator=g).float()).cuda().to(dt)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp = pack(ops, w, False, False)
    o = S // 2
    osp = (o, o, o)
    xin = ndhwc(torch.randn(N, cout, o, o, o, generator=g).float()).cuda()
    _, mean, rstd = ops.instnorm_fwd(xin, act=act)
    part_ref = ops.in_partials_buffer(N, osp, cout, "cuda")
    y_ref, ch_ref = ops.conv3d_bwd_stats(x16.float(), wp, cout, 3, 2, 1, osp, None, xin, mean, rstd, act, part_ref)
    part = ops.in_partials_buffer(N, osp, cout, "cuda")
    y, ch = ops.conv3d_op16_bwd_stats(x16, wp, cout, 3, 2, 1, osp, xin, mean, rstd, act, part)
    assert ch == ch_ref
    assert torch.equal(y, y_ref)
    n = N * ch * cout * 2
    assert torch.equal(part[:n], part_ref[:n])


@pytest.mark.parametrize("N,cin,S", [(2, 64, 16), (1, 64, 8), (2, 128, 8)])
def test_op16_brickT_plane(op16, N, cin, S):
    """Round 4: brickT (32-output-channel ConvTranspose3d k3 s2 p1 op1: G up2, G down1's data
    gradient) on the operand plane of its input — output and InstanceNorm partials bit-identical to
    the fp32-input launch of the same mode."""
    ops = op16
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N * 29 + cin + S)
    x16 = ndhwc(torch.randn(N, cin, S, S, S, generator=g).float()).cuda().to(dt)
    w = torch.randn(cin, 32, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp = pack(ops, w, True, False)
    osp = (2 * S, 2 * S, 2 * S)
    part_ref = ops.in_partials_buffer(N, osp, 32, "cuda")
    y_ref, ch_ref = ops.conv3d_in_stats(x16.float(), wp, 32, 3, 2, 1, osp, None, part_ref, transposed=True)
    part = ops.in_partials_buffer(N, osp, 32, "cuda")
    y, ch = ops.conv3d_op16(x16, wp, 32, 3, 2, 1, osp, None, part, transposed=True)
    assert ch == ch_ref > 0
    assert torch.equal(y, y_ref)
    n = N * ch * 32 * 2
    assert torch.equal(part[:n], part_ref[:n])


def test_op16_stride2_plane_rejected_outside_one_plane_modes(ops):
    """ABI 14: the 16-bit gathered operand of wgrad3s2 exists only in the bf16 / fp16 modes."""
    from mragan_hip import MraganError
    ops.set_conv_precision("bf16x3")
    try:
        x16 = torch.zeros(1, 16, 16, 32, 32, device="cuda", dtype=torch.bfloat16)
        dy = torch.zeros(1, 8, 8, 16, 64, device="cuda")
        gw = torch.empty(64 * 32 * 27, device="cuda")
        with pytest.raises((MraganError, ValueError)):
            ops.conv3d_wgrad_g16(dy, x16, 3, 2, 1, gw, False)
    finally:
        ops.set_conv_precision("f32")


@pytest.mark.parametrize("N,C,S,W,act", [(2, 128, 16, 16, "relu"), (1, 64, 9, 16, "relu"), (1, 128, 5, 32, "lrelu"),
                                          (2, 64, 6, 16, None)])
def test_op16_dgrad_backward_statistics(op16, N, C, S, W, act):
    """ABI 11: the whole-grid data gradient's epilogue partials of the preceding InstanceNorm's
    backward statistics give the same IN backward as the statistics pass: dz bit-identical to the
    plain data gradient, dx within fp32 summation-order noise of the statistics-pass result (the
    partials sum the fold in fp64 where the statistics pass sums it in fp32 first)."""
    ops = op16
    dt = ops.op16_dtype()
    g = torch.Generator().manual_seed(N * 13 + C + S)
    h1 = ndhwc(torch.randn(N, C, S, S, W, generator=g).float()).cuda()             # conv1 output (pre-IN)
    _, z16, mean, rstd = ops.instnorm_fwd_op16(h1, act=act, ypad=1)
    w = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    wp_b = pack(ops, w, False, True)
    ws_b = _presplit(ops, w, C, C, True)
    dh2 = ndhwc(torch.randn(N, C, S, S, W, generator=g).float()).cuda().to(dt)
    dz_ref, _ = ops.conv3d_op16(dh2, wp_b, C, 3, 1, 0, (S + 2, S + 2, W + 2), ws_b, transposed=True)
    part = ops.in_partials_buffer(N, (S + 2, S + 2, W + 2), C, "cuda")
    dz, chunks = ops.conv3d_op16_dgrad_in_stats(dh2, wp_b, C, ws_b, h1, mean, rstd, act, part)
    assert chunks > 0
    assert torch.equal(dz, dz_ref)
    ref = ops.instnorm_bwd(h1, mean, rstd, dz, 1, None, act=act)                     # fp32 statistics pass
    got = ops.instnorm_bwd_partials_op16(h1, mean, rstd, dz, 1, None, act, part, chunks)
    assert rel(got.float(), ref) < (4e-3 if dt == torch.bfloat16 else 6e-4)           # one 16-bit rounding
    plane = ops.instnorm_bwd_op16(h1, mean, rstd, dz, 1, None, act=act)
    # 16-bit words that differ from the statistics-pass plane: only round-half cases of ~1e-7 shifts
    assert (got != plane).float().mean().item() < 1e-3


@pytest.mark.parametrize("N,S,act,nc", [(2, 16, "relu", 1), (1, 13, "lrelu", 1), (2, 16, "relu", 2),
                                        (1, 13, "lrelu", 2)])
def test_head_dgrad_backward_statistics(x3, N, S, act, nc):
    """ABI 12: the G head's data gradient (conv 32 → nc, k7 p0, transposed form on the thin1 ring
    kernel; nc = 2 in the one-plane modes) leaves the backward statistics of the InstanceNorm in
    front of the head (its output replication-padded by 3): dz bit-identical to the plain data
    gradient, dx within fp32 summation-order noise of the statistics-pass result."""
    ops = x3
    if nc == 2 and ops.get_conv_precision() == "bf16x3":
        pytest.skip("two-channel thin1 runs in the one-plane modes only")
    C, k, f = 32, 7, 3
    g = torch.Generator().manual_seed(N * 17 + S)
    x = ndhwc(torch.randn(N, C, S, S, S, generator=g).float()).cuda()                # up-conv output (pre-IN)
    _, mean, rstd = ops.instnorm_fwd(x, act=act, ypad=f)
    w = torch.randn(nc, C, k, k, k, generator=g, dtype=torch.float64) * 0.02         # head Conv3d(32 → nc)
    wp_b = pack(ops, w, False, True)
    P = S + 2 * f
    O = P - k + 1
    dy = ndhwc(torch.randn(N, nc, O, O, O, generator=g).float()).cuda()
    dz_ref = ops.conv3d(dy, wp_b, C, k, 1, 0, (P, P, P), transposed=True)
    part = ops.in_partials_buffer(N, (P, P, P), C, "cuda")
    dz, chunks = ops.conv3d_dgrad_in_stats(dy, wp_b, C, k, x, mean, rstd, act, f, part)
    assert chunks > 0
    assert torch.equal(dz, dz_ref)
    ref = ops.instnorm_bwd(x, mean, rstd, dz, f, None, act=act)                      # statistics pass
    got = ops.instnorm_bwd_partials(x, mean, rstd, dz, f, None, act, part, chunks)
    assert rel(got, ref) < 1e-5


@pytest.mark.parametrize("N,cin,cout,S,k,tr,act,expect", [
    (2, 128, 64, 16, 3, True, "relu", True),     # G down2's data gradient (convT form) → down1's IN
    (2, 32, 64, 16, 3, True, "lrelu", True),     # convT form, 32 → 64 channels
    (2, 32, 64, 32, 3, False, "relu", True),     # G up2's data gradient (forward form) → up1's IN
    (1, 64, 32, 8, 3, True, "lrelu", True),      # 32 output channels: brickT's epilogue (round 5)
    (2, 64, 32, 8, 4, True, "lrelu", None),      # PatchGAN layer 2's data gradient (k4 s2 p1, convT form, 8³ → 16³)
    (2, 128, 64, 4, 4, True, "lrelu", None),     # PatchGAN layer 3's data gradient (4³ → 8³)
    (2, 32, 64, 16, 4, False, "lrelu", None),    # k4 s2 p1 in the forward form
    (1, 128, 32, 5, 3, True, "relu", True),      # ragged: 5³ → 9³ (output padding 0): brickT's partial bricks
])
def test_stride2_dgrad_backward_statistics(x3, N, cin, cout, S, k, tr, act, expect):
    """ABI 12: the stride-2 data gradient's implicit-GEMM epilogue leaves the backward statistics of
    the InstanceNorm whose output was the layer's input: output bit-identical to the plain conv, dx
    within fp32 summation-order noise of the statistics-pass result.  (tr: the conv run here is
    the transposed form, i.e. the data gradient of a forward stride-2 conv.)"""
    ops = x3
    g = torch.Generator().manual_seed(N * 19 + cin + cout + S)
    x = ndhwc(torch.randn(N, cin, S, S, S, generator=g).float()).cuda()
    w = torch.randn(cin, cout, k, k, k, generator=g, dtype=torch.float64) * 0.05 if tr else \
        torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) * 0.05
    wp = pack(ops, w, tr, False)
    # the data gradient of Conv3d(k, s2, p1) from an even size (k4: output padding 0); the ragged
    # case (S = 5, k3, output padding 0: 9³ outputs, parity classes of 5 and 4): on brickT since
    # round 5, whose partial bricks count only the voxels inside the output
    op = 0 if (k == 4 or S % 2) else 1
    o = ops.convT_out_size(S, k, 2, 1, op) if tr else ops.conv_out_size(S, k, 2, 1)
    osp = (o, o, o)
    y_ref = ops.conv3d(x, wp, cout, k, 2, 1, osp, transposed=tr)
    xin = ndhwc(torch.randn(N, cout, o, o, o, generator=g).float()).cuda()          # the IN's input
    _, mean, rstd = ops.instnorm_fwd(xin, act=act)
    part = ops.in_partials_buffer(N, osp, cout, "cuda")
    y, chunks = ops.conv3d_bwd_stats(x, wp, cout, k, 2, 1, osp, None, xin, mean, rstd, act, part, transposed=tr)
    assert torch.equal(y, y_ref)
    if expect is not None:
        assert (chunks > 0) == expect
    ref = ops.instnorm_bwd(xin, mean, rstd, y, 0, None, act=act)
    if chunks:
        got = ops.instnorm_bwd_partials(xin, mean, rstd, y, 0, None, act, part, chunks)
        assert rel(got, ref) < 1e-5


def test_op16_rejected_outside_16bit_modes(ops):
    from mragan_hip import MraganError
    ops.set_conv_precision("bf16x3")
    try:
        x = torch.zeros(1, 4, 4, 4, 64, device="cuda")
        with pytest.raises((MraganError, ValueError)):
            ops.instnorm_fwd_op16(x)
    finally:
        ops.set_conv_precision("f32")


@pytest.mark.parametrize("N,cin,cout,S,k,s,p,tr,expect,dc", [
    (2, 32, 64, 16, 3, 2, 1, False, True, 0),      # G down1 (k3 s2 p1)
    (2, 64, 128, 32, 3, 2, 1, False, True, 0),     # G down2 (16³ outputs: no K split)
    (2, 128, 64, 8, 3, 2, 1, True, True, 0),       # G up1 (ConvTranspose3d k3 s2 p1 op1)
    (2, 64, 32, 8, 3, 2, 1, True, True, 0),        # G up2 (32 output channels: brickT epilogue partials)
    (1, 64, 32, 6, 3, 2, 1, True, True, 0),        # up2 form with partial 4×16×16 output bricks (12³)
    (2, 1, 32, 22, 7, 1, 0, False, True, 0),       # G stem (k7, 1 → 32: thin1 epilogue partials, 16³)
    (1, 1, 32, 27, 7, 1, 0, False, True, 0),       # stem form with partial 16×16 output columns (21³)
    (2, 1, 32, 22, 7, 1, 0, False, True, 10.0),    # stem on a non-centred volume (x + 10): fp64 partials
    (2, 2, 32, 22, 7, 1, 0, False, "1p", 0),       # nc = 2 stem: thin1 with two channels (one-plane modes)
    (1, 2, 32, 27, 7, 1, 0, False, "1p", 0),       # … with partial output columns
    (2, 32, 64, 16, 4, 2, 1, False, False, 0),     # PatchGAN layer 2 (k4 s2 p1): split in K → stats pass
    (1, 256, 256, 8, 4, 2, 1, False, False, 0),    # UNet inner down conv: 16 slices → stats pass
    (1, 128, 256, 8, 4, 1, 1, False, False, 0),    # PatchGAN layer 4: 7³ rows, no whole tiles → stats pass
])
def test_igemm_in_stats_partials(x3, N, cin, cout, S, k, s, p, tr, expect, dc):
    """ABI 11: the 16-bit implicit GEMM's epilogue InstanceNorm partials (no K split, tiles inside
    one instance and class) and the brickT epilogue's (per output brick) feed mragan_instnorm_fwd_partials; output, mean / rstd and the
    normalised tensor match the statistics-pass path."""
    ops = x3
    if expect == "1p":
        expect = ops.get_conv_precision() in ("bf16", "fp16")
    g = torch.Generator().manual_seed(N * 7 + cin + cout + S + k)
    x = torch.randn(N, cin, S, S, S, generator=g, dtype=torch.float64) + dc
    shape_w = (cin, cout, k, k, k) if tr else (cout, cin, k, k, k)
    w = torch.randn(*shape_w, generator=g, dtype=torch.float64) * 0.05
    xg = ndhwc(x.float()).cuda()
    wp = pack(ops, w, tr, False)
    if tr:
        o = ops.convT_out_size(S, k, s, p, 1)
    else:
        o = ops.conv_out_size(S, k, s, p)
    osp = (o, o, o)
    y_ref = ops.conv3d(xg, wp, cout, k, s, p, osp, transposed=tr)
    part = ops.in_partials_buffer(N, osp, cout, "cuda")
    y, chunks = ops.conv3d_in_stats(xg, wp, cout, k, s, p, osp, None, part, transposed=tr)
    if expect:
        assert chunks > 0
    assert torch.equal(y, y_ref)
    z_ref, m_ref, r_ref = ops.instnorm_fwd(y_ref, act="lrelu", ypad=1)
    z, m, r = ops.instnorm_fwd(y, act="lrelu", ypad=1, part=part, chunks=chunks)
    assert rel(m, m_ref) < 1e-6 and rel(r, r_ref) < 1e-6
    assert rel(z, z_ref) < 1e-6


def test_instnorm_single_voxel_raises(ops):
    from mragan_hip import MraganError
    with pytest.raises(MraganError, match="more than 1 spatial element"):
        ops.instnorm_fwd(torch.zeros(1, 1, 1, 1, 8, device="cuda"))


@pytest.mark.parametrize("C,p", [(1, 3), (32, 1), (2, 3)])
def test_rpad_and_fold(ops, C, p):
    g = torch.Generator().manual_seed(C + p)
    x = torch.randn(2, C, 5, 6, 7, generator=g, dtype=torch.float64, requires_grad=True)
    y = F.pad(x, (p,) * 6, mode="replicate")
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (dx_ref,) = torch.autograd.grad(y, x, dy)
    out = ops.rpad(ndhwc(x.detach().float()).cuda(), p)
    assert rel(ncdhw(out), y.detach()) < 1e-7
    add = torch.randn(x.shape, generator=g, dtype=torch.float64)
    dx = ops.rpad_fold(ndhwc(dy.float()).cuda(), p, add=ndhwc(add.float()).cuda())
    assert rel(ncdhw(dx), dx_ref + add) < 1e-6


@pytest.mark.parametrize("lsgan", [False, True])
@pytest.mark.parametrize("target", [0.0, 1.0])
def test_gan_loss(ops, lsgan, target):
    """Loss value and d(loss)/d(D output) — the Sigmoid backward is D's last layer's job."""
    g = torch.Generator().manual_seed(3)
    z = torch.randn(2, 1, 6, 6, 6, generator=g, dtype=torch.float64)
    p = (z if lsgan else torch.sigmoid(z)).requires_grad_()
    if lsgan:
        loss = ((p - target) ** 2).mean()
    else:
        loss = F.binary_cross_entropy(p, torch.full_like(p, target))
    (dp,) = torch.autograd.grad(0.5 * loss, p)
    slot = torch.zeros(1, device="cuda")
    dout = torch.empty(p.numel(), device="cuda")
    ops.gan_loss(p.detach().float().cuda().reshape(-1), target, lsgan, 0.5, slot, dout)
    assert abs(float(slot) - 0.5 * float(loss.detach())) < 1e-6 * max(1.0, abs(float(loss.detach())))
    assert rel(dout, dp.reshape(-1)) < 1e-5


def test_l1_loss(ops):
    g = torch.Generator().manual_seed(4)
    a = torch.randn(3, 5, 7, 9, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(3, 5, 7, 9, generator=g, dtype=torch.float64)
    loss = (a - b).abs().mean() * 5.0
    (da,) = torch.autograd.grad(loss, a)
    slot = torch.zeros(1, device="cuda")
    grad = torch.empty(a.numel(), device="cuda")
    ops.l1_loss(a.detach().float().cuda(), b.float().cuda(), 5.0, slot, grad)
    assert abs(float(slot) - float(loss)) < 1e-5
    assert rel(grad, da.reshape(-1)) < 1e-6
    # the loss scale (fp16 mode) multiplies the emitted gradients only, exactly (a power of two)
    try:
        ops.set_loss_scale(1024.0)
        slot2 = torch.zeros(1, device="cuda")
        grad2 = torch.empty_like(grad)
        ops.l1_loss(a.detach().float().cuda(), b.float().cuda(), 5.0, slot2, grad2)
        dp = torch.empty(a.numel(), device="cuda")
        dp2 = torch.empty_like(dp)
        p = torch.rand(a.numel(), generator=g).float().cuda() * 0.9 + 0.05
        ops.set_loss_scale(1.0)
        ops.gan_loss(p, 1.0, False, 0.5, torch.zeros(1, device="cuda"), dp)
        ops.set_loss_scale(1024.0)
        s2 = torch.zeros(1, device="cuda")
        ops.gan_loss(p, 1.0, False, 0.5, s2, dp2)
    finally:
        ops.set_loss_scale(1.0)
    assert float(slot2) == float(slot)
    assert torch.equal(grad2, grad * 1024.0)
    assert torch.equal(dp2, dp * 1024.0)


def test_adam_matches_torch_formula(ops):
    from oracle.cyclegan_oracle import adam_update
    g = torch.Generator().manual_seed(5)
    n = 10007
    p0 = torch.randn(n, generator=g)
    m0, v0 = torch.zeros(n), torch.zeros(n)
    pd, md, vd = p0.cuda(), m0.cuda(), v0.cuda()
    p, m, v = p0.clone(), m0.clone(), v0.clone()
    for step in range(1, 4):
        gr = torch.randn(n, generator=g)
        adam_update(p, gr, m, v, step, 2e-4, 0.5)
        ops.adam(pd, gr.cuda(), md, vd, 2e-4, 0.5, 0.999, 1e-8, step)
    assert rel(pd, p) < 1e-7
    assert rel(md, m) < 1e-6


def test_channel_sum(ops):
    x = torch.randn(1000, 12)
    out = torch.empty(12, device="cuda")
    ops.channel_sum(x.cuda(), out)
    assert rel(out, x.sum(0)) < 1e-6


@pytest.mark.parametrize("N,cin,cout,S", [(2, 16, 1, 8), (1, 16, 2, 6)])
def test_conv_transpose3d_thin_bias_tanh(ops, N, cin, cout, S):
    """UnetGenerator outermost upconv: ConvTranspose3d(2ngf → nc, k4 s2 p1) + bias + Tanh fused."""
    g = torch.Generator().manual_seed(cin + cout + S)
    x = torch.randn(N, cin, S, S + 1, S, generator=g, dtype=torch.float64)
    w = torch.randn(cin, cout, 4, 4, 4, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(cout, generator=g, dtype=torch.float64)
    ref = torch.tanh(F.conv_transpose3d(x, w, b, stride=2, padding=1))
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, True, False), cout, 4, 2, 1, ref.shape[2:],
                     bias=b.float().cuda(), act="tanh", transposed=True)
    assert rel(ncdhw(out), ref) < TOL


@pytest.mark.parametrize("Ca,Cb", [(8, 8), (16, 16), (3, 5)])
def test_channel_concat_split(ops, Ca, Cb):
    """UNet skip: relu(cat([lrelu(x), u], 1)) forward and its backward."""
    g = torch.Generator().manual_seed(Ca * 10 + Cb)
    a = torch.randn(2, Ca, 3, 4, 5, generator=g, dtype=torch.float64, requires_grad=True)
    u = torch.randn(2, Cb, 3, 4, 5, generator=g, dtype=torch.float64, requires_grad=True)
    r = torch.relu(torch.cat([a, u], 1))
    out = ops.channel_concat(ndhwc(a.detach().float()).cuda(), "relu", ndhwc(u.detach().float()).cuda(), None)
    assert rel(ncdhw(out), torch.cat([torch.relu(a), u], 1).detach()) < 1e-7
    dr = torch.randn(r.shape, generator=g, dtype=torch.float64)
    da_ref, du_ref = torch.autograd.grad(r, (a, u), dr)
    da, du = ops.channel_split(ndhwc(dr.float()).cuda(), Ca, ndhwc(a.detach().float()).cuda(), "relu", None, None)
    assert rel(ncdhw(da), da_ref) < 1e-7
    assert rel(ncdhw(du), dr[:, Ca:]) < 1e-7      # raw: the IN backward applies ReLU'


@pytest.mark.parametrize("N,ngf,S,p", [(2, 32, 12, 0), (1, 32, 40, 0), (1, 32, 11, 3), (2, 32, 9, 3)])
def test_thin1_bf16x3_stem_fwd_head_dgrad(x3, N, ngf, S, p):
    """1 → ngf k7 s1 convolutions on the bf16x3 MFMA path (conv_thin1_x3.hip): the G stem forward
    and the G head's data gradient (transposed form, flipped taps), incl. partial w/h/d tiles."""
    ops = x3
    g = torch.Generator().manual_seed(ngf + S + p)
    x = torch.randn(N, 1, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = torch.randn(ngf, 1, 7, 7, 7, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(ngf, generator=g, dtype=torch.float64)
    y = F.conv3d(x, w, b, padding=p)
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, False, False), ngf, 7, 1, p, y.shape[2:],
                     bias=b.float().cuda(), act="lrelu")
    check_rounded(ncdhw(out), F.leaky_relu(F.conv3d(R(x), R(w), b, padding=p), 0.2), F.leaky_relu(y, 0.2))
    xh = torch.randn(N, ngf, S, S + 1, S + 2, generator=g, dtype=torch.float64, requires_grad=True)
    wh = torch.randn(1, ngf, 7, 7, 7, generator=g, dtype=torch.float64) * 0.1
    yh = F.conv3d(xh, wh, padding=p)
    dy = torch.randn(yh.shape, generator=g, dtype=torch.float64)
    (dx_ref,) = torch.autograd.grad(yh, xh, dy)
    dx = ops.conv3d(ndhwc(dy.float()).cuda(), pack(ops, wh, False, True), ngf, 7, 1, p, xh.shape[2:], transposed=True)
    check_rounded(ncdhw(dx), torch.nn.grad.conv3d_input(xh.shape, R(wh), R(dy), padding=p), dx_ref)


@pytest.mark.parametrize("N,ngf,S,p", [(2, 32, 12, 0), (1, 32, 37, 0), (2, 32, 9, 3)])
def test_thin1_bf16x3_wgrad(x3, N, ngf, S, p):
    """Weight gradients of the 1-channel k7 convolutions on the bf16x3 MFMA path
    (conv_thin1_wgrad_x3.hip): G stem Conv3d(1→ngf) and G head Conv3d(ngf→1), partial bricks."""
    ops = x3
    g = torch.Generator().manual_seed(7 * ngf + S + p)
    x = torch.randn(N, 1, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = (torch.randn(ngf, 1, 7, 7, 7, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    y = F.conv3d(x, w, padding=p)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (dw_ref,) = torch.autograd.grad(y, w, dy)
    dw = torch.full((ngf, 1, 7, 7, 7), 3.0, device="cuda")
    dw_rnd = torch.nn.grad.conv3d_weight(R(x), w.shape, R(dy), padding=p)
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), 7, 1, p, dw, accumulate=False)
    check_rounded(dw, dw_rnd, dw_ref)
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), 7, 1, p, dw, accumulate=True)
    check_rounded(dw, 2 * dw_rnd, 2 * dw_ref)
    xh = torch.randn(N, ngf, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    wh = (torch.randn(1, ngf, 7, 7, 7, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    yh = F.conv3d(xh, wh, padding=p)
    dz = torch.randn(yh.shape, generator=g, dtype=torch.float64)
    (dwh_ref,) = torch.autograd.grad(yh, wh, dz)
    dwh = torch.empty(1, ngf, 7, 7, 7, device="cuda")
    ops.conv3d_wgrad(ndhwc(dz.float()).cuda(), ndhwc(xh.float()).cuda(), 7, 1, p, dwh, accumulate=False)
    check_rounded(dwh, torch.nn.grad.conv3d_weight(R(xh), wh.shape, R(dz), padding=p), dwh_ref)


@pytest.mark.parametrize("N,S,p", [(2, 12, 0), (1, 37, 0), (2, 9, 3), (1, 70, 0)])
def test_thinn_bf16x3_head_fwd_stem_dgrad(x3, N, S, p):
    """32 → 1 k7 s1 convolutions on the bf16x3 MFMA path (conv_thinn_x3.hip): the G head forward
    (bias + tanh fused) and the G stem's data gradient (transposed form, flipped taps)."""
    ops = x3
    g = torch.Generator().manual_seed(3 * S + p + N)
    x = torch.randn(N, 32, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = torch.randn(1, 32, 7, 7, 7, generator=g, dtype=torch.float64) * 0.05
    b = torch.randn(1, generator=g, dtype=torch.float64)
    y = torch.tanh(F.conv3d(x, w, b, padding=p))
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, False, False), 1, 7, 1, p, y.shape[2:],
                     bias=b.float().cuda(), act="tanh")
    check_rounded(ncdhw(out), torch.tanh(F.conv3d(R(x), R(w), b, padding=p)), y)
    xs = torch.randn(N, 1, S, S + 1, S + 2, generator=g, dtype=torch.float64, requires_grad=True)
    ws = torch.randn(32, 1, 7, 7, 7, generator=g, dtype=torch.float64) * 0.05
    ys = F.conv3d(xs, ws, padding=p)
    dy = torch.randn(ys.shape, generator=g, dtype=torch.float64)
    (dx_ref,) = torch.autograd.grad(ys, xs, dy)
    dx = ops.conv3d(ndhwc(dy.float()).cuda(), pack(ops, ws, False, True), 1, 7, 1, p, xs.shape[2:], transposed=True)
    check_rounded(ncdhw(dx), torch.nn.grad.conv3d_input(xs.shape, R(ws), R(dy), padding=p), dx_ref)


@pytest.mark.parametrize("N,cin,S,k,op", [(2, 64, 8, 3, 1), (1, 64, 13, 3, 1), (2, 128, 6, 4, 0), (1, 32, 9, 4, 0)])
def test_brickT_bf16x3(x3, N, cin, S, k, op):
    """Stride-2 transposed convolutions to 32 channels on the LDS-halo path (conv_brickT_x3.hip):
    ConvTranspose3d k3 s2 p1 op1 / k4 s2 p1 forward and the equivalent Conv3d data gradients,
    incl. partial output bricks."""
    ops = x3
    g = torch.Generator().manual_seed(cin + S + k)
    x = torch.randn(N, cin, S, S + 1, S + 2, generator=g, dtype=torch.float64)
    w = torch.randn(cin, 32, k, k, k, generator=g, dtype=torch.float64) * 0.1
    y = F.conv_transpose3d(x, w, stride=2, padding=1, output_padding=op)
    out = ops.conv3d(ndhwc(x.float()).cuda(), pack(ops, w, True, False), 32, k, 2, 1, y.shape[2:], transposed=True)
    check_rounded(ncdhw(out), F.conv_transpose3d(R(x), R(w), stride=2, padding=1, output_padding=op), y)
    # the same form as the data gradient of Conv3d(32 → cin, k, s2, p1)
    xc = torch.randn(N, 32, 2 * S, 2 * S + 1, 2 * S + 2, generator=g, dtype=torch.float64, requires_grad=True)
    wc = torch.randn(cin, 32, k, k, k, generator=g, dtype=torch.float64) * 0.1
    yc = F.conv3d(xc, wc, stride=2, padding=1)
    dy = torch.randn(yc.shape, generator=g, dtype=torch.float64)
    (dx_ref,) = torch.autograd.grad(yc, xc, dy)
    dx = ops.conv3d(ndhwc(dy.float()).cuda(), pack(ops, wc, False, True), 32, k, 2, 1, xc.shape[2:], transposed=True)
    check_rounded(ncdhw(dx), torch.nn.grad.conv3d_input(xc.shape, R(wc), R(dy), stride=2, padding=1), dx_ref)


@pytest.mark.parametrize("N,cin,cout,D,H,W", [(4, 128, 128, 16, 16, 16), (2, 128, 128, 8, 9, 16), (1, 64, 192, 5, 3, 32),
                                              (3, 64, 64, 7, 2, 16), (1, 192, 64, 2, 2, 48)])
def test_wgrad3_bf16x3(x3, N, cin, cout, D, H, W):
    """Multi-tap weight gradient (conv_wgrad3_x3.hip) of the ResnetBlock form: valid k3 s1 conv
    on a (D+2, H+2, W+2) input, W a multiple of 16 — incl. partial last stages, several channel
    tiles and several w-segments per row."""
    ops = x3
    g = torch.Generator().manual_seed(N + cin + D * H + W)
    x = torch.randn(N, cin, D + 2, H + 2, W + 2, generator=g, dtype=torch.float64)
    w = (torch.randn(cout, cin, 3, 3, 3, generator=g, dtype=torch.float64) * 0.1).requires_grad_()
    y = F.conv3d(x, w)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (dw_ref,) = torch.autograd.grad(y, w, dy)
    dw = torch.full((cout, cin, 3, 3, 3), 3.0, device="cuda")
    dw_rnd = torch.nn.grad.conv3d_weight(R(x), w.shape, R(dy))
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), 3, 1, 0, dw, accumulate=False)
    check_rounded(dw, dw_rnd, dw_ref)
    ops.conv3d_wgrad(ndhwc(dy.float()).cuda(), ndhwc(x.float()).cuda(), 3, 1, 0, dw, accumulate=True)
    check_rounded(dw, 2 * dw_rnd, 2 * dw_ref)


def test_pack_weights_batched_equals_single(ops):
    """mragan_pack_weights (one launch for a network's packs) = mragan_pack_weight per pack."""
    g = torch.Generator().manual_seed(21)
    packs, ref = [], []
    # tiled LDS path (A % 8, B % 16, T ≤ 64) and element-wise path; fp32 tr 0/1 and the bf16 / fp16
    # split fragment orders tr 2..5 (T = 27, channels % 32)
    for (A, B, T, tr) in [(128, 128, 27, 0), (32, 1, 343, 1), (64, 32, 27, 1), (1, 32, 64, 0), (64, 128, 64, 1),
                          (256, 128, 64, 0), (128, 64, 27, 2), (64, 128, 27, 3), (128, 128, 27, 4),
                          (64, 96, 27, 5), (40, 32, 27, 2)]:
        src = torch.randn(A * B * T, generator=g).cuda()
        dst = torch.empty_like(src)
        want = torch.empty_like(src)
        ops.pack_weight(src, A, B, T, tr, want)
        packs.append((src, A, B, T, tr, dst))
        ref.append(want)
    tab = ops.PackTable()
    tab.run(packs)
    tab.run(packs)          # cached table path
    torch.cuda.synchronize()
    for (_, _, _, _, _, dst), want in zip(packs, ref):
        assert torch.equal(dst, want)


@pytest.mark.parametrize("N,cin,cout,S,transposed", [(2, 64, 128, 13, False), (1, 128, 128, 8, False),
                                                     (2, 128, 64, 9, True), (1, 128, 128, 7, True)])
def test_brick_presplit_equals_per_call_split(ops, N, cin, cout, S, transposed):
    """mragan_conv3d_presplit with weights split by a tr 2/3 batched pack is bit-identical to the
    brick kernel splitting the fp32 pack itself (both forms of a k3 s1 conv, bf16x3)."""
    prev = ops.get_conv_precision()
    ops.set_conv_precision("bf16x3")
    try:
        g = torch.Generator().manual_seed(5 + cin + S)
        w = (torch.randn(cout, cin, 3, 3, 3, generator=g) * 0.05).cuda()
        x = torch.randn(N, S, S, S, cin, generator=g).cuda()
        A, B, T = cout, cin, 27
        # forward form uses [t][cout][cin] (tr 0); the transposed form of the same layer's dgrad
        # uses [t][cin][cout] (tr 1) with ny = cin
        tr = 1 if transposed else 0
        ny = cin if transposed else cout
        if transposed:
            x = torch.randn(N, S, S, S, cout, generator=g).cuda()
        wp = torch.empty(w.numel(), device="cuda")
        wsp = torch.empty(w.numel(), device="cuda")
        ops.PackTable().run([(w, A, B, T, tr, wp), (w, A, B, T, 2 + tr, wsp)])
        single = torch.empty_like(wsp)
        ops.pack_weight(w, A, B, T, 2 + tr, single)
        want = ops.conv3d(x, wp, ny, 3, 1, 1, (S, S, S), transposed=transposed)
        got = ops.conv3d(x, wp, ny, 3, 1, 1, (S, S, S), transposed=transposed, wsplit=wsp)
        torch.cuda.synchronize()
        assert torch.equal(single, wsp)
        assert torch.equal(got, want)
    finally:
        ops.set_conv_precision(prev)


def test_x3_batch_over_2gib(ops):
    """A 16-bit-mode convolution whose batch tensor exceeds 2 GiB (the MFMA kernels address their
    operands with 32-bit byte offsets): conv_igemm runs it as consecutive instance ranges, the
    weight gradient accumulates over them (bf16 training at 128³ batch 2 reached
    2^31 bytes in G's batched down1 pass).  Checked against per-instance launches (the ops are per
    instance) and, for two instances, the fp32 CPU convolution of the rounded operands."""
    prev = ops.get_conv_precision()
    ops.set_conv_precision("bf16")
    try:
        N, S, cin, cout = 9, 128, 32, 64
        assert N * S ** 3 * cin * 4 > 2 ** 31
        gen = torch.Generator(device="cuda").manual_seed(3)
        x = torch.randn(N, S, S, S, cin, device="cuda", generator=gen)
        w = torch.randn(cout, cin, 3, 3, 3, device="cuda", generator=gen) * 0.05
        wp = pack(ops, w, False, False)
        osp = (S // 2,) * 3
        y = ops.conv3d(x, wp, cout, 3, 2, 1, osp)
        for n in (0, N - 1):
            yn = ops.conv3d(x[n:n + 1].contiguous(), wp, cout, 3, 2, 1, osp)
            assert rel(y[n:n + 1], yn) < 1e-6
        xr = R(x[N - 1:N].permute(0, 4, 1, 2, 3).cpu()).float()
        ref = F.conv3d(xr, R(w.cpu()).float(), stride=2, padding=1)
        assert rel(ncdhw(y[N - 1:N]), ref.double()) < 2e-5
        # weight gradient over the whole batch = the sum of two sub-batch gradients
        dy = torch.randn(N, *osp, cout, device="cuda", generator=gen)
        dw = torch.zeros(cout, cin, 3, 3, 3, device="cuda")
        ops.conv3d_wgrad(dy, x, 3, 2, 1, dw, accumulate=False)
        dw2 = torch.zeros_like(dw)
        ops.conv3d_wgrad(dy[:4].contiguous(), x[:4].contiguous(), 3, 2, 1, dw2, accumulate=False)
        ops.conv3d_wgrad(dy[4:].contiguous(), x[4:].contiguous(), 3, 2, 1, dw2, accumulate=True)
        assert rel(dw, dw2) < 1e-5
    finally:
        ops.set_conv_precision(prev)


def test_fp16_found_inf_skips_adam(ops):
    """fp16 loss scaling: a non-finite gradient anywhere in an optimizer's flat buffers leaves
    every parameter and both moments untouched and counts one skipped step."""
    g = torch.Generator().manual_seed(4)
    n = 100_003
    p = [torch.randn(n, generator=g).cuda() for _ in range(2)]
    gr = [torch.randn(n, generator=g).cuda() for _ in range(2)]
    m = [torch.zeros(n, device="cuda") for _ in range(2)]
    v = [torch.zeros(n, device="cuda") for _ in range(2)]
    hyper = torch.tensor(ops.adam_hyper(2e-4, 0.5, 0.999, 1e-8, 1, 1.0 / 1024), device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    count = torch.zeros(1, dtype=torch.int32, device="cuda")
    # clean step: updates, no skip
    p0 = [t.clone() for t in p]
    for t in gr:
        ops.nonfinite_flag(t, flag)
    for i in range(2):
        ops.adam_dev_checked(p[i], gr[i], m[i], v[i], hyper, flag)
    ops.skip_count(flag, count)
    torch.cuda.synchronize()
    assert int(count) == 0 and int(flag) == 0
    assert all(not torch.equal(a, b) for a, b in zip(p, p0))
    # overflow in the second buffer: nothing moves
    gr[1][n // 2] = float("inf")
    gr[1][7] = float("nan")
    snap = [t.clone() for t in p + m + v]
    for t in gr:
        ops.nonfinite_flag(t, flag)
    for i in range(2):
        ops.adam_dev_checked(p[i], gr[i], m[i], v[i], hyper, flag)
    ops.skip_count(flag, count)
    torch.cuda.synchronize()
    assert int(count) == 1 and int(flag) == 0
    assert all(torch.equal(a, b) for a, b in zip(p + m + v, snap))


def test_adam_rebias_skipped_steps(ops):
    """ABI 13: the device scalars for host step t with k skipped updates equal adam_hyper at t − k
    (bit for bit), so a skipped step does not advance the bias corrections (GradScaler semantics)."""
    lr, b1, b2, eps, scale = 2e-4, 0.5, 0.999, 1e-8, 1.0 / 1024
    hyper = torch.empty(6, device="cuda")
    for t, k in ((1, 0), (5, 0), (5, 2), (37, 11)):
        base = torch.tensor([lr, b1, b2, eps, float(t), scale], device="cuda")
        skipped = torch.tensor([k], dtype=torch.int32, device="cuda")
        ops.adam_rebias(base, skipped, hyper)
        torch.cuda.synchronize()
        want = torch.tensor(ops.adam_hyper(lr, b1, b2, eps, t - k, scale))
        assert torch.equal(hyper.cpu(), want), (t, k, hyper.cpu(), want)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_stale_fp32_packs_not_exposed(ops, prec):
    """The per-step repack skips a ResnetBlock conv's fp32 packs in the one-plane modes (its kernels
    read the pre-split copies): the layer then exposes no fp32 pack (wp_fwd / wp_bwd are None, so no
    kernel can read the stale buffers — ABI 19), and its forward and data gradient still run, on
    the pre-split copies, against fp64 of the rounded operands."""
    from mragan_hip import engine
    ops.set_conv_precision(prec)
    try:
        import types
        torch.manual_seed(0)
        C = 64
        w = torch.nn.Parameter(torch.randn(C, C, 3, 3, 3, device="cuda") * 0.05)
        m = types.SimpleNamespace(weight=w, kernel_size=3, stride=1, padding=0, in_channels=C, out_channels=C)
        layer = engine.ConvLayer(m, False)
        for src, A, B, T, tr, dst in layer.packs():
            ops.pack_weight(src, A, B, T, tr, dst)
        if engine._FP32_PACKS:
            pytest.skip("fp32 packs refreshed by every repack in this environment")
        assert layer.fp32_stale and layer.wp_fwd is None and layer.wp_bwd is None
        dt = ops.op16_dtype()
        N, S = 2, 24
        x = ndhwc(torch.randn(N, C, S + 2, S + 2, S + 2).float()).cuda()
        y, _, _ = layer.forward_in_stats_op16(x.to(dt))
        dz = layer.dgrad_op16(y.to(dt), (S + 2,) * 3)
        torch.cuda.synchronize()
        wr = w.detach().double().cpu().to(dt).double()
        y64 = F.conv3d(ncdhw(x.to(dt).double().cpu()), wr)
        assert rel(ncdhw(y.double().cpu()), y64) < 2e-5
        dz64 = F.conv_transpose3d(ncdhw(y.to(dt).double().cpu()), wr)
        assert rel(ncdhw(dz.double().cpu()), dz64) < 2e-5
    finally:
        ops.set_conv_precision("f32")
