"""torch.ops.mragan.* on the GPU (mragan_hip/torch_ops.py): forward and autograd of each
registered op against float64 PyTorch-CPU modules (nn.Conv3d / ConvTranspose3d, InstanceNorm3d,
ReplicationPad3d — the reference's layers, networks3D.py:15-24, 183-213) in the fp32 mode;
relative L2 gate 1e-5 as test_kernels_gpu.py."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 1e-5
ACTF = {"none": lambda t: t, "relu": F.relu, "lrelu": lambda t: F.leaky_relu(t, 0.2), "tanh": torch.tanh}


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def ndhwc(t):
    return t.permute(0, 2, 3, 4, 1).contiguous()


def ncdhw(t):
    return t.permute(0, 4, 1, 2, 3)


@pytest.fixture(scope="module")
def tops():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mragan_hip import ops
    import mragan_hip.torch_ops as m
    ops.set_conv_precision("f32")
    ops.set_loss_scale(1.0)
    return m


@pytest.mark.parametrize("transposed,N,cin,cout,S,k,s,p,op,bias,act", [
    (False, 2, 8, 16, 9, 3, 2, 1, 0, True, "none"),
    (False, 1, 16, 32, 8, 3, 1, 1, 0, False, "relu"),
    (False, 2, 1, 8, 14, 7, 1, 0, 0, False, "none"),       # stem-shaped (k7, one input channel)
    (False, 1, 8, 16, 10, 4, 2, 1, 0, True, "lrelu"),      # PatchGAN layer
    (True, 2, 16, 8, 6, 3, 2, 1, 1, False, "none"),        # G up (ConvTranspose3d, output_padding 1)
    (False, 1, 8, 1, 12, 7, 1, 0, 0, True, "tanh"),        # head-shaped (k7 → 1 channel + Tanh)
])
def test_conv3d_op_and_grad(tops, transposed, N, cin, cout, S, k, s, p, op, bias, act):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, cin, S, S, S, generator=g, dtype=torch.float64)
    w = torch.randn(*((cin, cout) if transposed else (cout, cin)), k, k, k, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(cout, generator=g, dtype=torch.float64) if bias else None
    # float64 CPU reference through torch autograd
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    br = b.clone().requires_grad_() if bias else None
    if transposed:
        yr = F.conv_transpose3d(xr, wr, br, stride=s, padding=p, output_padding=op)
    else:
        yr = F.conv3d(xr, wr, br, stride=s, padding=p)
    yr = ACTF[act](yr)
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    # the registered op on NDHWC device tensors
    xd = ndhwc(x.float()).cuda().requires_grad_()
    wd = w.float().cuda().requires_grad_()
    bd = b.float().cuda().requires_grad_() if bias else None
    y = torch.ops.mragan.conv3d(xd, wd, bd, s, p, op, transposed, act)
    assert rel(ncdhw(y.detach()), yr.detach()) < TOL
    y.backward(ndhwc(dy.float()).cuda())
    assert rel(ncdhw(xd.grad), xr.grad) < TOL
    assert rel(wd.grad, wr.grad) < TOL
    if bias:
        assert rel(bd.grad, br.grad) < TOL


@pytest.mark.parametrize("act,ypad", [("none", 0), ("relu", 1), ("lrelu", 0), ("relu", 3)])
def test_instance_norm_op_and_grad(tops, act, ypad):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 16, 8, 8, 8, generator=g, dtype=torch.float64) * 3 + 1
    xr = x.clone().requires_grad_()
    yr = ACTF[act](F.instance_norm(xr, eps=1e-5))
    if ypad:
        yr = F.pad(yr, (ypad,) * 6, mode="replicate")
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    xd = ndhwc(x.float()).cuda().requires_grad_()
    y, mean, rstd = torch.ops.mragan.instance_norm(xd, act, ypad)
    assert rel(ncdhw(y.detach()), yr.detach()) < TOL
    assert rel(mean, x.mean(dim=(2, 3, 4))) < TOL
    assert rel(rstd, (x.var(dim=(2, 3, 4), unbiased=False) + 1e-5).rsqrt()) < TOL
    y.backward(ndhwc(dy.float()).cuda())
    assert rel(ncdhw(xd.grad), xr.grad) < TOL


def test_replication_pad_op_and_grad(tops):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, 4, 6, 7, 5, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_()
    yr = F.pad(xr, (3,) * 6, mode="replicate")
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    xd = ndhwc(x.float()).cuda().requires_grad_()
    y = torch.ops.mragan.replication_pad(xd, 3)
    assert torch.equal(ncdhw(y.detach()).cpu().double(), yr.detach().float().double())
    y.backward(ndhwc(dy.float()).cuda())
    assert rel(ncdhw(xd.grad), xr.grad) < TOL


def test_composed_block_matches_torch(tops):
    """A ResnetBlock-shaped composition (RPad1 → Conv k3 → IN+ReLU → RPad1 → Conv k3 → IN, + x;
    networks3D.py:233-257) through the registered ops, forward and input gradient."""
    g = torch.Generator().manual_seed(3)
    C, S = 16, 8
    x = torch.randn(1, C, S, S, S, generator=g, dtype=torch.float64)
    w1 = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    w2 = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
    xr = x.clone().requires_grad_()
    h = F.relu(F.instance_norm(F.conv3d(F.pad(xr, (1,) * 6, mode="replicate"), w1), eps=1e-5))
    yr = xr + F.instance_norm(F.conv3d(F.pad(h, (1,) * 6, mode="replicate"), w2), eps=1e-5)
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    xd = ndhwc(x.float()).cuda().requires_grad_()
    mr = torch.ops.mragan
    h1 = mr.instance_norm(mr.conv3d(mr.replication_pad(xd, 1), w1.float().cuda(), None, 1, 0, 0, False, "none"),
                          "relu", 1)[0]             # IN output already replication-padded by 1
    y = xd + mr.instance_norm(mr.conv3d(h1, w2.float().cuda(), None, 1, 0, 0, False, "none"), "none", 0)[0]
    assert rel(ncdhw(y.detach()), yr.detach()) < TOL
    y.backward(ndhwc(dy.float()).cuda())
    assert rel(ncdhw(xd.grad), xr.grad) < TOL


@pytest.mark.parametrize("n", [1, 1000, 262144 + 17])
def test_l1_loss_op_and_grad(tops, n):
    g = torch.Generator().manual_seed(n)
    a, b = torch.randn(n, generator=g, dtype=torch.float64), torch.randn(n, generator=g, dtype=torch.float64)
    ar, br = a.clone().requires_grad_(), b.clone().requires_grad_()
    lr_ = F.l1_loss(ar, br)
    (2.5 * lr_).backward()
    ad, bd = a.float().cuda().requires_grad_(), b.float().cuda().requires_grad_()
    loss = torch.ops.mragan.l1_loss(ad, bd)
    assert abs(float(loss.detach()) - float(lr_.detach())) <= 1e-5 * abs(float(lr_.detach()))
    (2.5 * loss).backward()
    assert rel(ad.grad, ar.grad) < TOL
    assert rel(bd.grad, br.grad) < TOL


@pytest.mark.parametrize("lsgan,target", [(True, 1.0), (True, 0.0), (False, 1.0), (False, 0.0)])
def test_gan_loss_op_and_grad(tops, lsgan, target):
    g = torch.Generator().manual_seed(9)
    p = torch.rand(2, 1, 6, 6, 6, generator=g, dtype=torch.float64) * 0.9 + 0.05
    pr = p.clone().requires_grad_()
    t = torch.full_like(p, target)
    lr_ = F.mse_loss(pr, t) if lsgan else F.binary_cross_entropy(pr, t)
    lr_.backward()
    pd = ndhwc(p.float()).cuda().requires_grad_()
    loss = torch.ops.mragan.gan_loss(pd, target, lsgan)
    assert abs(float(loss.detach()) - float(lr_.detach())) <= 1e-5 * max(abs(float(lr_.detach())), 1e-6)
    loss.backward()
    assert rel(ncdhw(pd.grad), pr.grad) < TOL


def test_adam_op_matches_torch(tops):
    g = torch.Generator().manual_seed(4)
    n = 4097
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) for _ in range(3)]
    pr = p0.clone().requires_grad_()
    opt = torch.optim.Adam([pr], lr=2e-4, betas=(0.5, 0.999), eps=1e-8)
    p, m, v = p0.cuda(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    for step, gr in enumerate(grads, 1):
        pr.grad = gr.clone()
        opt.step()
        torch.ops.mragan.adam_(p, gr.cuda(), m, v, 2e-4, 0.5, 0.999, 1e-8, step, 1.0)
    assert rel(p, pr.detach()) < 1e-6
    assert rel(m, opt.state[pr]["exp_avg"]) < 1e-6


def test_opcheck_registrations(tops):
    """torch.library.opcheck: schema (no hidden mutation or aliasing), autograd registration and
    the fake kernels against the real outputs, one sample per op."""
    checks = ("test_schema", "test_autograd_registration", "test_faketensor")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(1, 6, 6, 6, 8, generator=g).cuda().requires_grad_()
    w = (torch.randn(16, 8, 3, 3, 3, generator=g) * 0.1).cuda().requires_grad_()
    torch.library.opcheck(torch.ops.mragan.conv3d.default, (x, w, None, 2, 1, 0, False, "relu"), test_utils=checks)
    torch.library.opcheck(torch.ops.mragan.instance_norm.default, (x, "lrelu", 1), test_utils=checks)
    torch.library.opcheck(torch.ops.mragan.replication_pad.default, (x, 2), test_utils=checks)
    b = torch.randn(x.shape, generator=g).cuda()
    torch.library.opcheck(torch.ops.mragan.l1_loss.default, (x, b), test_utils=checks)


def test_argument_refusals(tops):
    """Wrong dtype, device or size is refused before any kernel sees the pointer."""
    x = torch.randn(1, 6, 6, 6, 8, device="cuda")
    w = torch.randn(16, 8, 3, 3, 3, device="cuda") * 0.1
    conv = torch.ops.mragan.conv3d
    for bad_w in (w.bfloat16(), w.half(), w.double(), w.cpu()):
        with pytest.raises(ValueError):
            conv(x, bad_w, None, 1, 1, 0, False, "none")
    for bad_b in (torch.zeros(15, device="cuda"), torch.zeros(16), torch.zeros(16, device="cuda", dtype=torch.float16)):
        with pytest.raises(ValueError):
            conv(x, w, bad_b, 1, 1, 0, False, "none")
    a = torch.randn(64, device="cuda")
    for bad in (a.half(), a.bfloat16(), a.double()):
        with pytest.raises(ValueError):
            torch.ops.mragan.l1_loss(bad, bad)
        with pytest.raises(ValueError):
            torch.ops.mragan.gan_loss(bad, 1.0, False)
    with pytest.raises(ValueError):
        torch.ops.mragan.l1_loss(a, a.cpu())
