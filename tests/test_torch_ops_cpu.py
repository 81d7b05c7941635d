"""torch.ops.mragan.* registration (mragan_hip/torch_ops.py) without a GPU: the ops exist, their
fake kernels propagate NDHWC shapes, and a CPU tensor is refused (no CPU kernel: the HIP
library is the only compute path)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import mragan_hip.torch_ops as tops


def test_ops_registered():
    for name in tops.OPS:
        assert hasattr(torch.ops.mragan, name), name


@pytest.mark.parametrize("transposed,k,s,p,op,shape,cin,cout,expect", [
    (False, 7, 1, 0, 0, (2, 70, 70, 70), 1, 32, (64, 64, 64)),     # G stem on the RPad3 input
    (False, 3, 2, 1, 0, (2, 64, 64, 64), 32, 64, (32, 32, 32)),    # G down
    (True, 3, 2, 1, 1, (2, 16, 16, 16), 128, 64, (32, 32, 32)),    # G up (ConvTranspose3d)
    (False, 4, 2, 1, 0, (1, 64, 64, 64), 1, 64, (32, 32, 32)),     # D first layer
])
def test_conv3d_fake_shapes(transposed, k, s, p, op, shape, cin, cout, expect):
    with FakeTensorMode():
        x = torch.empty(shape + (cin,))
        w = torch.empty((cin, cout, k, k, k) if transposed else (cout, cin, k, k, k))
        y = torch.ops.mragan.conv3d(x, w, None, s, p, op, transposed, "none")
    assert tuple(y.shape) == (shape[0],) + expect + (cout,)


def test_instance_norm_and_pad_fake_shapes():
    with FakeTensorMode():
        x = torch.empty(2, 16, 16, 16, 128)
        y, mean, rstd = torch.ops.mragan.instance_norm(x, "relu", 1)
        z = torch.ops.mragan.replication_pad(x, 3)
    assert tuple(y.shape) == (2, 18, 18, 18, 128)
    assert tuple(mean.shape) == tuple(rstd.shape) == (2, 128)
    assert tuple(z.shape) == (2, 22, 22, 22, 128)


def test_loss_and_adam_fake():
    with FakeTensorMode():
        a = torch.empty(2, 8, 8, 8, 1)
        assert torch.ops.mragan.l1_loss(a, a).shape == ()
        assert torch.ops.mragan.gan_loss(a, 1.0, True).shape == ()
        p = torch.empty(10)
        assert torch.ops.mragan.adam_(p, p, p, p, 1e-3, 0.5, 0.999, 1e-8, 1, 1.0) is None


def test_geometry_errors():
    with FakeTensorMode():
        x = torch.empty(1, 8, 8, 8, 4)
        with pytest.raises(ValueError):
            torch.ops.mragan.conv3d(x, torch.empty(8, 5, 3, 3, 3), None, 1, 1, 0, False, "none")
        with pytest.raises(ValueError):
            torch.ops.mragan.conv3d(x, torch.empty(8, 4, 3, 3, 3), None, 1, 1, 1, False, "none")


def test_cpu_tensor_refused():
    x = torch.zeros(1, 4, 4, 4, 2)
    with pytest.raises(Exception):
        torch.ops.mragan.replication_pad(x, 1)


def test_argument_guard():
    """_need_f32 is the guard every op runs before handing raw pointers to a kernel."""
    cpu = torch.device("cpu")
    tops._need_f32(None, "t", cpu)
    tops._need_f32(torch.zeros(3), "t", cpu, 3)
    for bad, numel in ((torch.zeros(3, dtype=torch.bfloat16), None), (torch.zeros(3, dtype=torch.float64), None),
                       (torch.zeros(3, device="meta"), None), (torch.zeros(4), 3)):
        with pytest.raises(ValueError):
            tops._need_f32(bad, "t", cpu, numel)
