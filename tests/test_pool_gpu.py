"""DeviceImagePool on the device against the reference's own ImagePool (tools/gen_fixtures.py
pool_seq_p2: 48 seeded queries through the reference's ImagePool(2), swaps included)."""
import pytest
import torch

from test_pool_cpu import _pool_seq, _replay

pytestmark = pytest.mark.gpu


def test_device_pool_on_gpu_pinned_to_reference():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from models.cycle_gan_model import DeviceImagePool
    z = _pool_seq()
    pool = DeviceImagePool(int(z["pool_size"]))
    got = _replay(lambda imgs: pool.query(imgs.cuda()).cpu(), z)
    assert got == [int(v) for v in z["ids"]]
    assert pool.buf.is_cuda
