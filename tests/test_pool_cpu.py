"""DeviceImagePool (the fused step's image history, models/cycle_gan_model.py) against the
oracle's restatement of the reference ImagePool (cycle_gan_model.py:8-35): same draws from the
global `random` stream, same returned images, same pool contents — incl. two swaps into the
same slot within one batch and pool_size 0.  Runs on CPU tensors (the plan/apply logic is the
same on the device)."""
import random

import pytest
import torch

from oracle.cyclegan_oracle import ImagePool


@pytest.mark.parametrize("pool_size,b,queries", [(3, 2, 40), (1, 4, 20), (0, 2, 3), (5, 1, 30), (2, 3, 40)])
def test_device_pool_matches_reference(pool_size, b, queries):
    from models.cycle_gan_model import DeviceImagePool
    g = torch.Generator().manual_seed(7)
    ref = ImagePool(pool_size, random.Random(11))
    random.seed(11)
    dev = DeviceImagePool(pool_size)
    for q in range(queries):
        fakes = torch.randn(b, 3, 2, 2, 1, generator=g)
        want = ref.query(fakes.clone())
        ret, store = dev.plan(b)
        out = torch.empty_like(fakes)
        dev.apply(fakes, out, torch.tensor(ret), torch.tensor(store))
        assert torch.equal(out, want), f"query {q}"
        for k in range(min(pool_size, dev.num_imgs)):
            assert torch.equal(dev.buf[k], ref.images[k][0]), f"slot {k} after query {q}"
