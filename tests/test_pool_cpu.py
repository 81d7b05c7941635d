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


@pytest.mark.parametrize("pool_size", [0, 1, 3, 5])
def test_device_pool_changing_batch_size(pool_size):
    """The last DataLoader batch of an epoch is smaller (train.py:52 has no drop_last): the pool
    must keep its images across batch-size changes, in both directions."""
    from models.cycle_gan_model import DeviceImagePool
    g = torch.Generator().manual_seed(8)
    ref = ImagePool(pool_size, random.Random(12))
    random.seed(12)
    dev = DeviceImagePool(pool_size)
    for q, b in enumerate([2, 2, 1, 3, 2, 1, 1, 4, 2, 3, 1, 2] * 3):
        fakes = torch.randn(b, 3, 2, 2, 1, generator=g)
        want = ref.query(fakes.clone())
        ret, store = dev.plan(b)
        out = torch.empty_like(fakes)
        dev.apply(fakes, out, torch.tensor(ret), torch.tensor(store))
        assert torch.equal(out, want), f"query {q} (b={b})"
        for k in range(min(pool_size, dev.num_imgs)):
            assert torch.equal(dev.buf[k], ref.images[k][0]), f"slot {k} after query {q}"


def test_query_returns_tensor_like_reference():
    """ImagePool.query / DeviceImagePool.query return ONE tensor (reference torch.cat, :34)."""
    from models.cycle_gan_model import DeviceImagePool
    from models.cycle_gan_model import ImagePool as EngineImagePool
    g = torch.Generator().manual_seed(9)
    ref = ImagePool(2, random.Random(13))
    random.seed(13)
    eng = EngineImagePool(2)
    for q in range(12):
        x = torch.randn(2, 1, 3, 4, 5, generator=g)
        want = ref.query(x.clone())
        got = eng.query(x.clone())
        assert isinstance(got, torch.Tensor) and torch.equal(got, want), q
    random.seed(14)
    ref = ImagePool(2, random.Random(14))
    dev = DeviceImagePool(2)
    for q in range(12):
        x = torch.randn(2, 1, 3, 4, 5, generator=g)
        want = ref.query(x.clone())
        got = dev.query(x.clone())
        assert isinstance(got, torch.Tensor) and got.shape == want.shape and torch.equal(got, want), q


def _pool_seq():
    import os
    import numpy as np
    from golden_util import GOLDEN
    return np.load(os.path.join(GOLDEN, "pool_seq_p2.npz"), allow_pickle=False)


def _replay(pool_query, z):
    """Feed the fixture's batches (images carrying their running id) through `pool_query` after
    seeding the global `random` like the reference run; returns the ids it hands back."""
    random.seed(int(z["seed"]))
    got, nid = [], 0
    for b in z["sizes"]:
        b = int(b)
        imgs = torch.arange(nid, nid + b, dtype=torch.float32).view(b, 1, 1, 1, 1).expand(b, 1, 2, 2, 2).contiguous()
        nid += b
        out = pool_query(imgs)
        got.extend(int(v) for v in out[:, 0, 0, 0, 0])
    return got


def test_pool_sequence_pinned_to_reference():
    """48 queries of batch 1/2/3 through the REFERENCE's ImagePool(2) (tools/gen_fixtures.py
    pool_seq_p2, seeded `random`): the oracle's ImagePool and the engine's host ImagePool and
    DeviceImagePool return the same images (swaps included) in the same order."""
    from models.cycle_gan_model import DeviceImagePool
    from models.cycle_gan_model import ImagePool as EngineImagePool
    z = _pool_seq()
    want = [int(v) for v in z["ids"]]
    assert sum(w != i for i, w in enumerate(want)) > 20          # the sequence exercises the swap path
    P = int(z["pool_size"])
    orc = ImagePool(P)                                            # global `random`, like the reference
    assert _replay(orc.query, z) == want
    assert _replay(EngineImagePool(P).query, z) == want
    assert _replay(DeviceImagePool(P).query, z) == want
