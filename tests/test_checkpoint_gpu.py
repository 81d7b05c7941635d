"""Resume from a REFERENCE-written checkpoint on the device (base_model.py:130-148 then
cycle_gan_model.py:227-240): load tests/golden/ckpt_r6_ngf4/1_net_*.pth through the engine's
load_networks (--continue_train --which_epoch 1) and take the step the reference took right after
saving them; its 8 losses must match the reference's (fp32 CPU) within the north star's value gate.
(The reference's image pool held one image per pool, but with pool_size 50 the second query is
still a pass-through, and the losses are computed before the Adam step, so neither the pool nor
the unsaved optimizer state enters these numbers.)"""
import numpy as np
import pytest
import torch

from test_checkpoint_cpu import GOLD, NAME, _meta, build

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_resume_from_reference_checkpoint(precision):
    from mragan_hip import ops
    from oracle.cyclegan_oracle import synthetic_pair
    meta = _meta()
    try:
        model = build(GOLD, NAME, ["--continue_train", "--which_epoch", "1", "--conv_precision", precision])
        shape = (meta["B"], meta["nc"], meta["S"], meta["S"], meta["S"])
        model.set_input(list(synthetic_pair(shape, 1000 + meta["seed"] + 1)))
        model.optimize_parameters()
        got = np.array(list(model.get_current_losses().values()))
    finally:
        ops.set_conv_precision("f32")
    want = np.array(meta["next_losses"])
    rel = float(np.linalg.norm(got - want) / np.linalg.norm(want))
    assert rel < {"f32": 1e-4, "bf16x3": 1e-3}[precision], (got, want)
