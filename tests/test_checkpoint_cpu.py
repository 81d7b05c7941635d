"""Checkpoint interop with the reference (base_model.py:89-148), CPU side.

tests/golden/ckpt_r6_ngf4/ holds the four files the REFERENCE's save_networks('1') wrote after one
training step (tools/gen_fixtures.py run_checkpoint), plus meta.json with the key / shape / dtype
table of each.  Checked here:
  * the engine's save_networks writes the same file names and the same key / shape / dtype
    table (117-style ResnetGenerator keys, InstanceNorm buffers included);
  * the engine's load_networks reads the reference's files (weights_only torch.load) and ends up
    holding exactly their values;
  * InstanceNorm's num_batches_tracked is 0 in the reference's files: torch's InstanceNorm never
    increments it, so the engine leaving it at 0 is the reference behaviour."""
import json
import os
import random
import sys

import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAME = "ckpt_r6_ngf4"


def _meta():
    with open(os.path.join(GOLD, NAME, "meta.json")) as fh:
        return json.load(fh)


def build(ckdir, name, extra=()):
    from models import create_model
    from options.train_options import TrainOptions
    meta = _meta()
    argv = sys.argv
    try:
        sys.argv = ["train.py", "--checkpoints_dir", str(ckdir), "--name", name] + meta["argv"].split() + list(extra)
        opt = TrainOptions().gather_options()
    finally:
        sys.argv = argv
    opt.isTrain, opt.gpu_ids = True, 0
    torch.manual_seed(meta["seed"])
    random.seed(meta["seed"])
    model = create_model(opt)
    model.setup(opt)
    return model


def test_saved_key_table_matches_reference(tmp_path):
    meta = _meta()
    model = build(tmp_path, "eng")
    model.save_networks("1")
    for net, table in meta["keys"].items():
        path = os.path.join(tmp_path, "eng", "1_net_%s.pth" % net)
        sd = torch.load(path, map_location="cpu", weights_only=True)
        ours = [[k, list(v.shape), str(v.dtype)] for k, v in sd.items()]
        assert ours == table, net


def test_reference_checkpoint_loads(tmp_path):
    meta = _meta()
    model = build(GOLD, NAME, ["--continue_train", "--which_epoch", "1"])
    for net in meta["keys"]:
        ref = torch.load(os.path.join(GOLD, NAME, "1_net_%s.pth" % net), map_location="cpu", weights_only=True)
        ours = getattr(model, "net" + net).state_dict()
        for k, v in ref.items():
            if k.endswith("num_batches_tracked"):
                assert int(v) == 0, (net, k)      # InstanceNorm never counts
                continue
            assert torch.equal(ours[k].cpu(), v), (net, k)
