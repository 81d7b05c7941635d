#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE (pedrob37/MRA-GAN) itself.

Runs only in the build container, where /root/reference exists.  It imports the
reference's models/ and options/ packages (a stub `monai` module is placed in
sys.modules — monai is only used by networks3D.Dynet, out of scope), builds the
CycleGANModel through the reference's own TrainOptions/create_model, and runs
`optimize_parameters()` on seeded synthetic patches.

Only data is written (tests/golden/*.npz): inputs are regenerated from their seed
by the tests; outputs, losses, gradient norms/samples and post-step parameter
samples are stored.  No reference source is copied.

Usage:  python tools/gen_fixtures.py            (≈1 min on 8 cores)
"""
import os
import sys
import types
import zlib

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

CASES = {
    # name: (argv, patch S, batch, dtype list, steps, seed)
    "step_r9_s32_b1": (["--netG", "resnet_9blocks"], 32, 1, 1, ["fp32", "fp64"], 2, 0),
    "step_r6_s24_b2_nc2_lsgan": (["--netG", "resnet_6blocks", "--input_nc", "2", "--output_nc", "2",
                                  "--ngf", "8", "--ndf", "8", "--no_lsgan"], 24, 2, 2, ["fp32", "fp64"], 2, 1),
    "step_r9_s32_b2_ngf16": (["--netG", "resnet_9blocks", "--ngf", "16", "--ndf", "16"], 32, 2, 1,
                             ["fp32", "fp64"], 3, 2),
    # UnetGenerator (BASELINE configs[3] generator family; unet_custom = 5 downsamplings)
    "step_unet_s32_b2_ngf8": (["--netG", "unet_custom", "--ngf", "8", "--ndf", "8"], 32, 2, 1, ["fp32", "fp64"], 2, 3),
}
N_SAMPLES = 256


def import_reference():
    sys.modules["monai"] = types.ModuleType("monai")
    sys.path.insert(0, REF)
    from options.train_options import TrainOptions   # noqa: E402
    from models import create_model                  # noqa: E402
    return TrainOptions, create_model


def synthetic_pair(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g), torch.randn(shape, generator=g)


def sample(t: torch.Tensor, key: str, out: dict, n=N_SAMPLES):
    flat = t.detach().reshape(-1).double()
    # the sample positions depend on the tensor's name only (not on the fp32/fp64 prefix), so
    # the fp32 and fp64 runs are sampled at identical indices and can be compared directly
    name = key.split("/", 1)[1] if key.startswith(("fp32/", "fp64/")) else key
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    idx = np.sort(rng.choice(flat.numel(), size=min(n, flat.numel()), replace=False))
    out[key + "/idx"] = idx.astype(np.int64)
    out[key + "/val"] = flat[torch.from_numpy(idx)].numpy()
    out[key + "/sum"] = np.array(flat.sum().item())
    out[key + "/abssum"] = np.array(flat.abs().sum().item())
    out[key + "/sqsum"] = np.array((flat * flat).sum().item())


def run_case(name, argv, S, B, nc, dtypes, steps, seed):
    TrainOptions, create_model = import_reference()
    import random
    out = {}
    for dt in dtypes:
        sys.argv = ["train.py", "--checkpoints_dir", "/tmp/gen_fixtures_ck"] + argv
        opt = TrainOptions().gather_options()
        opt.isTrain = True
        opt.gpu_ids = 0
        torch.manual_seed(seed)
        random.seed(seed)
        model = create_model(opt)
        model.setup(opt)
        if dt == "fp64":
            for n in ("G_A", "G_B", "D_A", "D_B"):
                getattr(model, "net" + n).double()
            model.criterionGAN.double()
        pre = f"{dt}"
        if dt == dtypes[0]:
            for n in ("G_A", "G_B", "D_A", "D_B"):
                for k, v in getattr(model, "net" + n).state_dict().items():
                    if v.is_floating_point() and k.endswith("weight"):
                        sample(v, f"init/{n}/{k}", out, n=32)
        shape = (B, nc, S, S, S)
        for step in range(steps):
            A, Bt = synthetic_pair(shape, 1000 + seed + step)
            if dt == "fp64":
                A, Bt = A.double(), Bt.double()
            model.set_input([A, Bt])
            model.optimize_parameters()
            losses = model.get_current_losses()
            out[f"{pre}/step{step}/losses"] = np.array([losses[k] for k in model.loss_names], dtype=np.float64)
            if step == 0:
                for vis in ("fake_B", "rec_A", "fake_A", "rec_B", "idt_A", "idt_B"):
                    sample(getattr(model, vis), f"{pre}/step0/{vis}", out)
                for n in ("G_A", "G_B", "D_A", "D_B"):
                    net = getattr(model, "net" + n)
                    for k, p in net.named_parameters():
                        g = p.grad
                        out[f"{pre}/step0/grad/{n}/{k}/norm"] = np.array(g.double().norm().item())
                        sample(g, f"{pre}/step0/grad/{n}/{k}", out, n=64)
                        sample(p.detach(), f"{pre}/step0/param/{n}/{k}", out, n=64)
                    for k, b in net.state_dict().items():
                        if "running" in k:
                            sample(b, f"{pre}/step0/buf/{n}/{k}", out, n=16)
        out[f"{pre}/loss_names"] = np.array(model.loss_names)
    meta = dict(argv=" ".join(argv), S=S, B=B, nc=nc, steps=steps, seed=seed, torch=torch.__version__)
    out["meta"] = np.array(repr(meta))
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(os.cpu_count())
    which = sys.argv[1:] or list(CASES)
    for name in which:
        argv, S, B, nc, dtypes, steps, seed = CASES[name]
        run_case(name, argv, S, B, nc, dtypes, steps, seed)


if __name__ == "__main__":
    main()
