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
    # BASELINE-size workloads (the per-GPU unit of each config), default widths ngf = ndf = 32.
    # "fp64pE" = an fp64 run at inputs perturbed by a relative E (N(0,1) noise, generator seed 77):
    # how far the exact gradient moves when the forward pass moves by that much (test gate)
    "step_r9_s64_b2": (["--netG", "resnet_9blocks"], 64, 2, 1, ["fp32", "fp64", "fp64p4e-6", "fp64p4e-5"], 2, 4),
    "step_unet_s64_b1_ngf32": (["--netG", "unet_custom"], 64, 1, 1, ["fp32", "fp64", "fp64p4e-6", "fp64p4e-5"], 2, 5),
    "step_r9_s96_b1_nc2": (["--netG", "resnet_9blocks", "--input_nc", "2", "--output_nc", "2"], 96, 1, 2,
                           ["fp32", "fp64", "fp64p4e-6", "fp64p4e-5"], 1, 6),
    "step_r9_s128_b1": (["--netG", "resnet_9blocks"], 128, 1, 1, ["fp32", "fp64", "fp64p4e-6", "fp64p4e-5"], 1, 7),
    # lambda_identity = 0: no identity passes (reference cycle_gan_model.py:174-194 else branch);
    # the running statistics then see only the four cycle passes
    "step_r6_s24_b1_noidt": (["--netG", "resnet_6blocks", "--ngf", "8", "--ndf", "8", "--lambda_identity", "0"],
                             24, 1, 1, ["fp32", "fp64"], 2, 9),
    # ImagePool of one image (cycle_gan_model.py:8-35): from the second step on every D query
    # draws random.uniform and, half the time, swaps the stored fake — the step itself takes the
    # swap path (the pool-50 cases never leave the pass-through phase)
    "step_r6_s24_b1_pool1": (["--netG", "resnet_6blocks", "--ngf", "4", "--ndf", "4", "--pool_size", "1"],
                             24, 1, 1, ["fp32", "fp64"], 6, 11),
    # UnetGenerator with 8 downsamplings (--netG unet_256, BASELINE configs[3]'s generator): it
    # trains only from 256³ (a 1³ bottleneck InstanceNorm raises below), so at 256³
    # with narrow widths
    "step_unet256_s256_b1_ngf4": (["--netG", "unet_256", "--ngf", "4", "--ndf", "4"], 256, 1, 1,
                                  ["fp32", "fp64", "fp64p4e-6", "fp64p4e-5"], 1, 12),
}
# reference-written checkpoint (base_model.py:89-112) of a tiny model after one step, plus the
# losses of the step the reference takes right after it (ckpt_* cases, see run_checkpoint)
CKPT_CASES = {
    "ckpt_r6_ngf4": (["--netG", "resnet_6blocks", "--ngf", "4", "--ndf", "4"], 24, 1, 1, 8),
}
N_SAMPLES = 256
DTYPE_PREFIXES = ("fp32", "fp64", "fp64p4e-6", "fp64p4e-5", "fp64p4e-6r1", "fp64p4e-6r2", "fp64p4e-6r3")
# further realisations of the exact-f32 mode's input perturbation for the BASELINE-size cases
# (generator seeds 78, 79; the stored fp64p4e-6 run is seed 77): the per-tensor gradient envelope is the max over realisations, as
# the small cases compute two at test time (tests/test_step_gpu.py `conditioning`)
EXTRA_REALISATIONS = ("fp64p4e-6r1", "fp64p4e-6r2")
BASELINE_SIZE = ("step_r9_s64_b2", "step_unet_s64_b1_ngf32", "step_r9_s96_b1_nc2", "step_r9_s128_b1",
                 "step_unet256_s256_b1_ngf4")


COL_LIMIT = 2 << 30      # bytes of one im2col buffer of an fp64 CPU convolution


def _chunked_conv3d(orig):
    """fp64 Conv3d on the CPU is ATen's slow_conv3d, whose im2col buffer is (Cin·k³) × (output
    voxels) elements: 78 GB for the 32→2 head conv at 96³, 184 GB at 128³.  For such calls the
    output depth is cut into slabs (zero padding applied once up front, each slab convolved
    'valid' on its input rows, results concatenated): every output element is the same sum over
    the same products, only the GEMM's blocking changes.  fp32 calls (mkldnn) are untouched."""
    import torch.nn.functional as F

    def conv3d(input, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
        def t3(v):
            return tuple(v) if isinstance(v, (tuple, list)) else (v, v, v)
        st, pd, dl = t3(stride), t3(padding), t3(dilation)
        if isinstance(padding, str) or input.dtype != torch.float64 or groups != 1 or dl != (1, 1, 1):
            return orig(input, weight, bias, stride, padding, dilation, groups)
        k = weight.shape[2:]
        x = F.pad(input, (pd[2], pd[2], pd[1], pd[1], pd[0], pd[0])) if any(pd) else input
        Do = (x.shape[2] - k[0]) // st[0] + 1
        Ho = (x.shape[3] - k[1]) // st[1] + 1
        Wo = (x.shape[4] - k[2]) // st[2] + 1
        per_row = weight.shape[1] * k[0] * k[1] * k[2] * Ho * Wo * 8
        rows = max(1, COL_LIMIT // per_row)
        if rows >= Do:
            return orig(input, weight, bias, stride, padding, dilation, groups)
        outs = []
        for o0 in range(0, Do, rows):
            o1 = min(Do, o0 + rows)
            xs = x[:, :, o0 * st[0]:(o1 - 1) * st[0] + k[0]]
            outs.append(orig(xs, weight, bias, st, 0, 1, 1))
        return torch.cat(outs, 2)
    return conv3d


def import_reference():
    import torch.nn.functional as F
    if not getattr(F.conv3d, "_chunked", False):
        F.conv3d = _chunked_conv3d(F.conv3d)
        F.conv3d._chunked = True
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
    name = key.split("/", 1)[1] if key.split("/", 1)[0] in DTYPE_PREFIXES else key
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    idx = np.sort(rng.choice(flat.numel(), size=min(n, flat.numel()), replace=False))
    out[key + "/idx"] = idx.astype(np.int64)
    out[key + "/val"] = flat[torch.from_numpy(idx)].numpy()
    out[key + "/sum"] = np.array(flat.sum().item())
    out[key + "/abssum"] = np.array(flat.abs().sum().item())
    out[key + "/sqsum"] = np.array((flat * flat).sum().item())


def perturb(x, eps, g):
    return x * (1 + eps * torch.randn(x.shape, generator=g, dtype=torch.float64))


def _eps_seed(dt):
    """fp64p<E>[r<i>]: relative perturbation E, noise generator seed 77 + i."""
    if not dt.startswith("fp64p"):
        return 0.0, 77
    body = dt[len("fp64p"):]
    e, _, r = body.partition("r")
    return float(e), 77 + (int(r) if r else 0)


def run_case(name, argv, S, B, nc, dtypes, steps, seed, out=None):
    TrainOptions, create_model = import_reference()
    import gc
    import random
    first = out is None
    out = {} if out is None else out
    for dt in dtypes:
        eps, pseed = _eps_seed(dt)
        gc.collect()
        sys.argv = ["train.py", "--checkpoints_dir", "/tmp/gen_fixtures_ck"] + argv
        opt = TrainOptions().gather_options()
        opt.isTrain = True
        opt.gpu_ids = 0
        torch.manual_seed(seed)
        random.seed(seed)
        model = create_model(opt)
        model.setup(opt)
        if dt.startswith("fp64"):
            for n in ("G_A", "G_B", "D_A", "D_B"):
                getattr(model, "net" + n).double()
            model.criterionGAN.double()
        pre = f"{dt}"
        if first and dt == dtypes[0]:
            for n in ("G_A", "G_B", "D_A", "D_B"):
                for k, v in getattr(model, "net" + n).state_dict().items():
                    if v.is_floating_point() and k.endswith("weight"):
                        sample(v, f"init/{n}/{k}", out, n=32)
        shape = (B, nc, S, S, S)
        for step in range(steps if not eps else 1):
            A, Bt = synthetic_pair(shape, 1000 + seed + step)
            if dt.startswith("fp64"):
                A, Bt = A.double(), Bt.double()
            if eps:
                g = torch.Generator().manual_seed(pseed)
                A, Bt = perturb(A, eps, g), perturb(Bt, eps, g)
            model.set_input([A, Bt])
            model.optimize_parameters()
            losses = model.get_current_losses()
            out[f"{pre}/step{step}/losses"] = np.array([losses[k] for k in model.loss_names], dtype=np.float64)
            if eps:
                for n in ("G_A", "G_B", "D_A", "D_B"):
                    for k, p in getattr(model, "net" + n).named_parameters():
                        sample(p.grad, f"{pre}/step0/grad/{n}/{k}", out, n=64)
                continue
            if step == 0:
                for vis in ("fake_B", "rec_A", "fake_A", "rec_B", "idt_A", "idt_B"):
                    if not hasattr(model, vis):      # lambda_identity = 0: no identity passes
                        continue
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
        del model
        print(f"  {name}: {dt} done", flush=True)
    meta = dict(argv=" ".join(argv), S=S, B=B, nc=nc, steps=steps, seed=seed, torch=torch.__version__)
    out["meta"] = np.array(repr(meta))
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def run_checkpoint(name, argv, S, B, nc, seed):
    """One reference step, save_networks('1') into tests/golden/<name>/, then record the losses of
    the next step (inputs seed 1000+seed+1) and the saved state_dicts' key / shape / dtype table."""
    import json
    import random
    TrainOptions, create_model = import_reference()
    ck = os.path.abspath(OUT)
    sys.argv = ["train.py", "--checkpoints_dir", ck, "--name", name] + argv
    opt = TrainOptions().gather_options()
    opt.isTrain = True
    opt.gpu_ids = 0
    torch.manual_seed(seed)
    random.seed(seed)
    model = create_model(opt)
    model.setup(opt)
    os.makedirs(os.path.join(ck, name), exist_ok=True)
    shape = (B, nc, S, S, S)
    model.set_input(list(synthetic_pair(shape, 1000 + seed)))
    model.optimize_parameters()
    model.save_networks("1")
    table = {}
    for n in ("G_A", "G_B", "D_A", "D_B"):
        sd = torch.load(os.path.join(ck, name, "1_net_%s.pth" % n), map_location="cpu", weights_only=True)
        table[n] = [[k, list(v.shape), str(v.dtype)] for k, v in sd.items()]
    model.set_input(list(synthetic_pair(shape, 1000 + seed + 1)))
    model.optimize_parameters()
    losses = model.get_current_losses()
    meta = dict(argv=" ".join(argv), S=S, B=B, nc=nc, seed=seed, torch=torch.__version__,
                next_losses=[losses[k] for k in model.loss_names], loss_names=list(model.loss_names), keys=table)
    with open(os.path.join(ck, name, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    opt_txt = os.path.join(ck, name, "train_opt.txt")
    if os.path.exists(opt_txt):
        os.remove(opt_txt)
    print("wrote", os.path.join(ck, name))


def run_pool_sequence(name="pool_seq_p2", pool_size=2, seed=123, queries=48):
    """The reference's ImagePool(pool_size) on a sequence of batches (sizes 1, 2, 3 cycling) whose
    images carry their running id: stores the ids it returns, per query, in order."""
    import random
    import itertools
    sys.modules["monai"] = types.ModuleType("monai")
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from models.cycle_gan_model import ImagePool     # noqa: E402  (the reference's)
    random.seed(seed)
    pool = ImagePool(pool_size)
    sizes, ids, nid = [], [], 0
    for q, b in zip(range(queries), itertools.cycle((1, 2, 3))):
        imgs = torch.arange(nid, nid + b, dtype=torch.float32).view(b, 1, 1, 1, 1).expand(b, 1, 2, 2, 2).contiguous()
        nid += b
        out = pool.query(imgs)
        sizes.append(b)
        ids.extend(int(v) for v in out[:, 0, 0, 0, 0])
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, sizes=np.array(sizes), ids=np.array(ids), pool_size=np.array(pool_size),
                        seed=np.array(seed))
    print("wrote", path, "returned ids differ from inputs at", int((np.array(ids) != np.arange(len(ids))).sum()),
          "of", len(ids))


def add_realisations(name):
    """Append the EXTRA_REALISATIONS runs to an existing fixture (the stored runs are kept as
    they are; the new ones sample the same indices)."""
    argv, S, B, nc, _, steps, seed = CASES[name]
    path = os.path.join(OUT, name + ".npz")
    with np.load(path, allow_pickle=False) as z:
        out = {k: z[k] for k in z.files}
    todo = [dt for dt in EXTRA_REALISATIONS if f"{dt}/loss_names" not in out]
    if todo:
        run_case(name, argv, S, B, nc, todo, steps, seed, out=out)


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(os.cpu_count())
    if sys.argv[1:2] == ["--realisations"]:
        for name in sys.argv[2:] or BASELINE_SIZE:
            add_realisations(name)
        return
    which = sys.argv[1:] or list(CASES) + list(CKPT_CASES) + ["pool_seq_p2"]
    for name in which:
        if name == "pool_seq_p2":
            run_pool_sequence()
            continue
        if name in CKPT_CASES:
            run_checkpoint(name, *CKPT_CASES[name])
            continue
        argv, S, B, nc, dtypes, steps, seed = CASES[name]
        run_case(name, argv, S, B, nc, dtypes, steps, seed)


if __name__ == "__main__":
    main()
