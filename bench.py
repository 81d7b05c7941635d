#!/usr/bin/env python3
"""Benchmark: 3D patches/sec of one full CycleGAN optimize_parameters() step
(G_A, G_B, D_A, D_B forward + backward + both Adam steps), BASELINE.json's metric.

Workload (N=1): BASELINE configs[1] — ResNet-9blocks G + 3-layer PatchGAN D, 1ch→1ch,
64³ patch, batch 2 per GPU, synthetic N(0,1) volumes, random init (seed 0).  Multi-GPU:
one process per GPU (torch.distributed over RCCL), each rank its own batch (weak scaling),
gradients all-reduced inside the step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 64] [--batch 2]

Prints ONE JSON line on rank 0 (contract in the task description), with:
  roofline     — the dominant kernel (res-block 3×3×3 conv, LDS-halo implicit GEMM): algorithmic
                 FLOP per launch ÷ its mean launch duration, timed with HIP events around every
                 such launch inside the timed region;
  cpu_baseline — the CPU oracle (oracle/cyclegan_oracle.py, the reference's algorithm restated
                 in PyTorch-CPU) timed on this host for one step of the same workload.
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "mra-gan_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

MFMA_F32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 matrix/vector peak
MFMA_BF16_PEAK_TFLOPS = 2516.6   # 16 × the f32 MFMA rate (dense bf16, no sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--ngf", type=int, default=32)
    ap.add_argument("--netG", default="resnet_9blocks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", default="bf16x3", choices=["f32", "bf16x3"],
                    help="dense-conv contraction: exact f32 MFMA or split-bf16 (bf16x3) MFMA, fp32 accumulate")
    ap.add_argument("--cpu-steps", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true",
                    help="launch the step's kernels from Python every step (default: replay the step as HIP graphs)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on the node; gloo only for rehearsal")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0 (use with --dist-backend gloo)")
    return ap.parse_args()


def g_layer_flops(netG, S, ngf=32, nc=1):
    """Forward conv FLOPs (2 × MAC) of each generator layer, stem first.  Transposed convs are
    priced on their input voxels (every input scatters k³ taps), like torch's flop counter."""
    def conv(cin, cout, k, vox):
        return 2.0 * cin * cout * k ** 3 * vox
    if netG.startswith("unet"):
        nd = 5 if netG == "unet_custom" else 8
        chans = [(nc, ngf, nc), (ngf, 2 * ngf, ngf), (2 * ngf, 4 * ngf, 2 * ngf), (4 * ngf, 8 * ngf, 4 * ngf)]
        chans += [(8 * ngf, 8 * ngf, 8 * ngf)] * (nd - 4)        # middle blocks + innermost
        downs, ups = [], []
        for L, (outer, inner, cin) in enumerate(chans):
            vox = (S >> (L + 1)) ** 3                           # down output = up input voxels
            downs.append(conv(cin, inner, 4, vox))
            ups.append(conv(inner if L == len(chans) - 1 else 2 * inner, outer, 4, vox))
        return downs + ups[::-1]
    n_blocks = 9 if netG == "resnet_9blocks" else 6
    s4 = (S // 4) ** 3
    g_layers = [conv(nc, ngf, 7, S ** 3), conv(ngf, 2 * ngf, 3, (S // 2) ** 3), conv(2 * ngf, 4 * ngf, 3, s4)]
    g_layers += [conv(4 * ngf, 4 * ngf, 3, s4)] * (2 * n_blocks)
    g_layers += [conv(2 * ngf, 4 * ngf, 3, s4), conv(ngf, 2 * ngf, 3, (S // 2) ** 3), conv(ngf, nc, 7, S ** 3)]
    return g_layers


def step_flops(S, batch, ngf=32, netG="resnet_9blocks", ndf=32, nc=1):
    """Algorithmic conv FLOPs of one optimize_parameters() step (2 × MAC; forward, dgrad where
    the reference computes it, wgrad).  Matches SURVEY §0 (1.6045 TFLOP per 64³ resnet_9blocks
    patch)."""
    def conv(cin, cout, k, out_vox):
        return 2.0 * cin * cout * k ** 3 * out_vox
    g_layers = g_layer_flops(netG, S, ngf, nc)
    g_fwd = sum(g_layers)
    first_g = g_layers[0]
    d_sp = [S // 2, S // 4, S // 8, S // 8 - 1, S // 8 - 2]
    d_layers = [conv(nc, ndf, 4, d_sp[0] ** 3), conv(ndf, 2 * ndf, 4, d_sp[1] ** 3), conv(2 * ndf, 4 * ndf, 4, d_sp[2] ** 3),
                conv(4 * ndf, 8 * ndf, 4, d_sp[3] ** 3), conv(8 * ndf, 1, 4, d_sp[4] ** 3)]
    d_fwd = sum(d_layers)
    first_d = d_layers[0]
    # 6 G passes: fwd + wgrad + dgrad, minus input dgrad for the 4 passes fed real data
    g = 6 * (3 * g_fwd) - 4 * first_g
    # D: 2 frozen passes (fwd + dgrad incl. input), 4 trainable passes (fwd + wgrad + dgrad w/o input)
    d = 2 * (2 * d_fwd) + 4 * (3 * d_fwd - first_d)
    return batch * (g + d)


def host_threads():
    """CPU threads this job may use: the affinity mask, capped by OMP_NUM_THREADS when set
    (os.cpu_count() reports the whole machine on the GPU box, not this job's share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(args):
    """Oracle step on the host CPU (same workload shape), bounded to a couple of steps."""
    from oracle.cyclegan_oracle import CycleGANOracle, synthetic_pair
    torch.set_num_threads(host_threads())
    threads = torch.get_num_threads()
    torch.manual_seed(0)
    orc = CycleGANOracle(ngf=args.ngf, ndf=args.ngf, netG=args.netG, pool_rng=random.Random(0))
    shape = (args.batch, 1, args.size, args.size, args.size)
    times = []
    for i in range(args.cpu_steps):
        A, B = synthetic_pair(shape, 1000 + i)
        t0 = time.perf_counter()
        orc.optimize_parameters(A, B)
        times.append(time.perf_counter() - t0)
    t = min(times)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": args.batch / t, "unit": "patches/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} optimize_parameters() step(s) of the CPU oracle (PyTorch-CPU fp32) on "
                      f"{args.batch}x1x{args.size}^3, best {t:.2f} s, {cpu_model}"}


def cpu_baseline_child(args, timeout_s=240):
    """Run cpu_baseline() in a child process (the GPU process only waits), bounded in time."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--size", str(args.size),
           "--batch", str(args.batch), "--ngf", str(args.ngf), "--netG", args.netG, "--cpu-steps", str(args.cpu_steps)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
        for line in r.stdout.splitlines():
            if line.startswith("{"):
                return json.loads(line)
        return {"value": None, "unit": "patches/s", "cores": host_threads(), "kind": "port",
                "sample": f"CPU baseline child failed (rc {r.returncode}): {r.stderr[-300:]}"}
    except subprocess.TimeoutExpired:
        return {"value": None, "unit": "patches/s", "cores": host_threads(), "kind": "port",
                "sample": f"CPU oracle step exceeded {timeout_s} s on this host; not reported"}


def measured_traffic(key):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes
    (profiles/traffic.json, written by tools/pmc_traffic.py: (2·FETCH_SIZE + WRITE_SIZE)·1 KiB,
    the gfx950 correction); None when no pass was recorded for this configuration."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as fh:
            return json.load(fh)[key]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def main():
    args = parse()
    if args.cpu_baseline_only:
        print(json.dumps(cpu_baseline(args)), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dev = 0 if args.same_device else local
        torch.cuda.set_device(dev)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)

    from models import create_model
    from mragan_hip import ops
    from options.train_options import TrainOptions

    sys_argv = sys.argv
    sys.argv = ["train.py", "--netG", args.netG, "--ngf", str(args.ngf), "--ndf", str(args.ngf),
                "--checkpoints_dir", "/tmp/mragan_bench", "--batch_size", str(args.batch),
                "--conv_precision", args.precision] + (["--no_cuda_graph"] if args.no_graph else [])
    opt = TrainOptions().gather_options()
    sys.argv = sys_argv
    opt.isTrain, opt.gpu_ids = True, 0
    torch.manual_seed(0)
    random.seed(0)
    # the reference's network-init banner goes to stderr: stdout carries only the JSON line
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):
        model = create_model(opt)
        model.setup(opt)

    g = torch.Generator().manual_seed(1000 + rank)
    shape = (args.batch, 1, args.size, args.size, args.size)
    n_in = args.warmup + args.steps
    inputs = [(torch.randn(shape, generator=g).cuda(), torch.randn(shape, generator=g).cuda()) for _ in range(n_in)]

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # dominant kernel of the batched first G pass: resnet — residual-block conv 4ngf→4ngf k3
    # (forward form); unet — the level-1 upconv ConvTranspose3d(4ngf → ngf, k4 s2) (the largest
    # conv of the net).  Its launches are bracketed by HIP events: recorded eagerly in --no-graph
    # mode, recorded into the captured step graph otherwise (event nodes, re-recorded by every
    # replay, so after the timed region they hold the last timed step's launches).
    unet = args.netG.startswith("unet")
    c4 = 4 * args.ngf
    s4 = args.size // 4
    n_launch = 2 * args.batch
    if unet:
        match = lambda i: (i["cin"] == c4 and i["cout"] == args.ngf and i["k"] == 4 and i["transposed"]
                           and i["N"] == n_launch)
    else:
        match = lambda i: (i["cin"] == c4 and i["cout"] == c4 and i["k"] == 3 and i["s"] == 1 and
                           not i["transposed"] and i["N"] == n_launch)
    ops.TIMER.match = match
    for i in range(args.warmup):
        model.set_input(inputs[i])
        model.optimize_parameters()
    barrier()
    ops.TIMER.reset()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    start.record()
    for i in range(args.steps):
        model.set_input(inputs[args.warmup + i])
        model.optimize_parameters()
    end.record()
    barrier()
    wall = time.perf_counter() - t0
    ops.TIMER.match = None
    graphed = getattr(model, "_graphs", None) is not None
    elapsed = start.elapsed_time(end) / 1e3
    elapsed = max(elapsed, wall)
    if dist is not None:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    timing = "HIP events around each launch inside the timed region"
    if graphed:
        # ROCm refuses timing events inside a captured graph (torch: "External events are
        # disallowed in rocm"; hipEventRecordWithFlags(external) fails in capture), so the same
        # launches are timed in two eager steps right after the timed region
        ops.TIMER.reset()
        ops.TIMER.match = match
        model._use_graph = False
        for i in range(2):
            model.set_input(inputs[args.warmup + i])
            model.optimize_parameters()
        model._use_graph = True
        ops.TIMER.match = None
        timing = "HIP events around each launch, 2 eager steps right after the timed (graph-replayed) region"
    kern_ms = ops.TIMER.mean_ms()
    n_kern = len(ops.TIMER.events)

    if rank != 0:
        dist.destroy_process_group() if dist is not None else None
        return

    patches = world * args.batch * args.steps
    value = patches / elapsed
    if unet:
        flops_launch = 2.0 * n_launch * s4 ** 3 * c4 * args.ngf * 64
    else:
        flops_launch = 2.0 * n_launch * s4 ** 3 * c4 * c4 * 27
    achieved = flops_launch / (kern_ms / 1e3) / 1e12 if kern_ms else None
    step_tf = step_flops(args.size, args.batch, args.ngf, args.netG) / 1e12
    x3 = args.precision == "bf16x3"
    # bf16x3 issues 3 bf16 MFMAs per fp32 product: its ceiling for the algorithmic (fp32) FLOPs is
    # the bf16 dense peak / 3
    peak = MFMA_BF16_PEAK_TFLOPS / 3 if x3 else MFMA_F32_PEAK_TFLOPS
    prec = "bf16x3 split MFMA" if x3 else "f32 MFMA"
    if unet:
        kname = (f"conv_igemm_kernel ({prec}, parity classes) level-1 upconv ConvTranspose3d {c4}->{args.ngf} k4 s2 "
                 f"[{n_launch}x{s4}^3 in]")
        traffic = measured_traffic(f"unet_up1:S{args.size}:N{n_launch}:ngf{args.ngf}" + (":bf16x3" if x3 else ""))
    else:
        kname = (f"{'conv_brick_x3_kernel' if x3 else 'conv_brick_kernel'} (LDS-halo implicit GEMM, {prec}) "
                 f"res-block conv {c4}->{c4} k3 [{n_launch}x{s4}^3] fwd")
        traffic = measured_traffic(f"res_fwd:S{args.size}:N{n_launch}:ngf{args.ngf}" + (":bf16x3" if x3 else ""))
    res = {
        "metric": "3D patches/sec per CycleGAN step (G+D fwd+bwd)",
        "value": round(value, 3),
        "unit": "patches/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if not x3 else "f32 (bf16x3 split products, f32 accumulate)",
        "data": "synthetic N(0,1) volumes, random init (seed 0)",
        "config": {"workload": f"CycleGAN optimize_parameters(), {args.netG} G + 3-layer PatchGAN D, 1ch->1ch, "
                               f"{args.size}^3 patch, batch {args.batch}/GPU ("
                               + ("BASELINE configs[3] generator family" if args.netG.startswith("unet")
                                  else "BASELINE configs[1] shape") + "; fp32 tensors)",
                   "conv_precision": args.precision,
                   "global_batch": world * args.batch, "patch": args.size, "ngf": args.ngf, "ndf": args.ngf,
                   "parallelism": f"dp{world}",
                   "step_launch": "hip_graph" if graphed else "eager"},
        "roofline": {"bound": "mfma", "kernel": kname,
                     "achieved": round(achieved, 2) if achieved else None, "peak": round(peak, 1),
                     "unit": "TFLOP/s", "frac": round(achieved / peak, 4) if achieved else None,
                     "traffic": traffic, "launch_ms": round(kern_ms, 4) if kern_ms else None,
                     "launches_timed": n_kern, "flop_per_launch": flops_launch, "timing": timing},
        "step_tflop": round(step_tf, 4),
        "step_tflops_achieved": round(step_tf * args.steps / elapsed, 2),
    }
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_child(args)
    print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
