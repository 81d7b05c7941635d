#!/usr/bin/env python3
"""Benchmark: 3D patches/sec of one full CycleGAN optimize_parameters() step
(G_A, G_B, D_A, D_B forward + backward + both Adam steps), BASELINE.json's metric.

Workload (N=1): BASELINE configs[1] — ResNet-9blocks G + 3-layer PatchGAN D, 1ch→1ch,
64³ patch, batch 2 per GPU, bf16 (every convolution operand rounded to bf16, fp32 accumulation;
the step is pinned against the oracle's rounded-operand step, tests/test_step_gpu.py), synthetic
N(0,1) volumes, random init (seed 0).  The fp32-grade modes (bf16x3 split products, exact f32)
are timed in the same run under alt_precisions.  Multi-GPU:
one process per GPU (torch.distributed over RCCL), each rank its own batch (weak scaling),
gradients all-reduced inside the step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 64] [--batch 2]

With --gpus N > 1 and no torch.distributed environment, the script launches its own N ranks
(torch.distributed.run, one process per GPU, 127.0.0.1 rendezvous) as a child process before
touching the GPU and exits with its status.

Prints ONE JSON line on rank 0 (contract in the task description), with:
  roofline      — the dominant kernel BY TIME: one eager single-stream step (right after the timed
                  region) records every instrumented C-ABI call by launch class (op + shape); each
                  class's call is re-issued 10× back to back (captured once as a HIP graph and
                  replayed) between HIP events on its stream, so the class mean is the kernels' own
                  duration; the class with the largest
                  per-step total is reported with its algorithmic FLOP (or bytes) per launch ÷ that
                  mean;
  step_roofline — SURVEY §8(d)'s whole-step figure, (F/P_mfma + B_ew/BW_hbm) / T_step;
  alt_precisions — the same workload and protocol in the other contraction precisions;
  legs          — further workloads (default: 128³ b1, BASELINE configs[2]'s per-GPU unit), each
                  with its own ms_per_step, roofline and step_roofline;
  cpu_baseline  — the CPU oracle (oracle/cyclegan_oracle.py, the reference's algorithm restated
                  in PyTorch-CPU) timed on this host: --cpu-warmup untimed steps, then the median
                  of --cpu-steps steps of the headline workload.
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
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E peak (spec)


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
    ap.add_argument("--precision", default="bf16", choices=["f32", "bf16x3", "bf16", "fp16"],
                    help="MFMA-conv contraction: exact f32, split-bf16 (bf16x3, fp32-grade), or bf16 / fp16 "
                         "operands (one MFMA per product); fp32 accumulation, fp32 tensors and master weights")
    ap.add_argument("--cpu-steps", type=int, default=3, help="CPU baseline: median of this many oracle steps")
    ap.add_argument("--nc", type=int, default=1, help="image channels (input_nc = output_nc)")
    ap.add_argument("--alt-precisions", default="bf16x3,f32",
                    help="comma list of further precisions timed in the same run (same workload, same protocol) "
                         "and reported under alt_precisions; '' for none")
    ap.add_argument("--legs", default="128:1,96:1:2:resnet_9blocks:fp16,64:1:1:unet_custom:bf16",
                    help="comma list of further workloads SIZE:BATCH[:NC[:NETG[:PRECISION]]] timed in the same run, "
                         "reported under legs; '' for none.  Default: BASELINE configs[2]'s per-GPU unit (128^3 b1), "
                         "configs[4]'s (2ch->2ch 96^3 b1 fp16) and configs[3]'s generator family at 64^3 "
                         "(unet_custom: the reference's unet_256 needs a >= 256^3 patch, networks3D.py:270-343)")
    ap.add_argument("--leg-alt-precisions", default="bf16x3",
                    help="alt precisions timed for each extra leg that runs the headline precision")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-launch-class timing (profiled runs: the trace then holds only the steps)")
    ap.add_argument("--cpu-warmup", type=int, default=2, help="CPU baseline: untimed oracle steps first")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch the step's kernels from Python every step (default: replay the step as HIP graphs)")
    ap.add_argument("--single-stream", action="store_true",
                    help="issue the step on one stream (default: G_A / G_B and D_A / D_B chains on two)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on the node; gloo only for rehearsal")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--full-out", default=os.path.join("gpurun_out", "bench_full.json"),
                    help="file for the full report (every launch class of every leg); the printed line keeps the "
                         "largest few and names this path; '' for none")
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
    orc = CycleGANOracle(input_nc=args.nc, output_nc=args.nc, ngf=args.ngf, ndf=args.ngf, netG=args.netG,
                         pool_rng=random.Random(0))
    shape = (args.batch, args.nc, args.size, args.size, args.size)
    times = []
    for i in range(args.cpu_warmup + args.cpu_steps):
        A, B = synthetic_pair(shape, 1000 + i)
        t0 = time.perf_counter()
        orc.optimize_parameters(A, B)
        if i >= args.cpu_warmup:
            times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": args.batch / t, "unit": "patches/s", "cores": threads, "kind": "port",
            "sample": f"{args.cpu_warmup} warm-up steps, then median of {len(times)} optimize_parameters() steps of the CPU oracle (PyTorch-CPU fp32) on "
                      f"{args.batch}x{args.nc}x{args.size}^3: {t:.2f} s (all: "
                      + ", ".join(f"{x:.2f}" for x in times) + f" s), {threads} threads, {cpu_model}"}


def cpu_baseline_child(args, timeout_s=300):
    """Run cpu_baseline() in a child process (the GPU process only waits), bounded in time."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--size", str(args.size),
           "--batch", str(args.batch), "--ngf", str(args.ngf), "--netG", args.netG, "--cpu-steps", str(args.cpu_steps),
           "--cpu-warmup", str(args.cpu_warmup), "--nc", str(args.nc)]
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


def measured_traffic(kernels, cls):
    """HBM bytes per launch of the dominant launch class from the committed PMC passes
    (profiles/traffic.json, written by tools/pmc_traffic.py: (2·FETCH_SIZE + WRITE_SIZE), the
    gfx950 FETCH_SIZE correction), keyed by "<kernel names>|<launch class>"; None when no pass was
    recorded for this configuration."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as fh:
            rec = json.load(fh)[f"{kernels}|{cls}"]
        return rec["hbm_bytes_per_launch"], rec.get("source")
    except (OSError, KeyError, ValueError):
        return None, None


def launch_ranks(args):
    """--gpus N without a torch.distributed environment: run this script as N ranks under
    torch.distributed.run (a child process; this process never touches the GPU) and return its
    exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def build_model(args, precision, batch=None, nc=None, netG=None):
    from models import create_model
    from options.train_options import TrainOptions
    nc, netG = nc or args.nc, netG or args.netG
    sys_argv = sys.argv
    sys.argv = ["train.py", "--netG", netG, "--ngf", str(args.ngf), "--ndf", str(args.ngf),
                "--input_nc", str(nc), "--output_nc", str(nc),
                "--checkpoints_dir", "/tmp/mragan_bench", "--batch_size", str(batch or args.batch),
                "--conv_precision", precision] + (["--no_cuda_graph"] if args.no_graph else []) + \
        (["--single_stream"] if args.single_stream else [])
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
    return model


def ew_bytes_per_patch(S, netG, elem_bytes=4):
    """SURVEY §8(d) secondary HBM term: the InstanceNorm/activation/pad/residual traffic of one
    patch's step, ≈ 8 passes × 118·S³ elements per G fwd+bwd × 6 G passes = 5664·S³ elements
    (resnet generators; None for the UNet).  Priced in the leg's activation dtype (2 B for the
    bf16 / fp16 modes, BASELINE.md §4: 2.97 GB per 64³ patch; 4 B otherwise)."""
    if netG.startswith("unet"):
        return None
    return 5664.0 * S ** 3 * elem_bytes




DTYPE = {"f32": "f32", "bf16x3": "bf16x3", "bf16": "bf16", "fp16": "fp16"}
DTYPE_DETAIL = {"f32": "exact f32 products (f32 MFMA / VALU), f32 accumulate",
                "bf16x3": "each f32 conv operand split into bf16 hi + lo, a*b as 3 bf16 MFMAs (<= 3*2^-18 per "
                          "product), f32 accumulate; f32 tensors, InstanceNorm, losses, Adam",
                "bf16": "bf16 conv operands (every conv's inputs and weights rounded RNE), f32 accumulate; f32 "
                        "InstanceNorm, losses, Adam, master weights",
                "fp16": "fp16 conv operands with a static loss scale, f32 accumulate; f32 InstanceNorm, losses, "
                        "Adam, master weights"}


def mfma_peak_of(precision):
    # bf16x3 issues 3 bf16 MFMAs per fp32 product: its ceiling for the algorithmic FLOPs is the
    # bf16 dense peak / 3; bf16 / fp16 run at the dense 16-bit MFMA peak
    return {"f32": MFMA_F32_PEAK_TFLOPS, "bf16x3": MFMA_BF16_PEAK_TFLOPS / 3}.get(precision, MFMA_BF16_PEAK_TFLOPS)


VALU_CONV_KERNELS = ("thin_dot", "thin_k", "thin_n", "thin_wgrad", "thin_naive")
FP64_ACC_KERNELS = ("thin_n_class8", "thin_n_tile8")


def kernel_arith(kernels, precision):
    """The arithmetic the named kernels really run (the roofline label): the thin VALU
    convolutions are dot products on the vector ALUs (two accumulate in fp64) whatever the
    contraction mode; InstanceNorm / elementwise kernels move bytes; the rest are MFMA kernels of
    the mode."""
    names = [k for k in kernels.split(";") if k]
    conv = [k for k in names if not k.startswith(("pack", "in_", "wgrad_reduce", "thin_wgrad_reduce", "channel_sum",
                                                   "conv_splitk_reduce", "thin1_wgrad_reduce"))] or names
    head = conv[0] if conv else ""
    rnd = {"f32": "f32", "bf16x3": "f32", "bf16": "bf16-rounded", "fp16": "fp16-rounded"}[precision]
    if head.startswith(FP64_ACC_KERNELS):
        return f"VALU dot, {rnd} operands, fp64 accumulate"
    if head.startswith(VALU_CONV_KERNELS):
        return f"VALU dot, {rnd} operands, f32 accumulate"
    if head.startswith(("in_", "rpad", "act_bwd", "concat", "split", "adam", "l1", "gan", "fill")):
        return "HBM-bound elementwise"
    return {"bf16x3": "bf16x3 split MFMA", "f32": "f32 MFMA", "bf16": "bf16 MFMA", "fp16": "fp16 MFMA"}[precision]


def make_inputs(shape, n, rank):
    g = torch.Generator().manual_seed(1000 + rank)
    return [(torch.randn(shape, generator=g).cuda(), torch.randn(shape, generator=g).cuda()) for _ in range(n)]


def time_steps(model, inputs, warmup, steps, barrier, dist):
    """W untimed steps, then K steps between barrier + synchronize; per-step events on the step's
    stream give the median.  Returns (elapsed s, median ms) as the max over ranks."""
    for i in range(warmup):
        model.set_input(inputs[i])
        model.optimize_parameters()
    barrier()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    barrier()
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(steps):
        model.set_input(inputs[warmup + i])
        model.optimize_parameters()
        marks[i + 1].record()
    barrier()
    wall = time.perf_counter() - t0
    step_ms = sorted(marks[i].elapsed_time(marks[i + 1]) for i in range(steps))
    median_ms = step_ms[len(step_ms) // 2]
    elapsed = max(marks[0].elapsed_time(marks[-1]) / 1e3, wall)
    if dist is not None:
        t = torch.tensor([elapsed, median_ms], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, median_ms = float(t[0]), float(t[1])
    return elapsed, median_ms


def h2d_inclusive(model, inputs, warmup, steps, barrier):
    """The same K steps with the inputs in pinned HOST memory: set_input's host→device copy (the
    reference's .to(device) of the patch pair, cycle_gan_model.py:131-135) inside the timed region.
    Returns ms per step (this rank)."""
    host = [(a.cpu().pin_memory(), b.cpu().pin_memory()) for a, b in inputs[:warmup + steps]]
    for i in range(warmup):
        model.set_input(host[i])
        model.optimize_parameters()
    barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        model.set_input(host[warmup + i])
        model.optimize_parameters()
    barrier()
    return 1e3 * (time.perf_counter() - t0) / steps


def phase_times(model, reps=10):
    """The replayed step's two HIP graphs timed apart (events on the current stream around `reps`
    back-to-back replays each): the G phase (generator forwards, losses, every backward) and the D
    phase (both discriminators' passes) — the D phase is the window the data-parallel G all-reduce
    overlaps.  None when the step is not graphed."""
    if getattr(model, "_graphs", None) is None:
        return None
    out = {}
    names = ("G", "D") if model._graphs[1] is not None else ("G+D overlapped",)
    for name, g in zip(names, model._graphs):
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(e0.elapsed_time(e1) / reps, 3)
    return out


def kernel_classes(model, inputs, reps=10):
    """Launch classes of one step: two eager single-stream steps record every instrumented C-ABI
    call; each class's call is then re-issued `reps` times back to back between HIP events
    (ops.KernelTimer).  The second step's records are the ones a step issues (the first one also
    holds one-off work), so launches per step = records of step 2."""
    from mragan_hip import ops
    use_graph, lanes = model._use_graph, model.parallel_lanes
    model._use_graph, model.parallel_lanes = False, False
    model.set_input(inputs[0])
    model.optimize_parameters()
    ops.TIMER.reset()
    ops.TIMER.match = lambda info: True
    model.set_input(inputs[1])
    model.optimize_parameters()
    ops.TIMER.match = None
    model._use_graph, model.parallel_lanes = use_graph, lanes
    return ops.TIMER.classes(reps)


def run_leg(args, size, batch, precision, alts, barrier, dist, world, rank, nc=None, netG=None, extras=False):
    """One workload: the timed step in `precision`, its launch classes and roofline, and the same
    protocol in each precision of `alts` (a fresh model each).  extras (the headline): also the
    host-input (H2D-inclusive) step time and the two graph phases timed apart."""
    from mragan_hip import ops
    nc, netG = nc or args.nc, netG or args.netG
    shape = (batch, nc, size, size, size)
    inputs = make_inputs(shape, args.warmup + args.steps, rank)
    model = build_model(args, precision, batch, nc, netG)
    elapsed, median_ms = time_steps(model, inputs, args.warmup, args.steps, barrier, dist)
    graphed = getattr(model, "_graphs", None) is not None
    h2d_ms = phases = None
    if extras:
        h2d_ms = h2d_inclusive(model, inputs, args.warmup, args.steps, barrier)
        phases = phase_times(model) if world == 1 else None
    classes = kernel_classes(model, inputs) if not args.no_kernel_timing else None
    loss_scale = model.loss_scale
    del model
    torch.cuda.empty_cache()
    alt = {}
    for p in alts:
        m = build_model(args, p, batch, nc, netG)
        e, med = time_steps(m, inputs, args.warmup, args.steps, barrier, dist)
        alt[p] = {"value": round(world * batch * args.steps / e, 3), "ms_per_step": round(1e3 * e / args.steps, 3),
                  "ms_per_step_median": round(med, 3), "dtype": DTYPE[p]}
        del m
        torch.cuda.empty_cache()
    ops.set_conv_precision(precision)
    ops.set_loss_scale(loss_scale)
    barrier()
    t_step = elapsed / args.steps
    mfma_peak = mfma_peak_of(precision)
    step_tf = step_flops(size, batch, args.ngf, netG, nc=nc) / 1e12
    act_bytes = 2 if precision in ("bf16", "fp16") else 4
    ew = ew_bytes_per_patch(size, netG, act_bytes)
    ew32 = ew_bytes_per_patch(size, netG, 4)
    ideal_s = step_tf / mfma_peak + (batch * ew / (HBM_PEAK_GBS * 1e9) if ew else 0.0)
    ideal32_s = step_tf / mfma_peak + (batch * ew32 / (HBM_PEAK_GBS * 1e9) if ew32 else 0.0)
    leg = {
        "value": round(world * batch * args.steps / elapsed, 3),
        "unit": "patches/s",
        "ms_per_step": round(1e3 * t_step, 3),
        "ms_per_step_median": round(median_ms, 3),
        "dtype": DTYPE[precision],
        "dtype_detail": DTYPE_DETAIL[precision],
        "workload": f"{netG} G + 3-layer PatchGAN D, {nc}ch->{nc}ch, {size}^3 patch, batch {batch}/GPU",
        "step_launch": "hip_graph" if graphed else "eager",
        "step_roofline": {"achieved": round(ideal_s / t_step, 4), "ideal_ms": round(1e3 * ideal_s, 3),
                          "formula": "(F/P_mfma + B_ew/BW_hbm) / T_step (SURVEY 8d)",
                          "F_tflop": round(step_tf, 4), "P_mfma_tflops": round(mfma_peak, 1),
                          "B_ew_gb": round(batch * ew / 1e9, 3) if ew else None, "B_ew_elem_bytes": act_bytes,
                          "BW_hbm_gbs": HBM_PEAK_GBS,
                          "achieved_fp32_storage": round(ideal32_s / t_step, 4),
                          "note": "B_ew priced in the activation dtype of the precision mode; achieved_fp32_storage "
                                  "prices it at 4 B per element"},
        "step_tflop": round(step_tf, 4),
        "step_tflops_achieved": round(step_tf / t_step, 2),
    }
    if h2d_ms is not None:
        leg["h2d_inclusive"] = {"ms_per_step": round(h2d_ms, 3), "value": round(world * batch * 1e3 / h2d_ms, 3),
                                "note": "same steps with the input pair in pinned host memory: set_input's "
                                        "host-to-device copy inside the timed region (never `value`)"}
    if phases:
        leg["phase_ms"] = dict(phases, note="the step's graphs replayed alone (10x each, events); single GPU runs "
                                            "the D phase beside the G backward (one graph), data parallel the "
                                            "two-phase schedule whose D phase the G all-reduce overlaps")
    if alt:
        leg["alt_precisions"] = alt
    if classes:
        dom_cls, dom = next(iter(classes.items()))
        prec = kernel_arith(dom["kernels"], precision)
        if dom["flops"]:
            achieved = dom["flops"] / (dom["mean_ms"] / 1e3) / 1e12
            peak, unit, bound = mfma_peak, "TFLOP/s", "mfma"
        else:
            achieved = dom["bytes"] / (dom["mean_ms"] / 1e3) / 1e9
            peak, unit, bound = HBM_PEAK_GBS, "GB/s", "hbm"
        traffic, traffic_src = measured_traffic(dom["kernels"], dom_cls)
        leg["roofline"] = {
            "bound": bound, "kernel": f"{dom['kernels']} ({prec}) — {dom_cls}",
            "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": unit, "frac": round(achieved / peak, 4),
            "traffic": traffic, "traffic_source": traffic_src,
            "launch_ms": round(dom["mean_ms"], 4), "launches_per_step": dom["n"],
            "ms_per_step": round(dom["total_ms"], 4),
            "flop_per_launch": dom["flops"], "bytes_per_launch": dom["bytes"],
            "timing": f"dominant launch class by time; its C-ABI call re-issued {dom['reps']}x back to back "
                      + ("as one captured HIP graph replayed " if dom.get("graphed") else "")
                      + "between HIP events on the step's stream (after one warm launch), mean per launch"}
        leg["top_kernels"] = [
            dict(cls=c, kernels=v["kernels"], launches_per_step=v["n"], ms_per_step=round(v["total_ms"], 4),
                 mean_us=round(1e3 * v["mean_ms"], 2),
                 frac=round((v["flops"] / (v["mean_ms"] / 1e3) / 1e12) / mfma_peak if v["flops"] else
                            (v["bytes"] / (v["mean_ms"] / 1e3) / 1e9) / HBM_PEAK_GBS, 4))
            for c, v in classes.items()]
        leg["kernel_ms_per_step_serial"] = round(sum(v["total_ms"] for v in classes.values()), 3)
    return leg


LINE_CAP = 7000        # bytes: the driver keeps the last 8000 bytes of stdout; the line must fit whole


def compact_line(res, full_out, n_head=10, n_leg=4):
    """The printed line: the full report (every launch class of every leg, all fields) goes to
    `full_out`, named in the line; the line keeps the headline's `n_head` and each leg's `n_leg`
    largest launch classes as compact rows [class, kernels, launches/step, us/launch, frac], drops
    the legs' explanatory strings, and trims rows further until it fits LINE_CAP."""
    full_path = None
    if full_out:
        if not os.path.isabs(full_out):
            full_out = os.path.join(ROOT, full_out)
        try:
            os.makedirs(os.path.dirname(full_out), exist_ok=True)
            with open(full_out, "w") as fh:
                json.dump(res, fh, indent=1)
            full_path = os.path.relpath(full_out, ROOT)
        except OSError:
            full_path = None

    def rows(tk, n):
        return [[r["cls"], r["kernels"], r["launches_per_step"], r["mean_us"], r["frac"]] for r in tk[:n]]

    out = json.loads(json.dumps(res))
    out["top_kernels_full"] = full_path
    out["top_kernels_cols"] = ["class", "kernels", "launches_per_step", "us_per_launch", "frac"]
    for leg in out.get("legs", {}).values():
        for k in ("dtype_detail", "kernel_ms_per_step_serial", "workload", "step_launch", "step_tflop"):
            leg.pop(k, None)
        for k in ("formula", "note", "BW_hbm_gbs", "P_mfma_tflops", "F_tflop", "B_ew_elem_bytes"):
            leg.get("step_roofline", {}).pop(k, None)
        for k in ("timing", "traffic_source", "flop_per_launch", "bytes_per_launch", "ms_per_step"):
            leg.get("roofline", {}).pop(k, None)
    for nh, nl in ((n_head, n_leg), (8, 3), (6, 2), (5, 1), (4, 0), (3, 0), (0, 0)):
        if "top_kernels" in res:
            out["top_kernels"] = rows(res["top_kernels"], nh)
        for key, leg in res.get("legs", {}).items():
            if "top_kernels" in leg:
                if nl:
                    out["legs"][key]["top_kernels"] = rows(leg["top_kernels"], nl)
                else:
                    out["legs"][key].pop("top_kernels", None)
        if len(json.dumps(out)) <= LINE_CAP:
            break
    return out


def main():
    args = parse()
    if args.cpu_baseline_only:
        print(json.dumps(cpu_baseline(args)), flush=True)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
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

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    alts = [p for p in args.alt_precisions.split(",") if p and p != args.precision]
    head = run_leg(args, args.size, args.batch, args.precision, alts, barrier, dist, world, rank, extras=True)
    legs = {}
    for spec in [s for s in args.legs.split(",") if s]:
        f = spec.split(":")
        S, bsz = int(f[0]), int(f[1])
        nc = int(f[2]) if len(f) > 2 and f[2] else args.nc
        netG = f[3] if len(f) > 3 and f[3] else args.netG
        prec = f[4] if len(f) > 4 and f[4] else args.precision
        if (S, bsz, nc, netG, prec) == (args.size, args.batch, args.nc, args.netG, args.precision):
            continue
        key = f"{S}^3 b{bsz}" + (f" nc{nc}" if nc != args.nc else "") + (f" {netG}" if netG != args.netG else "") + \
            (f" {prec}" if prec != args.precision else "")
        alt_l = [p for p in args.leg_alt_precisions.split(",") if p and p != prec] if prec == args.precision else []
        legs[key] = run_leg(args, S, bsz, prec, alt_l, barrier, dist, world, rank, nc=nc, netG=netG)
        legs[key]["config"] = {"patch": S, "batch": bsz, "nc": nc, "netG": netG, "conv_precision": prec}
    if rank != 0:
        dist.destroy_process_group() if dist is not None else None
        return

    res = {
        "metric": "3D patches/sec per CycleGAN step (G+D fwd+bwd)",
        "value": head["value"],
        "unit": "patches/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "ms_per_step_median": head["ms_per_step_median"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": head["dtype"],
        "dtype_detail": head["dtype_detail"],
        "data": "synthetic N(0,1) volumes, random init (seed 0)",
        "config": {"workload": f"CycleGAN optimize_parameters(), {args.netG} G + 3-layer PatchGAN D, "
                               f"{args.nc}ch->{args.nc}ch, {args.size}^3 patch, batch {args.batch}/GPU ("
                               + ("BASELINE configs[3] generator family" if args.netG.startswith("unet")
                                  else "BASELINE configs[1] shape" if (args.size, args.nc) == (64, 1)
                                  else "per-GPU unit of a BASELINE config") + "; fp32 tensors)",
                   "conv_precision": args.precision,
                   "global_batch": world * args.batch, "patch": args.size, "ngf": args.ngf, "ndf": args.ngf,
                   "parallelism": f"dp{world}",
                   "step_launch": head["step_launch"],
                   "streams": 1 if args.single_stream else 2,
                   "inputs": "device-resident before the timed region (the per-step host-to-device copy of "
                             "the patch pair is timed apart: h2d_inclusive)"},
    }
    for k in ("roofline", "step_roofline", "step_tflop", "step_tflops_achieved", "alt_precisions", "top_kernels",
              "kernel_ms_per_step_serial", "h2d_inclusive", "phase_ms"):
        if k in head:
            res[k] = head[k]
    if legs:
        res["legs"] = legs
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_child(args)
    print(json.dumps(compact_line(res, args.full_out)), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
