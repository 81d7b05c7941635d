#!/usr/bin/env python3
"""Per-kernel microbenchmark at the 64³ / batch-2 bench shapes (GPU box), for rocprofv3
kernel traces and PMC counter passes.  Each selected op runs `--reps` times.

    python tools/kbench.py [--ops head_fwd,stem_fwd,...] [--reps 20] [--S 64] [--N 4]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mra-gan_amd"))

import torch  # noqa: E402

from mragan_hip import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="all")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--S", type=int, default=64)
    ap.add_argument("--N", type=int, default=4)
    ap.add_argument("--ngf", type=int, default=32)
    ap.add_argument("--precision", default="f32")
    args = ap.parse_args()
    ops.set_conv_precision(args.precision)
    S, N, ngf = args.S, args.N, args.ngf
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape):
        return torch.randn(shape, device=dev, generator=g)

    c4 = 4 * ngf
    s4 = S // 4
    x_head = rnd(N, S + 6, S + 6, S + 6, ngf)           # padded up2 output
    w_head = rnd(343 * 1 * ngf) * 0.01
    x_stem = rnd(N, S + 6, S + 6, S + 6, 1)
    w_stem = rnd(343 * ngf) * 0.01
    x_res = rnd(N, s4 + 2, s4 + 2, s4 + 2, c4)
    w_res = rnd(27 * c4 * c4) * 0.01
    dy_res = rnd(N, s4, s4, s4, c4)
    dz = rnd(N, S, S, S, 1)
    dh1 = rnd(N, S, S, S, ngf)
    x_in = rnd(N, S, S, S, ngf)
    dy_in = rnd(N, S + 6, S + 6, S + 6, ngf)
    gw_res = torch.empty(c4 * c4 * 27, device=dev)
    gw_head = torch.empty(343 * ngf, device=dev)

    s2 = S // 2
    x_up2 = rnd(N, s2, s2, s2, 2 * ngf)
    w_up2 = rnd(27 * ngf * 2 * ngf) * 0.01
    x_dn1 = rnd(N, S, S, S, ngf)
    w_dn1 = rnd(27 * ngf * 2 * ngf) * 0.01
    x_dl = rnd(N, S // 8 - 1, S // 8 - 1, S // 8 - 1, 512)   # PatchGAN last layer input (ndf 64)
    w_dl = rnd(64 * 512) * 0.01
    dy_dn1 = rnd(N, s2, s2, s2, 2 * ngf)
    gw_dn1 = torch.empty(27 * ngf * 2 * ngf, device=dev)
    x_dn2 = rnd(N, s2, s2, s2, 2 * ngf)
    dy_dn2 = rnd(N, s4, s4, s4, c4)
    gw_dn2 = torch.empty(27 * 2 * ngf * c4, device=dev)
    x_in16 = rnd(N, s4, s4, s4, c4)                      # res-block InstanceNorm [N x 16^3 x 128]
    dy_in16 = rnd(N, s4 + 2, s4 + 2, s4 + 2, c4)
    dy_df = rnd(N, s2, s2, s2, ngf)                      # D first layer output gradient (ndf = ngf)
    w_df = rnd(64 * ngf) * 0.01
    x_up1 = rnd(N, s4, s4, s4, c4)                        # G up1 ConvTranspose3d(128 -> 64, k3 s2) input
    w_up1 = rnd(27 * c4 * 2 * ngf) * 0.01
    w_dn2 = rnd(27 * 2 * ngf * c4) * 0.01
    x_d2 = rnd(N, s2, s2, s2, ngf)                        # PatchGAN layer 2 Conv3d(ndf -> 2ndf, k4 s2 p1) input
    w_d2 = rnd(64 * ngf * 2 * ngf) * 0.01
    dy_d2 = rnd(N, S // 4, S // 4, S // 4, 2 * ngf)     # its output gradient
    gw_d2 = torch.empty(64 * ngf * 2 * ngf, device=dev)
    x_ut = rnd(N, s4, s4, s4, c4)                        # UNet up conv ConvTranspose3d(128 -> 32, k4 s2) input
    dy_ut = rnd(N, s2, s2, s2, ngf)                      # and its output gradient
    gw_ut = torch.empty(64 * c4 * ngf, device=dev)
    w_ut = rnd(64 * c4 * ngf) * 0.01                      # ConvTranspose3d(128 -> 32, k4 s2 p1) weights
    x_df = rnd(N, S, S, S, 1)                            # D first layer input (1 channel)
    w_dfw = rnd(64 * ngf) * 0.01
    b_df = rnd(ngf)
    part_stem = ops.in_partials_buffer(N, (S, S, S), ngf, dev)
    h_up2 = rnd(N, S, S, S, ngf)                         # G up2's conv output (the head's IN input)
    m_up2 = rnd(N, ngf) * 0.1
    r_up2 = torch.rand(N, ngf, device=dev) + 0.5
    part_head = ops.in_partials_buffer(N, (S + 6, S + 6, S + 6), ngf, dev)
    x_uo = rnd(N, s2, s2, s2, 2 * ngf)                    # UNet outermost upconv input (2·ngf channels)
    w_uo = rnd(64 * 2 * ngf) * 0.01
    b_uo = rnd(1)
    # a generator's repack: 18 res-block convs x (fp32 fwd / bwd packs + bf16 split fwd / bwd)
    w_g = [rnd(c4 * c4 * 27) for _ in range(18)]
    pk = [(w, c4, c4, 27, tr, torch.empty_like(w)) for w in w_g for tr in (0, 1, 2, 3)]
    pack_tab = ops.PackTable()
    # 16-bit operand planes (ABI 11; bf16 / fp16 modes): the res-block convs on planes
    dt16 = ops.op16_dtype()
    if dt16 is not None:
        x_res16, dy_res16 = x_res.to(dt16), dy_res.to(dt16)
        ws_res_f = torch.empty(w_res.numel(), device=dev)
        ws_res_b = torch.empty(w_res.numel(), device=dev)
        base = 4 if args.precision == "fp16" else 2
        ops.pack_weight(w_res, c4, c4, 27, base, ws_res_f)
        ops.pack_weight(w_res, c4, c4, 27, base + 1, ws_res_b)
        part_res = ops.in_partials_buffer(N, (s4, s4, s4), c4, dev)
        h1_res = rnd(N, s4, s4, s4, c4)
        _, m_res, r_res = ops.instnorm_fwd(h1_res, act="relu", ypad=1)
        part_bs = ops.in_partials_buffer(N, (s4 + 2,) * 3, c4, dev)
        # G down1 / down2 on the planes of their inputs (ABI 14)
        x_dn1_16, x_dn2_16 = x_dn1.to(dt16), x_dn2.to(dt16)
        # ... with their pre-split forward weights and IN partials: the stride-2 brick (round 6)
        ws_dn1, ws_dn2 = torch.empty(w_dn1.numel(), device=dev), torch.empty(w_dn2.numel(), device=dev)
        ops.pack_weight(w_dn1, 2 * ngf, ngf, 27, base, ws_dn1)
        ops.pack_weight(w_dn2, c4, 2 * ngf, 27, base, ws_dn2)
        part_dn1 = ops.in_partials_buffer(N, (s2, s2, s2), 2 * ngf, dev)
        part_dn2 = ops.in_partials_buffer(N, (s4, s4, s4), c4, dev)
    table = {
        "down1_fwd16": lambda: ops.conv3d_op16(x_dn1_16, w_dn1, 2 * ngf, 3, 2, 1, (s2, s2, s2), None),
        "down2_fwd16": lambda: ops.conv3d_op16(x_dn2_16, w_dn2, c4, 3, 2, 1, (s4, s4, s4), None),
        "down1_fwd16s": lambda: ops.conv3d_op16(x_dn1_16, w_dn1, 2 * ngf, 3, 2, 1, (s2, s2, s2), ws_dn1, part_dn1),
        "down2_fwd16s": lambda: ops.conv3d_op16(x_dn2_16, w_dn2, c4, 3, 2, 1, (s4, s4, s4), ws_dn2, part_dn2),
        "down1_wgrad16": lambda: ops.conv3d_wgrad_g16(dy_dn1, x_dn1_16, 3, 2, 1, gw_dn1, False),
        "down2_wgrad16": lambda: ops.conv3d_wgrad_g16(dy_dn2, x_dn2_16, 3, 2, 1, gw_dn2, False),
        "res_fwd16": lambda: ops.conv3d_op16(x_res16, w_res, c4, 3, 1, 0, (s4, s4, s4), ws_res_f, part_res),
        "res_dgrad16": lambda: ops.conv3d_op16(dy_res16, w_res, c4, 3, 1, 0, (s4 + 2,) * 3, ws_res_b, transposed=True),
        "res_wgrad16": lambda: ops.conv3d_wgrad_op16(dy_res16, x_res16, 3, 1, 0, gw_res, False),
        # the step's form since round 6 (ABI 19): a generator's first-pass (N) and cycle-pass (N/2)
        # instances of one ResnetBlock conv in one launch
        "res_wgrad16p": lambda: ops.conv3d_wgrad_op16_pair(dy_res16, x_res16, dy_res16[:N // 2], x_res16[:N // 2],
                                                           3, 1, 0, gw_res, False),
        # the step's form of the res dgrad: with the backward statistics of the IN in front (ABI 11)
        "res_dgrad16s": lambda: ops.conv3d_op16_dgrad_in_stats(dy_res16, w_res, c4, ws_res_b, h1_res, m_res, r_res,
                                                               "relu", part_bs),
        "pack_g": lambda: pack_tab.run(pk),
        "up1_fwd": lambda: ops.conv3d(x_up1, w_up1, 2 * ngf, 3, 2, 1, (s2, s2, s2), transposed=True),
        "down2_fwd": lambda: ops.conv3d(x_dn2, w_dn2, c4, 3, 2, 1, (s4, s4, s4)),
        "d2_fwd": lambda: ops.conv3d(x_d2, w_d2, 2 * ngf, 4, 2, 1, (S // 4, S // 4, S // 4)),
        "unet_ct": lambda: ops.conv3d(x_ut, w_ut, ngf, 4, 2, 1, (s2, s2, s2), transposed=True),
        "d2_wgrad": lambda: ops.conv3d_wgrad(dy_d2, x_d2, 4, 2, 1, gw_d2, False),
        "unet_up_wgrad": lambda: ops.conv3d_wgrad(x_ut, dy_ut, 4, 2, 1, gw_ut, False),
        "dfirst_fwd": lambda: ops.conv3d(x_df, w_dfw, ngf, 4, 2, 1, (s2, s2, s2), bias=b_df, act="lrelu"),
        "head_fwd16": lambda: ops.conv3d_thin_op16(x_head.to(dt16), w_head, 1, 7, 1, 0, (S, S, S), act="tanh"),
        "stem_dgrad16": lambda: ops.conv3d_thin_op16(dh1.to(dt16), w_head, 1, 7, 1, 0, (S + 6,) * 3, transposed=True),
        "head_wgrad16": lambda: ops.conv3d_wgrad_thin_op16(dz, x_head.to(dt16), 7, 1, 0, gw_head, False),
        "stem_wgrad16": lambda: ops.conv3d_wgrad_thin_op16(dh1.to(dt16), x_stem, 7, 1, 0, gw_head, False),
        "stem_fwd_st": lambda: ops.conv3d_in_stats(x_stem, w_stem, ngf, 7, 1, 0, (S, S, S), None, part_stem),
        "head_dgrad_st": lambda: ops.conv3d_dgrad_in_stats(dz, w_stem, ngf, 7, h_up2, m_up2, r_up2, "relu", 3,
                                                           part_head),
        "unet_up": lambda: ops.conv3d(x_uo, w_uo, 1, 4, 2, 1, (S, S, S), bias=b_uo, act="tanh", transposed=True),
        "dfirst_dgrad": lambda: ops.conv3d(dy_df, w_df, 1, 4, 2, 1, (S, S, S), transposed=True),
        "down1_wgrad": lambda: ops.conv3d_wgrad(dy_dn1, x_dn1, 3, 2, 1, gw_dn1, False),
        "down2_wgrad": lambda: ops.conv3d_wgrad(dy_dn2, x_dn2, 3, 2, 1, gw_dn2, False),
        "dlast_fwd": lambda: ops.conv3d(x_dl, w_dl, 1, 4, 1, 1, (S // 8 - 2,) * 3),
        "up2_fwd": lambda: ops.conv3d(x_up2, w_up2, ngf, 3, 2, 1, (S, S, S), transposed=True),
        "down1_fwd": lambda: ops.conv3d(x_dn1, w_dn1, 2 * ngf, 3, 2, 1, (s2, s2, s2)),
        "head_fwd": lambda: ops.conv3d(x_head, w_head, 1, 7, 1, 0, (S, S, S), act="tanh"),
        "stem_dgrad": lambda: ops.conv3d(dh1, w_head, 1, 7, 1, 0, (S + 6,) * 3, transposed=True),
        "stem_fwd": lambda: ops.conv3d(x_stem, w_stem, ngf, 7, 1, 0, (S, S, S)),
        "head_dgrad": lambda: ops.conv3d(dz, w_stem, ngf, 7, 1, 0, (S + 6,) * 3, transposed=True),
        "head_wgrad": lambda: ops.conv3d_wgrad(dz, x_head, 7, 1, 0, gw_head, False),
        "stem_wgrad": lambda: ops.conv3d_wgrad(dh1, x_stem, 7, 1, 0, gw_head, False),
        "res_fwd": lambda: ops.conv3d(x_res, w_res, c4, 3, 1, 0, (s4, s4, s4)),
        "res_dgrad": lambda: ops.conv3d(dy_res, w_res, c4, 3, 1, 0, (s4 + 2,) * 3, transposed=True),
        "res_wgrad": lambda: ops.conv3d_wgrad(dy_res, x_res, 3, 1, 0, gw_res, False),
        "in_fwd": lambda: ops.instnorm_fwd(x_in, act="relu", ypad=3),
        "in_fwd16": lambda: ops.instnorm_fwd(x_in16, act="relu", ypad=1),
        "in_bwd16": lambda: ops.instnorm_bwd(x_in16, *ops.instnorm_fwd(x_in16, act="relu")[1:], dy_in16, 1, None,
                                             act="relu"),
        "in_bwd": lambda: ops.instnorm_bwd(x_in, *ops.instnorm_fwd(x_in, act="relu")[1:], dy_in, 3, None, act="relu"),
    }
    names = [n for n in table if not n.endswith(("16", "16s"))] if args.ops == "all" else args.ops.split(",")
    for name in names:
        fn = table[name]
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        print(f"{name:12s} {1e6 * (time.perf_counter() - t0) / args.reps:9.1f} us/call (wall, incl. launch)")


if __name__ == "__main__":
    main()
