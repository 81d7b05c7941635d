#!/usr/bin/env python3
"""ResnetBlock whole-grid data gradient (k3 s1 p0 transposed, 16-bit operand plane of dY) against
fp64 on the rounded operands, and its HIP-event time — run once with MRAGAN_DGRAD_SPLIT=1 (interior
brick + shell pass) and once without (whole-grid brick) to compare the two dispatches.
    python tools/probes/split_dgrad_probe.py [bf16|fp16] [NxS,...]"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mra-gan_amd"))
from mragan_hip import ops  # noqa: E402


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    ops.set_conv_precision(prec)
    dt = ops.op16_dtype()
    C = 128
    tag = {"1": "split", "0": "whole"}.get(os.environ.get("MRAGAN_DGRAD_SPLIT", ""), "default")
    cases = [(2, 16), (4, 16), (1, 32), (2, 32), (1, 24)]
    if len(sys.argv) > 2:                      # e.g. "2x24,4x24"
        cases = [tuple(int(v) for v in c.split("x")) for c in sys.argv[2].split(",")]
    for N, S in cases:
        g = torch.Generator().manual_seed(N * 7 + S)
        w = torch.randn(C, C, 3, 3, 3, generator=g, dtype=torch.float64) * 0.05
        wf = w.float().cuda().contiguous()
        wp_b = torch.empty(w.numel(), device="cuda")
        ops.pack_weight(wf, C, C, 27, 1, wp_b)
        ws_b = torch.empty(w.numel(), device="cuda")
        ops.pack_weight(wf, C, C, 27, (4 if prec == "fp16" else 2) + 1, ws_b)
        dy = torch.randn(N, S, S, S, C, generator=g).cuda().to(dt)
        out = (S + 2,) * 3
        dx, _ = ops.conv3d_op16(dy, wp_b, C, 3, 1, 0, out, ws_b, transposed=True)
        torch.cuda.synchronize()
        w16 = wf.to(dt).double().cpu()
        ref = F.conv_transpose3d(dy.double().cpu().permute(0, 4, 1, 2, 3), w16).permute(0, 2, 3, 4, 1)
        err = ((dx.double().cpu() - ref).norm() / ref.norm()).item()
        ok = torch.isfinite(dx).all().item() and err < 2e-5
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            ops.conv3d_op16(dy, wp_b, C, 3, 1, 0, out, ws_b, transposed=True)
        e0.record(st)
        for _ in range(20):
            ops.conv3d_op16(dy, wp_b, C, 3, 1, 0, out, ws_b, transposed=True)
        e1.record(st)
        torch.cuda.synchronize()
        print(f"{tag} {prec} N={N} S={S}: rel err {err:.2e} {'OK' if ok else 'FAIL'}  {e0.elapsed_time(e1) / 20 * 1000:.1f} us")
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
