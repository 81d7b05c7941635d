#!/usr/bin/env python3
"""Out-of-bounds write probe for the ResnetBlock data gradient (whole-grid brick, or the interior +
shell split with MRAGAN_DGRAD_SPLIT=1): the output is placed in the middle of a sentinel-filled
buffer, the guard bands must come back untouched and the output must equal ops.conv3d_op16's.
    python tools/probes/oob_probe.py [bf16|fp16] [NxS,...]"""
import ctypes as _ct
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mra-gan_amd"))
from mragan_hip import ops  # noqa: E402
from mragan_hip.ops import call, query, WS  # noqa: E402

SENT = 12345.0


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    ops.set_conv_precision(prec)
    dt = ops.op16_dtype()
    C = 128
    cases = [(2, 32), (1, 32), (4, 16), (2, 16)]
    if len(sys.argv) > 2:
        cases = [tuple(int(v) for v in c.split("x")) for c in sys.argv[2].split(",")]
    bad = 0
    for N, S in cases:
        g = torch.Generator().manual_seed(N + S)
        wf = (torch.randn(27 * C * C, generator=g) * 0.05).cuda()
        wp = torch.empty_like(wf)
        ops.pack_weight(wf, C, C, 27, 1, wp)
        ws_b = torch.empty_like(wf)
        ops.pack_weight(wf, C, C, 27, (4 if prec == "fp16" else 2) + 1, ws_b)
        dy = torch.randn(N, S, S, S, C, generator=g).cuda().to(dt)
        O = S + 2
        total = N * O * O * O * C
        G = 1 << 20
        buf = torch.full((total + 2 * G,), SENT, device="cuda")
        y = buf[G:G + total]
        nbytes = query("mragan_conv3d_workspace", N, S, S, S, C, C, 3, 1, 0, O, O, O, 1)
        ws = WS.get(nbytes) if nbytes else None
        call("mragan_conv3d_op16", dy.data_ptr(), N, S, S, S, C, wp.data_ptr(), ws_b.data_ptr(), C, 3, 1, 0,
             y.data_ptr(), O, O, O, 1, None if ws is None else ws.data_ptr(), nbytes, None, 0, None,
             torch.cuda.current_stream().cuda_stream)
        ref, _ = ops.conv3d_op16(dy, wp, C, 3, 1, 0, (O, O, O), ws_b, transposed=True)
        torch.cuda.synchronize()
        lo = int((buf[:G] != SENT).sum())
        hi = int((buf[G + total:] != SENT).sum())
        untouched = int((y == SENT).sum())
        same = torch.equal(y.view_as(ref), ref)
        ok = lo == 0 and hi == 0 and untouched == 0 and same
        bad += not ok
        print(f"N={N} S={S}: guard writes below {lo} above {hi}, outputs left unwritten {untouched}, "
              f"equal to ops.conv3d_op16 {same}  {'OK' if ok else 'FAIL'}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
