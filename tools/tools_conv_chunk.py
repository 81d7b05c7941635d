"""Importing this module makes fp64 CPU F.conv3d calls run in output-depth slabs (same sums, a
bounded im2col buffer): ATen's fp64 CPU convolution (slow_conv3d) allocates (Cin·k³) × (output
voxels) elements, 184 GB for the 32→1 k7 head at 128³.  Shared by the fixture generators."""
import torch.nn.functional as F

COL_LIMIT = 2 << 30      # bytes of one im2col buffer


def _chunked(orig):
    def conv3d(input, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
        def t3(v):
            return tuple(v) if isinstance(v, (tuple, list)) else (v, v, v)
        st, pd, dl = t3(stride), t3(padding), t3(dilation)
        if isinstance(padding, str) or input.dtype.itemsize != 8 or groups != 1 or dl != (1, 1, 1):
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
        import torch
        outs = []
        for o0 in range(0, Do, rows):
            o1 = min(Do, o0 + rows)
            xs = x[:, :, o0 * st[0]:(o1 - 1) * st[0] + k[0]]
            outs.append(orig(xs, weight, bias, st, 0, 1, 1))
        return torch.cat(outs, 2)
    return conv3d


if not getattr(F.conv3d, "_chunked", False):
    F.conv3d = _chunked(F.conv3d)
    F.conv3d._chunked = True
