"""Child process of test_kernels_gpu.py::test_splitk_in_launch_reduce_bit_identical: recomputes the
split-K convolutions of the input file with the environment the parent gives it (MRAGAN_SK_FUSE=1: the split-K
slices reduced in the launch) and saves the outputs; with partials requested, also the
InstanceNorm statistics from them."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mra-gan_amd"))


def run(ops, cases):
    outs = []
    for c in cases:
        ops.set_conv_precision(c["prec"])
        x, w, b = c["x"].cuda(), c["w"].cuda(), c["b"].cuda() if c["b"] is not None else None
        y = ops.conv3d(x, w, c["cout"], c["k"], c["s"], c["p"], tuple(c["osp"]), bias=b, act=c["act"],
                       transposed=c["tr"])
        outs.append(y.cpu())
        if c.get("stats"):     # the forward InstanceNorm statistics from the conv's partials
            part = ops.in_partials_buffer(x.shape[0], tuple(c["osp"]), c["cout"], "cuda")
            y2, chunks = ops.conv3d_in_stats(x, w, c["cout"], c["k"], c["s"], c["p"], tuple(c["osp"]), None, part)
            _, m, r = ops.instnorm_fwd(y2, act="lrelu", ypad=1, part=part if chunks else None, chunks=chunks)
            outs.append(torch.tensor([float(chunks)]))
            outs.append(m.cpu())
            outs.append(r.cpu())
    ops.set_conv_precision("f32")
    return outs


if __name__ == "__main__":
    from mragan_hip import ops
    cases = torch.load(sys.argv[1], weights_only=True)
    torch.save(run(ops, cases), sys.argv[2])
