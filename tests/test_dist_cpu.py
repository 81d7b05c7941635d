"""Data-parallel path on CPU with torch.distributed/gloo, world_size 2.

* GradSync (mragan_hip/dist.py) sums flat gradient buffers across ranks and returns 1/world
  (folded into the fused Adam kernel on the GPU).
* The exchange is exact for this step: averaging the per-rank gradients of the CycleGAN step
  on one patch each equals the gradient of the same step on both patches (InstanceNorm is
  per instance; the losses are means over equal shards).  Checked with the fp64 CPU oracle,
  whose gradients are flattened and exchanged through the same GradSync.
"""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _flat(grads):
    return torch.cat([g.reshape(-1) for net in ("G_A", "G_B", "D_A", "D_B") for g in grads[net].values()])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [root, os.path.join(root, "mra-gan_amd")]
        from mragan_hip.dist import GradSync, default_sync
        from oracle.cyclegan_oracle import CycleGANOracle, synthetic_pair

        sync = default_sync()
        assert isinstance(sync, GradSync) and sync.world == world
        # 1) sum + scale semantics
        bufs = [torch.full((5,), float(rank + 1)), torch.arange(3, dtype=torch.float32) * (rank + 1)]
        sync.start(bufs)
        scale = sync.finish()
        assert scale == 0.5
        assert torch.equal(bufs[0], torch.full((5,), 3.0))
        assert torch.equal(bufs[1], torch.arange(3, dtype=torch.float32) * 3)
        # 2) averaged per-rank step gradients == full-batch step gradients (fp64 oracle)
        kw = dict(input_nc=1, output_nc=1, ngf=4, ndf=4, n_blocks=2, dtype=torch.float64)
        A, B = synthetic_pair((2, 1, 24, 24, 24), 4242)
        torch.manual_seed(0)
        mine = CycleGANOracle(pool_rng=random.Random(0), **kw)
        mine.optimize_parameters(A[rank:rank + 1], B[rank:rank + 1])
        g = _flat(mine.grads)
        sync.start([g])
        g *= sync.finish()
        if rank == 0:
            torch.manual_seed(0)
            full = CycleGANOracle(pool_rng=random.Random(0), **kw)
            full.optimize_parameters(A, B)
            ref = _flat(full.grads)
            q.put(float((g - ref).norm() / ref.norm()))
    finally:
        dist.destroy_process_group()


def test_gradsync_and_dp_exactness_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    err = q.get(timeout=5)
    assert err < 1e-10, err


def test_no_sync_without_process_group():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "mra-gan_amd")]
    from mragan_hip.dist import default_sync
    if dist.is_initialized():
        pytest.skip("a process group is already initialised")
    assert default_sync() is None


def test_group_grads_one_buffer_per_optimizer():
    """DP exchanges one buffer per optimizer (G_A + G_B, D_A + D_B):
    networks3D.group_grads makes each net's flat gradient (and its .grad views) a slice of one
    contiguous buffer, keeps the current gradients, is idempotent, and regroups after a net is
    re-flattened."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "mra-gan_amd")]
    from models import networks3D as N3
    torch.manual_seed(0)
    nets = [N3.ResnetGenerator(1, 1, 4, norm_layer=N3.get_norm_layer("instance"), n_blocks=2) for _ in range(2)]
    for n in nets:
        N3.flatten_parameters(n)
        n._flat_grad.normal_()
    before = [n._flat_grad.clone() for n in nets]
    buf = N3.group_grads(nets)
    assert buf.numel() == sum(b.numel() for b in before)
    assert torch.equal(buf, torch.cat(before))
    p0 = next(nets[1].parameters())
    p0.grad.fill_(7.0)                      # a .grad view writes into the shared buffer
    off = nets[0]._flat_grad.numel()
    assert float(buf[off]) == 7.0
    assert N3.group_grads(nets) is buf      # idempotent
    for n in nets:
        assert not N3.ensure_flat(n)        # the grouping keeps the parameter storage
    assert N3.group_grads(nets) is buf
    N3.flatten_parameters(nets[0])          # re-flattened: a new, regrouped buffer
    buf2 = N3.group_grads(nets)
    assert buf2 is not buf and nets[0]._flat_grad.data_ptr() == buf2.data_ptr()
