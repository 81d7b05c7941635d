"""Data-parallel gradient exchange for the CycleGAN step (one process per GPU).

The reference is single-device (networks3D.py:69-75 DataParallel commented out).  Here each
rank trains on its own patch batch and the per-network flat gradient buffers are summed with
one all-reduce each (RCCL over xGMI when the backend is "nccl"; gloo in CPU tests).  The
1/world_size factor is folded into the fused Adam kernel (`grad_scale`), so averaging costs no
extra pass.  Every op in G and D is per-instance (InstanceNorm) and the losses are means over
equal-sized shards, so the averaged gradient equals the global-batch gradient.

Overlap: the G all-reduce is launched asynchronously right after backward_G and waited on only
before the G optimizer step, which runs after the whole D phase (exact: the D phase reads the
pre-update fakes and D weights only).  torch.distributed's NCCL backend runs collectives on its
own stream, ordered after the work already queued on the current stream.
"""
from __future__ import annotations

from typing import List, Optional


class GradSync:
    """Asynchronous SUM all-reduce of a list of flat gradient buffers."""

    def __init__(self, dist_mod=None, group=None):
        self.dist = dist_mod
        self.group = group
        self.works: List = []

    @property
    def world(self) -> int:
        return self.dist.get_world_size(self.group) if self.dist is not None else 1

    def start(self, flat_grads) -> None:
        if self.dist is None:
            return
        self.works = [self.dist.all_reduce(g, group=self.group, async_op=True) for g in flat_grads]

    def finish(self) -> float:
        """Wait for the launched all-reduces; returns the gradient scale 1/world_size."""
        for w in self.works:
            w.wait()
        self.works = []
        return 1.0 / self.world


def default_sync() -> Optional[GradSync]:
    """A GradSync over the default process group if one with >1 ranks is initialised."""
    try:
        import torch.distributed as dist
    except ImportError:
        return None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return GradSync(dist)
    return None
