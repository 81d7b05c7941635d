#!/usr/bin/env python3
"""Per-launch cost of a dependent kernel chain in a replayed HIP graph (the regime of the step's
two lanes): K tiny fills on one stream captured in a graph, replayed R times; and the same chain
with each kernel sized to a given number of workgroups.  Prints µs per kernel.

    python3 tools/probes/graph_chain_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mra-gan_amd"))
import torch  # noqa: E402

from mragan_hip import ops  # noqa: E402


def chain_cost(numel, K=200, R=20):
    buf = torch.empty(numel, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            for _ in range(K):
                ops.fill(buf, 1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(K):
            ops.fill(buf, 1.0)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(R):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    graph_us = a.elapsed_time(b) * 1000.0 / (R * K)
    # eager, same stream, no host sync between launches
    a.record()
    for _ in range(R):
        for _ in range(K):
            ops.fill(buf, 1.0)
    b.record()
    torch.cuda.synchronize()
    eager_us = a.elapsed_time(b) * 1000.0 / (R * K)
    return graph_us, eager_us


def main():
    for numel in (256, 256 * 256, 256 * 4096, 8 << 20):
        g, e = chain_cost(numel)
        print(f"fill of {numel:>9} floats ({(numel + 255) // 256:>6} wg max): graph {g:6.2f} us/kernel, eager {e:6.2f} us/kernel",
              flush=True)


if __name__ == "__main__":
    main()
