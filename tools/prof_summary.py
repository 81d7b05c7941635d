#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV of `bench.py --steps K --warmup W` into a markdown
table: per kernel (template instance) total ms per step, launches per step, mean µs, and the
per-(kernel, grid) mean for the bench's dominant kernel (the res-block conv forward).

    python3 tools/prof_summary.py gpurun_out/r01/trace/bench_kernel_trace.csv --steps 13 \
        --dominant "conv_igemm_f32_kernel<2, 2, 1, 1, 32>" --grid 16384,128,1 > profiles/r01_bench_kernels.md
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True, help="warmup + timed steps profiled")
    ap.add_argument("--dominant", default=None)
    ap.add_argument("--grid", default=None, help="Grid_Size_X,Y,Z of the dominant launch (threads)")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    tot = defaultdict(float)
    cnt = defaultdict(int)
    grid_t = defaultdict(list)
    t_min, t_max = None, None
    with open(a.trace, newline="") as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if name.startswith("__amd_rocclr") or "at::" in name or "elementwise" in name.lower():
                key = "[torch/runtime] " + name.split("(")[0][:60]
            else:
                key = name.split("(")[0].replace("void ", "").replace("mragan::", "")
            dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3  # µs
            tot[key] += dt
            cnt[key] += 1
            g = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
            grid_t[(key, ",".join(g))].append(dt)
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            t_min = s if t_min is None else min(t_min, s)
            t_max = e if t_max is None else max(t_max, e)
    all_us = sum(tot.values())
    print(f"# rocprofv3 kernel trace summary: {a.trace}\n")
    print(f"{a.steps} profiled steps (warm-up included); kernel time {all_us / a.steps / 1e3:.2f} ms/step "
          f"(sum of kernel durations).\n")
    print("| kernel | ms/step | launches/step | mean µs | % |")
    print("|---|---:|---:|---:|---:|")
    for k in sorted(tot, key=lambda k: -tot[k])[:a.top]:
        print(f"| `{k}` | {tot[k] / a.steps / 1e3:.3f} | {cnt[k] / a.steps:.1f} | {tot[k] / cnt[k]:.1f} | "
              f"{100 * tot[k] / all_us:.1f} |")
    if a.dominant:
        key = a.dominant.replace("mragan::", "")
        print(f"\n## dominant kernel `{key}` by grid\n")
        print("| grid (threads x,y,z) | launches | mean µs |")
        print("|---|---:|---:|")
        for (k, g), v in sorted(grid_t.items(), key=lambda kv: -sum(kv[1])):
            if k == key:
                mark = " **(bench roofline launch)**" if g == a.grid else ""
                print(f"| {g}{mark} | {len(v)} | {sum(v) / len(v):.1f} |")


if __name__ == "__main__":
    main()
