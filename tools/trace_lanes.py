#!/usr/bin/env python3
"""Lane / idle analysis of a rocprofv3 --kernel-trace CSV of `bench.py --no-kernel-timing`
(graph-replayed steps on two streams).

Per step (steps end at every 4th `adam_dev` dispatch: G_A+G_B, D_A+D_B): wall time, kernel time
per hardware queue, the union of all kernels' busy intervals and the idle rest; and the cost of
the generator-to-generator boundary of the cycle pass (the north star's "fused G_A→G_B pass"):
on one queue, G_A's 32→1 k7 head (`thinn_x3`) → `rpad` of fake_B → G_B's stem weight pack
(`thin1_pack`) → G_B's 1→32 k7 stem (`thin1`): the launches and gaps a fused head+stem kernel
could remove at most.

    python3 tools/trace_lanes.py gpurun_out/TAG/trace/.../bench_kernel_trace.csv --last 10
"""
import argparse
import csv
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("mragan::", "")
    return n.split("<")[0]


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=10, help="analyse the last N steps")
    a = ap.parse_args()
    rows = []
    with open(a.trace, newline="") as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], short(r["Kernel_Name"]),
                         r["Grid_Size_X"]))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if r[3] == "adam_dev_kernel"]
    ends = [rows[adam[k]][1] for k in range(3, len(adam), 4)]
    if len(ends) < 2:
        raise SystemExit("fewer than 2 steps found (adam_dev_kernel × 4 per step)")
    bounds = list(zip(ends[:-1], ends[1:]))[-a.last:]
    print(f"# lanes / idle: {a.trace}\n\n{len(bounds)} steps (each from the previous step's last D Adam)\n")
    print("| step | wall ms | kernel ms (all queues) | busy ms (union) | idle ms | per queue ms |")
    print("|---:|---:|---:|---:|---:|---|")
    agg = defaultdict(float)
    bnd = []
    for si, (t0, t1) in enumerate(bounds):
        sel = [r for r in rows if r[0] >= t0 and r[1] <= t1]
        perq = defaultdict(int)
        for s, e, q, n, g in sel:
            perq[q] += e - s
        busy = union_len([(s, e) for s, e, *_ in sel])
        wall = t1 - t0
        tot = sum(perq.values())
        agg["wall"] += wall
        agg["tot"] += tot
        agg["busy"] += busy
        print(f"| {si} | {wall / 1e6:.3f} | {tot / 1e6:.3f} | {busy / 1e6:.3f} | {(wall - busy) / 1e6:.3f} | "
              + ", ".join(f"q{q}: {v / 1e6:.2f}" for q, v in sorted(perq.items())) + " |")
        # generator boundary: thinn_x3 → rpad → thin1_pack → thin1 on one queue
        byq = defaultdict(list)
        for r in sel:
            byq[r[2]].append(r)
        for q, lst in byq.items():
            for i in range(len(lst) - 3):
                names = [lst[i + k][3] for k in range(4)]
                if names[0].startswith("thinn_x3_kernel") and names[1] == "rpad_kernel" and \
                        "pack" in names[2] and names[3].startswith("thin1"):
                    h, rp, pk, st = lst[i:i + 4]
                    bnd.append(dict(gap1=rp[0] - h[1], rpad=rp[1] - rp[0], gap2=pk[0] - rp[1], pack=pk[1] - pk[0],
                                    gap3=st[0] - pk[1], head=h[1] - h[0], stem=st[1] - st[0]))
    n = len(bounds)
    print(f"\nmean: wall {agg['wall'] / n / 1e6:.3f} ms, kernel time {agg['tot'] / n / 1e6:.3f} ms, busy (union) "
          f"{agg['busy'] / n / 1e6:.3f} ms, idle {(agg['wall'] - agg['busy']) / n / 1e6:.3f} ms per step")
    if bnd:
        m = {k: sum(b[k] for b in bnd) / len(bnd) / 1e3 for k in bnd[0]}
        per_step = len(bnd) / n
        removable = m["gap1"] + m["rpad"] + m["gap2"] + m["pack"] + m["gap3"]
        print(f"\n## G_A head → G_B stem boundary ({len(bnd)} occurrences, {per_step:.1f} per step; µs)\n")
        print("| head | gap | rpad | gap | stem pack | gap | stem | removable by fusing head + stem |")
        print("|---:|---:|---:|---:|---:|---:|---:|---:|")
        print(f"| {m['head']:.1f} | {m['gap1']:.1f} | {m['rpad']:.1f} | {m['gap2']:.1f} | {m['pack']:.1f} | "
              f"{m['gap3']:.1f} | {m['stem']:.1f} | {removable:.1f} (× {per_step:.1f} per step = "
              f"{removable * per_step / 1e3:.3f} ms) |")


if __name__ == "__main__":
    main()
