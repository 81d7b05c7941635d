#!/usr/bin/env python3
"""Per-stream view of graph-replayed steps in a rocprofv3 --kernel-trace CSV of `bench.py
--no-kernel-timing`: steps are separated by instants where every queue is idle; per step and queue the
busy time, the first start / last end relative to the step start and the idle gaps inside the queue's
active span (waits on other streams' events).  The queue that ends last bounds the step; its longest
kernels and gaps are listed.

    python3 tools/trace_crit.py TRACE.csv [--last 5] [--top 15]
"""
import argparse
import csv
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("mragan::", "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=5)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--min-step-us", type=float, default=2000.0)
    a = ap.parse_args()
    ks = []
    for r in csv.DictReader(open(a.trace)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], short(r["Kernel_Name"])))
    ks.sort()
    # split at all-idle instants
    steps, cur, end = [], [], None
    for k in ks:
        if cur and k[0] > end:
            steps.append(cur)
            cur, end = [], None
        cur.append(k)
        end = k[1] if end is None else max(end, k[1])
    if cur:
        steps.append(cur)
    steps = [s for s in steps if (max(k[1] for k in s) - s[0][0]) / 1e3 >= a.min_step_us]
    print(f"{len(steps)} steps of >= {a.min_step_us} us; showing the last {a.last}")
    for si, s in enumerate(steps[-a.last:]):
        t0 = s[0][0]
        t1 = max(k[1] for k in s)
        byq = defaultdict(list)
        for k in s:
            byq[k[2]].append(k)
        print(f"\nstep {si}: wall {(t1 - t0) / 1e3:.1f} us, {len(s)} kernels")
        crit = max(byq, key=lambda q: max(k[1] for k in byq[q]))
        for q, v in sorted(byq.items()):
            busy = sum(k[1] - k[0] for k in v)
            first, last = v[0][0] - t0, max(k[1] for k in v) - t0
            gaps, e = [], v[0][1]
            for k in v[1:]:
                if k[0] > e:
                    gaps.append((k[0] - e, k[0] - t0, k[3]))
                e = max(e, k[1])
            gsum = sum(g[0] for g in gaps)
            mark = " <- ends last" if q == crit else ""
            print(f"  queue {q}: {len(v):4d} kernels, busy {busy / 1e3:8.1f} us, span {first / 1e3:7.1f} .. {last / 1e3:8.1f} us,"
                  f" gaps {gsum / 1e3:7.1f} us ({len(gaps)}){mark}")
        if si == min(a.last, len(steps)) - 1:
            v = byq[crit]
            gaps, e = [], v[0][1]
            for k in v[1:]:
                if k[0] > e:
                    gaps.append((k[0] - e, k[0] - t0, k[3]))
                e = max(e, k[1])
            print(f"\n  queue {crit}: largest gaps (waits) — us, at us, next kernel")
            for g in sorted(gaps, reverse=True)[:a.top]:
                print(f"    {g[0] / 1e3:7.1f}  @{g[1] / 1e3:8.1f}  {g[2]}")
            agg = defaultdict(lambda: [0, 0])
            for k in v:
                agg[k[3]][0] += k[1] - k[0]
                agg[k[3]][1] += 1
            print(f"  queue {crit}: kernel time by name")
            for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:a.top]:
                print(f"    {t / 1e3:8.1f} us  {c:4d}x  {n}")


if __name__ == "__main__":
    main()
