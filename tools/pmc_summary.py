#!/usr/bin/env python3
"""Per-kernel PMC summary (tools/pmc_probe.sh passes p1..p4): counters averaged per dispatch (the
first dispatch of each kernel dropped), per-MFMA instruction mix, wave-cycle split (parked =
SQ_WAIT_ANY, issue-stall = SQ_WAIT_INST_ANY, issuing = SQ_ACTIVE_INST_ANY; quad-cycle units, the
ratios are unit-free), HBM bytes (2·FETCH_SIZE + WRITE_SIZE, gfx950 correction).

    python3 tools/pmc_summary.py gpurun_out/TAG [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
want = sys.argv[2:]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if k.startswith("void at::") or "rocclr" in k:
            continue
        per[(k, int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    byk = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, d, c), v in per.items():
        byk[k][c].append((d, v))
    for k, cs in byk.items():
        for c, lst in cs.items():
            lst.sort()
            use = lst[1:] if len(lst) > 1 else lst
            vals[k][c].extend(v for _, v in use)
for k, cs in sorted(vals.items()):
    if want and not any(w in k for w in want):
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k[:90])
    print("   ", " ".join(f"{c}={m[c]:.4g}" for c in sorted(m)))
    mf = m.get("SQ_INSTS_MFMA")
    if mf:
        print("    per MFMA: " + " ".join(f"{n} {m[c] / mf:.2f}" for n, c in
                                          (("VALU", "SQ_INSTS_VALU"), ("SALU", "SQ_INSTS_SALU"), ("LDS", "SQ_INSTS_LDS"),
                                           ("VMEM", "SQ_INSTS_VMEM_RD")) if c in m))
    if "SQ_WAVE_CYCLES" in m:
        w = m["SQ_WAVE_CYCLES"]
        parts = [(n, m[c] / w) for n, c in (("parked", "SQ_WAIT_ANY"), ("issue-stall", "SQ_WAIT_INST_ANY"),
                                               ("issuing", "SQ_ACTIVE_INST_ANY")) if c in m]
        print("    wave cycles: " + " ".join(f"{n} {x:.2f}" for n, x in parts))
    if "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
        print(f"    LDS conflict cycles / LDS active: {m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        pass
    if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
        print(f"    HBM MB/launch: {(2 * m.get('FETCH_SIZE', 0) + m.get('WRITE_SIZE', 0)) * 1024 / 1e6:.1f}")
