#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from rocprofv3 PMC passes (gfx950 recipe).

Two separate counter passes (TCC slots cannot hold both in one pass) over the same command:

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o run -- python3 tools/kbench.py --ops res_fwd
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o run -- python3 tools/kbench.py --ops res_fwd

then

    python3 tools/pmc_traffic.py --fetch OUT/fetch --write OUT/write --kernel conv_igemm \
        --key res_fwd:S64:N4:ngf32 --out profiles/traffic.json

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced stream, so
hbm_bytes = (2·FETCH_SIZE + WRITE_SIZE)·1024.  The first launch of each pass is dropped (cold
caches / code-object load).  The result is merged into a JSON map keyed by `--key`, which
bench.py reads for `roofline.traffic`.
"""
import argparse
import csv
import glob
import json
import os


def per_launch(root, counter, kernel):
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    vals = {}
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                    continue
                key = (f, row.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    v = [vals[k] for k in sorted(vals, key=lambda k: (k[0], int(k[1])))]
    if len(v) > 1:
        v = v[1:]
    if not v:
        raise SystemExit(f"no {counter} rows for kernel '{kernel}' under {root}")
    return sum(v) / len(v), len(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--algorithmic-bytes", type=float, default=None)
    ap.add_argument("--out", required=True)
    ap.add_argument("--source", default=None, help="what was profiled (recorded in the entry)")
    a = ap.parse_args()
    # a launch class may be several kernels (e.g. "wgrad3_x3_kernel;wgrad_reduce_kernel", ';'-separated:
    # template names hold commas): per-launch
    # averages of each, summed
    fetch_kib = write_kib = 0.0
    nf = nw = 0
    for k in a.kernel.split(";"):
        f, n1 = per_launch(a.fetch, "FETCH_SIZE", k)
        w, n2 = per_launch(a.write, "WRITE_SIZE", k)
        fetch_kib += f
        write_kib += w
        nf, nw = max(nf, n1), max(nw, n2)
    entry = {
        "kernel": a.kernel,
        "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
        "hbm_bytes_per_launch": (2.0 * fetch_kib + write_kib) * 1024.0,
        "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)",
        "launches": [nf, nw],
    }
    if a.source:
        entry["source"] = a.source
    if a.algorithmic_bytes:
        entry["algorithmic_bytes"] = a.algorithmic_bytes
        entry["ratio"] = entry["hbm_bytes_per_launch"] / a.algorithmic_bytes
    data = {}
    if os.path.exists(a.out):
        with open(a.out) as fh:
            data = json.load(fh)
    data[a.key] = entry
    with open(a.out, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps({a.key: entry}))


if __name__ == "__main__":
    main()
