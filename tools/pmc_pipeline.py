#!/usr/bin/env python3
"""HBM bytes per attribution launch, per kernel, from two rocprofv3 passes
(FETCH_SIZE alone, WRITE_SIZE alone: MI355X_MICROARCH.md, HBM/rocprofv3), for
bench.py's roofline.traffic.

    python tools/pmc_pipeline.py --workload c4 --fetch DIR --write DIR [--out FILE]

FETCH_SIZE and WRITE_SIZE are KiB per dispatch.  gfx950 tallies a wide
coalesced streaming read at half its bytes; the record streams (route_kernel:
the 40 B records; local_kernel: the 24 B compact records; attribute_kernel:
the 40 B records) are such reads, so their kernels' FETCH_SIZE is doubled
(an upper bound for their small table loads); the other kernels' reads are
taken as counted.  The output carries the kernel-source hash
(numamma_amd/srchash.py) of the tree the passes ran from."""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PIPELINE = ("route2_kernel", "route_kernel", "overflow_kernel", "count_kernel", "plan_kernel", "scatter_kernel", "local_kernel",
            "attribute_kernel", "reduce")
STREAMING = ("route2_kernel", "route_kernel", "local_kernel", "attribute_kernel")


def per_kernel(d):
    """kernel short name -> (sum of counter values, number of dispatches)."""
    val = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
                name = name.split("::")[-1]
                val[name] += float(r["Counter_Value"])
                disp[name].add((f, r["Dispatch_Id"]))
    return {k: (val[k], len(disp[k])) for k in val}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out")
    args = ap.parse_args()
    from numamma_amd.srchash import kernel_source_hash

    fetch, write = per_kernel(args.fetch), per_kernel(args.write)
    first = next(k for k in ("route2_kernel", "route_kernel", "attribute_kernel") if k in fetch)
    launches = fetch[first][1]
    wlaunches = write[first][1]
    kernels = {}
    total = 0.0
    for k in sorted(set(fetch) | set(write)):
        if not any(k.startswith(p) or k == p for p in PIPELINE):
            continue
        f_kib, f_n = fetch.get(k, (0.0, 1))
        w_kib, w_n = write.get(k, (0.0, 1))
        scale = 2.0 if k in STREAMING else 1.0
        rd = f_kib * 1024 * scale / launches  # per launch (a kernel may run several times per launch)
        wr = w_kib * 1024 / wlaunches
        kernels[k] = {"FETCH_SIZE_KiB_per_dispatch": f_kib / max(1, f_n),
                      "WRITE_SIZE_KiB_per_dispatch": w_kib / max(1, w_n),
                      "dispatches_per_launch": f_n / launches, "fetch_x2": scale == 2.0,
                      "hbm_read_bytes": rd, "hbm_write_bytes": wr}
        total += rd + wr
    out = {"workload": args.workload, "source_hash": kernel_source_hash(), "launches": launches,
           "kernels": kernels, "hbm_bytes_per_launch": total,
           "note": "bytes per attribution launch; FETCH_SIZE x2 for the streaming kernels (gfx950 under-count)"}
    s = json.dumps(out, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
