#!/usr/bin/env python3
"""Counter passes over engine variants in one process (rocprofv3 --pmc):

    rocprofv3 --pmc <counters> --kernel-trace -d DIR -o run --output-format csv \
        -- python3 tools/pmc_variants.py run --workload c4 --variants full,match --reps 3
    python3 tools/pmc_variants.py parse DIR [DIR ...] --variants full,match --reps 3

`run` analyses the same HBM-resident batch `reps` times per variant, the
variants one after the other; `parse` splits the attribution-kernel
dispatches of each pass in that order and prints per-variant averages (one
JSON line per variant, every counter of every pass)."""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NMG_INTERNAL_FLAGS", "1")  # (internal ablation / timing switches)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def run(args):
    import torch

    from ablate import VARIANTS, WORKLOADS
    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    rp = generate(SynthConfig(seed=1, **WORKLOADS[args.workload]))
    arena, offs, lens, ranks, acc = rp.packed()
    d = torch.from_numpy(arena).cuda()
    for v in args.variants.split(","):
        e = Engine(flags=VARIANTS[v], nb_threads=rp.nb_threads)
        e.set_objects(rp.table)
        e.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
        for _ in range(args.reps):
            e.reset()
            e.analyze()
            e.synchronize()
        print(json.dumps({"variant": v, "last_ms": e.last_analyze_ms()}), flush=True)
        e.close()


def parse(args):
    variants = args.variants.split(",")
    out = collections.defaultdict(dict)
    for d in args.dirs:
        rows = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if args.kernel not in r["Kernel_Name"]:
                    continue
                i = int(r["Dispatch_Id"])
                rows[i][r["Counter_Name"]] += float(r["Counter_Value"])
                names[i] = r["Kernel_Name"].split("(")[0]
        ids = sorted(rows)
        if len(ids) != len(variants) * args.reps:
            print(f"# {d}: {len(ids)} attribution dispatches, expected {len(variants) * args.reps}", file=sys.stderr)
            continue
        for j, v in enumerate(variants):
            grp = ids[j * args.reps:(j + 1) * args.reps]
            for c in rows[grp[0]]:
                out[v][c] = sum(rows[i][c] for i in grp) / len(grp)
            out[v]["kernel"] = names[grp[0]]
    for v in variants:
        print(json.dumps({"variant": v, **out[v]}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["run", "parse"])
    ap.add_argument("dirs", nargs="*")
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--variants", default="full,match")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--kernel", default="attribute_kernel", help="kernel-name substring of the dispatches to count")
    args = ap.parse_args()
    run(args) if args.cmd == "run" else parse(args)


if __name__ == "__main__":
    main()
