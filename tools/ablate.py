#!/usr/bin/env python3
"""Kernel ablation on the GPU: time nmg::attribute_kernel with parts of its
work switched off, interleaved in one process (cdna_hip_programming.md
§5.4 rule 24).  Prints one JSON line per (workload, variant)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NMG_INTERNAL_FLAGS", "1")  # (internal ablation / timing switches)
sys.path.insert(0, ROOT)

VARIANTS = {
    "load_only": 0x100,
    "decode_global": 0x0,               # decode + global mem_counters, no matching
    "lookup_only": 0x1 | 0x200 | 0x800,  # decode + lookup, nothing accumulated
    "match_no_global": 0x1 | 0x200,     # lookup + object counters only
    "match": 0x1,                       # + object counters
    "full_noflush": 0x3 | 0x400,        # LDS tables filled, never flushed to global
    "full": 0x3,                        # + page histogram (default product path)
    # large tables: the partition-first path (nmg_route.h) and its parts
    "legacy": 0x3 | 0x10000,            # attribute_kernel on a large table (kDbgNoRoute)
    "route": 0x3,                       # route2 + count + plan + scatter + local (default for > 1023 keys)
    "route_nolines": 0x3 | 0x20000000,  # ... without the route pass's LDS line stage (every record stored to its slot)
    "route_atomics": 0x3 | 0x80000000,  # every local-pass flush through atomics
    "route_nopages": 0x1,               # ... without the page histogram
    "route_noloc": 0x3 | 0x400000,      # local pass loads its chunks only
    "route_lapnowait": 0x3 | 0x100000,  # ... every partition's line given up at its first record ahead of the lap
    "local_noobj": 0x3 | 0x1000000,     # local pass without object counters / first ordinals
    "local_nopage": 0x3 | 0x2000000,    # ... without page cells
    "local_noglobal": 0x3 | 0x4000000,  # ... without the global counters
    "local_nosearch": 0x3 | 0x8000000,  # ... without the lookup (nothing matches)
}

WORKLOADS = {
    "c2": dict(nb_samples=10_000_000, nb_intervals=1_000),
    "k100k": dict(nb_samples=10_000_000, nb_intervals=100_000),
    "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
    "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
    "c3": dict(nb_samples=100_000_000, nb_intervals=100_000),
    # same table, samples concentrated on few objects (no gap samples): the
    # lookup's cost when every table line it touches is cache-hot
    "c4hot": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024, zipf_s=2.0, frac_gap=0.0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,k100k,k1m")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    args = ap.parse_args()
    import torch

    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    for wname in args.workloads.split(","):
        t0 = time.time()
        rp = generate(SynthConfig(seed=1, **WORKLOADS[wname]))
        arena, offs, lens, ranks, acc = rp.packed()
        d = torch.from_numpy(arena).cuda()
        nbytes = int(lens.sum())
        engines = {}
        for v in args.variants.split(","):
            f = VARIANTS[v]
            e = Engine(flags=f, nb_threads=rp.nb_threads)
            e.set_objects(rp.table)
            e.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
            engines[v] = e
        print(f"# {wname}: generated in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        times = {v: [] for v in engines}
        first = {v: [] for v in engines}
        for r in range(args.reps + 2):
            for v, e in engines.items():
                e.reset()
                e.analyze()
                e.synchronize()
                if r >= 2:
                    times[v].append(e.last_analyze_ms())
                    first[v].append(e.phase_times(1)[0][-1])
        for v, ts in times.items():
            med = float(np.median(ts))
            print(json.dumps({"workload": wname, "variant": v, "median_ms": med, "min_ms": float(np.min(ts)),
                              "first_kernel_ms": float(np.median(first[v])),
                              "GBps": nbytes / med / 1e6, "Gsamples_s": nbytes / 40 / med / 1e6}), flush=True)
        for e in engines.values():
            e.close()
        del d


if __name__ == "__main__":
    main()
