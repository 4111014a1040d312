#!/usr/bin/env python3
"""Experiment: does the record arena's allocation type change how the object
table stays cached?  The same synthetic batch is copied into arenas allocated
with hipExtMallocWithFlags (default / fine-grained / uncached) and analysed by
engines with parts of the work switched off (tools/ablate.py's variants), all
interleaved in one process.  One JSON line per (arena, variant)."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NMG_INTERNAL_FLAGS", "1")  # (internal ablation / timing switches)
sys.path.insert(0, ROOT)

VARIANTS = {"load_only": 0x100, "lookup_only": 0x1 | 0x200 | 0x800, "full": 0x3}
ARENAS = {"default": 0x0, "finegrained": 0x1, "uncached": 0x3}
WORKLOADS = {
    "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
    "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    import torch  # noqa: F401  (initialises the runtime the engine shares)

    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    hip = C.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    t0 = time.time()
    rp = generate(SynthConfig(seed=1, **WORKLOADS[args.workload]))
    arena, offs, lens, ranks, acc = rp.packed()
    print(f"# generated {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    nbytes = int(lens.sum())
    ptrs = {}
    for name, fl in ARENAS.items():
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), arena.nbytes, fl)
        if rc != 0:
            print(f"# {name}: hipExtMallocWithFlags rc={rc}", file=sys.stderr, flush=True)
            continue
        rc = hip.hipMemcpy(p, arena.ctypes.data, arena.nbytes, 1)  # hipMemcpyHostToDevice
        if rc != 0:
            print(f"# {name}: hipMemcpy rc={rc}", file=sys.stderr, flush=True)
            continue
        ptrs[name] = p.value
    engines = {}
    for an, ptr in ptrs.items():
        for v, f in VARIANTS.items():
            e = Engine(flags=f, nb_threads=rp.nb_threads)
            e.set_objects(rp.table)
            e.set_device_buffers(ptr, offs, lens, ranks, acc)
            engines[(an, v)] = e
    times = {k: [] for k in engines}
    for r in range(args.reps + 2):
        for k, e in engines.items():
            e.reset()
            e.analyze()
            e.synchronize()
            if r >= 2:
                times[k].append(e.last_analyze_ms())
    for (an, v), ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"workload": args.workload, "arena": an, "variant": v, "median_ms": med,
                          "Gsamples_s": nbytes / 40 / med / 1e6}), flush=True)
    for e in engines.values():
        e.close()
    for p in ptrs.values():
        hip.hipFree(C.c_void_p(p))


if __name__ == "__main__":
    main()
