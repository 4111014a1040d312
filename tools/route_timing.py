#!/usr/bin/env python3
"""Where the route pass's time goes (partition-first path, nmg_route.h): run
route_kernel's timing variant (internal flag 0x800000; s_memtime stamps at
the phase edges) and print, per workload, the mean shader cycles per wave:

  wait     per window: waiting for its records + fast-path check + barrier
  issue    per window: slow path, next-window loads issued
  global   per window: the global counters (update_counters)
  search   per window: partition search in the LDS tree
  rank     per window: batch rank (LDS atomic), X word, held records, tallies
  scan     per batch: barrier + exclusive scan of the partition counts
  alloc    per batch: chunk allocation + held records into LDS + barrier
  write    per batch: the sorted runs to their chunks + barrier
  state    per batch: open-chunk state update

The stamps cost a little themselves; compare phases with each other."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NMG_INTERNAL_FLAGS", "1")  # (internal ablation / timing switches)
sys.path.insert(0, ROOT)

TIMING = 0x800000
WORDS = 16
# route2_kernel: per wave window
PHASES_V2 = ["wait", "check_loads", "global", "search", "encode", "claim"]
WORKLOADS = {
    "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
    "c3": dict(nb_samples=100_000_000, nb_intervals=100_000),
    "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c4")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--flags", type=lambda x: int(x, 0), default=0x3)
    args = ap.parse_args()
    import torch

    from numamma_amd._lib import lib
    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    lib.nmg_debug_timing.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_size_t)]
    lib.nmg_debug_timing.restype = C.c_int
    for wname in args.workloads.split(","):
        rp = generate(SynthConfig(seed=1, **WORKLOADS[wname]))
        arena, offs, lens, ranks, acc = rp.packed()
        d = torch.from_numpy(arena).cuda()
        e = Engine(flags=args.flags | TIMING, nb_threads=rp.nb_threads)
        e.set_objects(rp.table)
        e.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
        ms = []
        for _ in range(args.reps):
            e.reset()
            e.analyze()
            e.synchronize()
            ms.append(e.last_analyze_ms())
        n = C.c_size_t(0)
        lib.nmg_debug_timing(e.h, None, 0, C.byref(n))
        buf = (C.c_uint64 * n.value)()
        lib.nmg_debug_timing(e.h, buf, n.value, C.byref(n))
        a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, WORDS).astype(np.float64)
        a = a[a[:, 9] > 0]
        win, bat = a[:, 9].sum(), a[:, 10].sum()
        out = {"workload": wname, "flags": hex(args.flags), "analyze_ms": float(np.median(ms)),
               "windows_per_wave": float(a[:, 9].mean()), "batches_per_wave": float(a[:, 10].mean())}
        for k, name in enumerate(PHASES_V2):
            out[f"{name}_cyc_per_window"] = float(a[:, k].sum() / win)
        out["line_stage_cyc_per_window"] = float(a[:, 11].sum() / win)
        out["store_cyc_per_window"] = float(a[:, 12].sum() / win)
        # the line stage: records staged / stored straight to their slot, records
        # that re-read the lap, partitions given up per workgroup
        tot = a[:, 6].sum() + a[:, 7].sum() + a[:, 8].sum()
        out["staged_frac"] = float(a[:, 6].sum() / tot) if tot else 0.0
        out["counted_direct_frac"] = float(a[:, 8].sum() / tot) if tot else 0.0  # (staged_frac: staged; rest: given up)
        out["broken_parts_per_wg"] = float(a[:, 10].sum() / max(1.0, a.shape[0] / 12))
        out["total_cyc_per_wave"] = float((a[:, :6].sum(axis=1) + a[:, 11] + a[:, 12]).mean())
        print(json.dumps(out), flush=True)
        e.close()
        del d


if __name__ == "__main__":
    main()
