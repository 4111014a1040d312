#!/usr/bin/env python3
"""Where the local pass's time goes (partition-first path, nmg_route.h): run
local_kernel's timing variant (internal flag kDbgLocalTiming = 0x10000000;
s_memtime stamps at the phase edges) and print, per workload, the mean
shader cycles per wave:

  wait     per chunk: waiting for its records (+ loop overhead)
  global   per chunk: update_counters (per-lane accumulators, LDS min/max)
  search   per chunk: directory slot + binary search among the partition's keys
  match    per chunk: node record, dates, older entries, match-bit word
  object   per chunk: packed object counters + first-match ordinal
  page     per chunk: page cells
  dequeue  per item: next work item (+ barrier)
  setup    per item: partition table into LDS, counters cleared (+ barrier)
  flush    per item: waiting for the item's slowest wave, counters to global memory

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

TIMING = 0x10000000
WORDS = 16
PHASES = ["wait", "global", "search", "match", "object", "page", "dequeue", "setup", "flush"]
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
        a = a[a[:, 10] > 0]
        ch, it = a[:, 9].sum(), a[:, 10].sum()
        out = {"workload": wname, "flags": hex(args.flags), "analyze_ms": float(np.median(ms)),
               "chunks_per_wave": float(a[:, 9].mean()), "items_per_wave": float(a[:, 10].mean())}
        for k, name in enumerate(PHASES):
            per = ch if k < 6 else it
            out[f"{name}_cyc_per_{'chunk' if k < 6 else 'item'}"] = float(a[:, k].sum() / per)
        out["imbalance_cyc_per_item"] = float(a[:, 11].sum() / it)  # waiting for the item's slowest wave
        recs = ch * 64
        out["exact_node_frac"] = float(a[:, 12].sum() / recs)  # decided on the exact node record (global)
        out["key_search_frac"] = float(a[:, 13].sum() / recs)  # lookups that read keys past the directory
        out["total_cyc_per_wave"] = float((a[:, :9].sum(axis=1) + a[:, 11]).mean())
        out["max_total_cyc_per_wave"] = float((a[:, :9].sum(axis=1) + a[:, 11]).max())
        print(json.dumps(out), flush=True)
        e.close()
        del d


if __name__ == "__main__":
    main()
