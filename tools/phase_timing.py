#!/usr/bin/env python3
"""Where a window's time goes: run nmg::attribute_kernel's timing variant
(internal flag 0x1000; s_memtime stamps at the phase edges of the window loop)
and print, per workload and variant, the mean shader cycles per wave per
window of each phase:

  load_check  waiting for the window's records + decode + fast-path check
  barrier     the per-window barrier (slowest wave of the workgroup)
  process     next-window issue + the records' lookup and accumulation
  rest        drain / buffer end / stream flush bookkeeping

and the process phase split (sub_*): global counters, lookup (until the
node record has arrived), object tables, page cells, levels, the next
window's speculative fence walk + directory issue, tallies.

The stamps themselves cost a few percent (MI355X_MICROARCH.md constants
table); compare variants with each other, not with the untimed kernel."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NMG_INTERNAL_FLAGS", "1")  # (internal ablation / timing switches)
sys.path.insert(0, ROOT)

TIMING = 0x1000
VARIANTS = {"load_only": 0x100, "lookup_only": 0x1 | 0x200 | 0x800, "match": 0x1, "full": 0x3}
WORKLOADS = {
    "c2": dict(nb_samples=10_000_000, nb_intervals=1_000),
    "k100k": dict(nb_samples=10_000_000, nb_intervals=100_000),
    "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
    "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
    "c4hot": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024, zipf_s=2.0, frac_gap=0.0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,k100k")
    ap.add_argument("--reps", type=int, default=5)
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
        for v, f in VARIANTS.items():
            e = Engine(flags=f | TIMING, nb_threads=rp.nb_threads)
            e.set_objects(rp.table)
            e.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
            res = []
            for r in range(args.reps + 1):
                e.reset()
                e.analyze()
                e.synchronize()
                n = C.c_size_t(0)
                lib.nmg_debug_timing(e.h, None, 0, C.byref(n))
                buf = np.zeros(n.value, dtype=np.uint64)
                lib.nmg_debug_timing(e.h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), n.value, C.byref(n))
                if r:
                    res.append((buf.reshape(-1, 24).astype(np.float64), e.last_analyze_ms()))
            t = np.mean([x[0] for x in res], axis=0)  # [waves][8]
            wins = t[:, 5].sum()
            out = {"workload": wname, "variant": v, "kernel_ms": float(np.median([x[1] for x in res])),
                   "windows_per_wave": float(t[:, 5].mean())}
            for k, name in enumerate(("load_check", "barrier", "process", "rest")):
                out[name + "_cyc_per_window"] = float(t[:, k].sum() / wins)
            for k, name in enumerate(("glob", "find", "obj", "page", "levels", "spec", "tail")):
                out["sub_" + name] = float(t[:, 16 + k].sum() / wins)
            out["total_cyc_per_wave"] = float(t[:, 4].mean())
            out["max_total_cyc"] = float(t[:, 4].max())
            print(json.dumps(out), flush=True)
            e.close()
        del d


if __name__ == "__main__":
    main()
