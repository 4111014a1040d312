#!/usr/bin/env python3
"""Per-step cost of the multi-GPU counter merge at 1M intervals, on one GPU.

1. The one-process-per-GPU path (numamma_amd/distributed.py): an engine holds
   the configs[3]-shard counters (125M records, 1M intervals, page histogram
   on); time nmg_export_array of every dense array into device tensors, the
   element-wise reduction a 2-rank RCCL reduce performs on the root (sum,
   and min / max through the x ^ 2^63 order map), and nmg_import_array.  The
   bytes are what RCCL moves per rank and step.
2. The in-process path (nmg_options.nb_gpus): nb_gpus = 2 workers on device
   0 (merge_kernel instead of RCCL, which needs distinct devices) against
   nb_gpus = 1, host-staged buffers, nmg_analyze + nmg_synchronize per step.

Prints one JSON line per measurement."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NMG_INTERNAL_FLAGS", "1")  # (internal switches: one-rank RCCL branch)
sys.path.insert(0, ROOT)

WORKLOADS = {
    "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
    "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--skip-multi", action="store_true")
    args = ap.parse_args()
    import torch

    from numamma_amd import _lib
    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    rp = generate(SynthConfig(seed=1, **WORKLOADS[args.workload]))
    arena, offs, lens, ranks, acc = rp.packed()
    dev = torch.device("cuda", 0)
    d_arena = torch.from_numpy(arena).to(dev)
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.set_device_buffers(d_arena.data_ptr(), offs, lens, ranks, acc)
    eng.analyze()
    eng.synchronize()
    arrays = []
    for which, dt in ((_lib.NMG_ARR_SUM64, torch.int64), (_lib.NMG_ARR_MIN64, torch.int64),
                      (_lib.NMG_ARR_MAX64, torch.int64), (_lib.NMG_ARR_HIST32, torch.int32)):
        n = eng.array_size(which)
        if n:
            arrays.append((which, torch.empty(n, dtype=dt, device=dev), torch.empty(n, dtype=dt, device=dev)))
    nbytes = sum(a.numel() * a.element_size() for _, a, _ in arrays)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t_exp, t_red, t_imp = [], [], []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        ev[0].record()
        for which, a, _ in arrays:
            eng.export_array(which, a.data_ptr())
        eng.synchronize()  # the exports run on the engine stream
        ev[1].record()
        for which, a, b in arrays:  # the root's side of a 2-rank reduce: combine with a peer's copy
            b.copy_(a)
            if which in (_lib.NMG_ARR_MIN64, _lib.NMG_ARR_MAX64):
                a.bitwise_xor_(-(1 << 63))
                b.bitwise_xor_(-(1 << 63))
                torch.minimum(a, b, out=a) if which == _lib.NMG_ARR_MIN64 else torch.maximum(a, b, out=a)
                a.bitwise_xor_(-(1 << 63))
            else:
                a.add_(b)
        ev[2].record()
        torch.cuda.synchronize()
        for which, a, _ in arrays:
            eng.import_array(which, a.data_ptr())
        eng.synchronize()
        ev[3].record()
        torch.cuda.synchronize()
        t_exp.append(ev[0].elapsed_time(ev[1]))
        t_red.append(ev[1].elapsed_time(ev[2]))
        t_imp.append(ev[2].elapsed_time(ev[3]))
    print(json.dumps({"measure": "rank_merge_one_gpu", "workload": args.workload, "bytes_per_rank": nbytes,
                      "arrays": {str(w): a.numel() * a.element_size() for w, a, _ in arrays},
                      "export_ms": float(np.median(t_exp)), "reduce_2way_ms": float(np.median(t_red)),
                      "import_ms": float(np.median(t_imp)), "attribute_step_ms": eng.last_analyze_ms()}),
          flush=True)
    # the packed page histogram of the one-process-per-GPU merge (distributed.HistPacker):
    # cells <= 255 // world as bytes (u8 reduce), the rest as (cell, count) words (gather)
    cells = eng.array_size(_lib.NMG_ARR_HIST32)
    # (the reduce loop above doubled the counters at every repetition: one
    # fresh analysis for the packed form)
    eng.reset()
    eng.analyze()
    eng.synchronize()
    if cells:
        u8 = torch.empty(cells, dtype=torch.uint8, device=dev)
        cap = max(1024, cells // 8)
        ovf = torch.zeros(cap, dtype=torch.int64, device=dev)
        for world in (2, 8):
            thr = 255 // world
            tp, tu = [], []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                n = eng.hist_pack(thr, u8.data_ptr(), ovf.data_ptr(), cap)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                if n <= cap:  # (a longer list: the u32 reduce instead)
                    eng.hist_unpack(u8.data_ptr(), ovf.data_ptr(), n)
                eng.synchronize()
                t2 = time.perf_counter()
                tp.append((t1 - t0) * 1e3)
                tu.append((t2 - t1) * 1e3)
            dense = sum(a.numel() * a.element_size() for w, a, _ in arrays if w != _lib.NMG_ARR_HIST32)
            print(json.dumps({"measure": "hist_packed", "workload": args.workload, "world": world, "cells": cells,
                              "hist_u32_bytes": cells * 4, "overflow_cells": n, "packed_bytes": cells + 8 * n,
                              "bytes_per_rank_packed": dense + cells + 8 * n, "pack_ms": float(np.median(tp)),
                              "unpack_ms": float(np.median(tu))}), flush=True)
    eng.close()
    del d_arena
    if args.skip_multi:
        return
    lins = rp.linear_buffers()
    for devices, flags, tag in ((None, 0, "single"), ([0, 0], 0, "two_shards_one_device"),
                                (None, 0x40000, "one_rank_rccl_handle")):
        e = Engine(nb_threads=rp.nb_threads, devices=devices, copy_threads=8, flags=_lib.NMG_F_DEFAULT | flags)
        e.set_objects(rp.table)
        e.submit_buffers(lins)
        ts = []
        for r in range(args.reps // 2 + 1):
            t0 = time.perf_counter()
            e.reset()
            e.analyze()
            e.synchronize()
            if r:
                ts.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"measure": "abi_multi_gpu_step", "workload": args.workload, "handle": tag,
                          "nb_gpus": len(devices) if devices else 1, "same_device": bool(devices),
                          "reset_analyze_sync_ms": float(np.median(ts)),
                          "analysis_launch_ms": e.last_analyze_ms() if not (devices or flags) else None}), flush=True)
        e.close()


if __name__ == "__main__":
    main()
