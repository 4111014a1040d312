#!/usr/bin/env python3
"""Device-resident analysis time of an online (--online-analysis) table at 1M
intervals: the configs[3] shard's records analysed against its table given
through nmg_update_objects with ids in creation order (a live host's ids,
mem_analyzer.c:567-568; page cells laid out in id order), on the
partition-first path (its partitions map table positions to ids) and on the
single-pass attribute_kernel (internal switch 0x10000), beside the offline
table (nmg_set_objects).  One JSON line per mode: ms per reset + analyze +
synchronize, the attribution launch's kernel time, Gsamples/s."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NMG_INTERNAL_FLAGS", "1")  # (internal switch: the single-pass kernel)
sys.path.insert(0, ROOT)

WORKLOADS = {
    "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
    "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
}
NO_ROUTE = 0x10000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    from numamma_amd import _lib
    from numamma_amd.engine import Engine, table_objects
    from numamma_amd.replay import ObjectTable, SynthConfig, generate

    rp = generate(SynthConfig(seed=1, sample_seed=1000, **WORKLOADS[args.workload]))
    arena, offs, lens, ranks, acc = rp.packed()
    samples = int(lens.sum()) // 40
    dev = torch.device("cuda", 0)
    d_arena = torch.from_numpy(arena).to(dev)
    del arena
    t = rp.table
    ent = t.entries
    order = np.lexsort((np.arange(t.nb_entries), ent["alloc_date"]))
    cid = np.empty(t.nb_entries, dtype=np.uint32)
    cid[order] = np.arange(t.nb_entries, dtype=np.uint32)
    ref = None
    for mode, flags, online in (("offline", 0, False), ("online_route", 0, True),
                                ("online_single_pass", NO_ROUTE, True)):
        eng = Engine(device=0, flags=_lib.NMG_F_DEFAULT | flags, nb_threads=rp.nb_threads)
        if online:
            eng.set_objects(ObjectTable.empty())
            eng.update_objects(t.keys, t.entry_off, cid, table_objects(t))
        else:
            eng.set_objects(t)
        eng.set_device_buffers(d_arena.data_ptr(), offs, lens, ranks, acc)
        for _ in range(2):
            eng.reset()
            eng.analyze()
        eng.synchronize()
        r0 = eng.route_count()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            eng.reset()
            eng.analyze()
        eng.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.reps
        attr, _ = eng.kernel_times(args.reps)
        _, cw = eng.object_counters()
        g, ns, nf = eng.global_counters()
        cw = cw[cid] if online else cw  # (by table position)
        res = (g, nf, cw)
        same = None
        if ref is None:
            ref = res
        else:
            same = bool(all(np.array_equal(np.asarray(a), np.asarray(b)) for a, b in zip(ref, res)))
        print(json.dumps({"workload": args.workload, "mode": mode, "samples": samples,
                          "ms_per_step": round(ms, 4), "attr_kernel_ms": round(float(np.mean(attr)), 4),
                          "gsamples_per_s": round(samples / ms / 1e6, 2),
                          "route_launches": eng.route_count() - r0, "same_counters_as_offline": same}),
              flush=True)
        eng.close()


if __name__ == "__main__":
    main()
