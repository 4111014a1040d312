#!/usr/bin/env python3
"""Host report stage at a bench workload: after one device-resident analysis,
times nmg_report with and without the per-call-site page files
(dump_single_items 1 / 0), and the number of files written.

    python tools/report_timing.py [--workload c4] [--reps 2]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--dir", default=None, help="output directory parent (default: a temporary directory)")
    a = ap.parse_args()
    import torch

    from bench import WORKLOADS
    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    cfg = {k: v for k, v in WORKLOADS[a.workload].items() if k != "desc"}
    rp = generate(SynthConfig(seed=1, sample_seed=1000, **cfg))
    arena, offs, lens, ranks, acc = rp.packed()
    d = torch.from_numpy(arena).cuda()
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
    eng.reset()
    eng.analyze()
    eng.synchronize()
    for single in (1, 0):
        ts, nfiles = [], 0
        for _ in range(a.reps):
            with tempfile.TemporaryDirectory(dir=a.dir) as tmp:
                out = os.path.join(tmp, "out")
                t0 = time.perf_counter()
                eng.report(out, os.path.join(tmp, "stdout.txt"), dump_single_items=single)
                ts.append(time.perf_counter() - t0)
                nfiles = len(os.listdir(out))
        print(json.dumps({"workload": a.workload, "dump_single_items": single, "report_s": min(ts),
                          "files": nfiles, "entries": rp.table.nb_entries}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
