#!/usr/bin/env python3
"""End-to-end rate of the drop-in path with host-resident buffers, as the
reference's C host would drive it, next to the device-resident
kernel time.  Buffers start in pageable host memory (the malloc'd
__copy_buffer copies of the `samples` list, mem_sampling.c:696); the results
come back D2H (global counters, per-buffer counts, object counters, page cells:
everything nmg_report reads).  Modes (one JSON line each):

  per_buffer  nmg_submit_buffer per buffer (a ctypes call each), then
              nmg_analyze: pinned staging copy, H2D, kernel, serialised
  batch       one nmg_submit_buffers call, copies split over T host threads,
              then nmg_analyze (H2D + kernel)
  stream      nmg_stream_begin(chunk, T) and nmg_submit_buffers in alarm-sized
              batches: each chunk's H2D (copy stream) and kernel (engine
              stream) overlap the copies of the next chunk (configs[4])
  zerocopy    the buffers live in one host arena registered once with
              nmg_register_host (like perf rings pinned at thread start; the
              registration is timed apart, register_s): one nmg_submit_buffers
              call copies nothing, the kernels read the arena over PCIe
  zerocopy_pipe  zerocopy analyses back to back, each one's results taken with
              nmg_results_begin / nmg_results_end: its copy to host memory
              runs while the next analysis reads its records over PCIe;
              e2e_s = the median interval between consecutive results

    python tools/e2e.py [c2|c4shard] [--threads 16] [--chunk-mb 64] [--batch 256]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", nargs="?", default="c2")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--chunk-mb", type=int, default=64)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--modes", default="per_buffer,batch,stream")
    ap.add_argument("--report", action="store_true", help="time nmg_report (counters D2H + report files) "
                    "instead of the raw result getters")
    a = ap.parse_args()

    from numamma_amd.engine import Engine
    from numamma_amd.replay import CONFIGS, SynthConfig, generate

    # c4shard: configs[3]'s per-GPU shard (bench.py's default workload)
    cfgs = dict(CONFIGS, c4shard=SynthConfig(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024))
    rp = generate(cfgs[a.workload])
    lins = rp.linear_buffers()
    nbytes = sum(x[2].shape[0] for x in lins)
    nsamples = nbytes // 40
    eng = Engine(nb_threads=rp.nb_threads, copy_threads=a.threads)
    eng.set_objects(rp.table)

    split = {}

    def results():  # D2H of everything the report reads (each getter timed: split)
        for name, f in (("global", eng.global_counters), ("buffers", eng.buffer_counts),
                        ("objects", eng.object_counters), ("page_cells", eng.page_cells)):
            t = time.perf_counter()
            f()
            split.setdefault(name, []).append(time.perf_counter() - t)

    zc_views, reg_s = None, None
    for mode in a.modes.split(","):
        if mode in ("zerocopy", "zerocopy_pipe") and zc_views is None:
            offs, o = [], 0
            for _, _, b in lins:
                offs.append(o)
                o = (o + b.shape[0] + 15) // 16 * 16
            from numamma_amd.engine import page_aligned_empty

            arena = page_aligned_empty(o + 64)
            base = 0
            for (_, _, b), off in zip(lins, offs):
                arena[base + off:base + off + b.shape[0]] = b
            zc_views = (arena, np.array(offs, dtype=np.uint64) + base,
                        np.array([b.shape[0] for _, _, b in lins], dtype=np.uint64),
                        np.array([r for r, _, _ in lins], dtype=np.uint32),
                        np.array([acc for _, acc, _ in lins], dtype=np.uint32))
            t = time.perf_counter()
            eng.register_host(arena)
            reg_s = time.perf_counter() - t
        if mode == "zerocopy_pipe":
            ends, cells = [], 0
            eng.synchronize()
            t_start = time.perf_counter()
            calls = {}
            for r in range(a.reps + 2):
                tc = [time.perf_counter()]
                eng.clear_buffers()
                tc.append(time.perf_counter())
                eng.reset()
                tc.append(time.perf_counter())
                eng.submit_arena(*zc_views)
                tc.append(time.perf_counter())
                eng.analyze()
                tc.append(time.perf_counter())
                if r:
                    res = eng.results_end()
                    cells = res[7].shape[0]
                    ends.append(time.perf_counter())
                tc.append(time.perf_counter())
                eng.results_begin()
                tc.append(time.perf_counter())
                for k, name in enumerate(("clear", "reset", "submit", "analyze", "end", "begin")):
                    calls.setdefault(name, []).append(tc[k + 1] - tc[k])
            res = eng.results_end()
            ends.append(time.perf_counter())
            iv = np.diff(np.array(ends))
            e2e = float(np.median(iv))
            print(json.dumps({
                "workload": a.workload, "mode": mode, "records": int(nsamples), "bytes": int(nbytes),
                "copy_threads": 0, "analyses": a.reps + 2, "intervals_s": iv.tolist(), "e2e_s": e2e,
                "e2e_samples_per_s": nsamples / e2e, "total_s": ends[-1] - t_start,
                "total_samples_per_s": (a.reps + 2) * nsamples / (ends[-1] - t_start), "cells": int(cells),
                "register_s": reg_s, "host_call_s": {k: float(np.median(v[1:])) for k, v in calls.items()},
                "note": "steady state: each interval is one analysis (PCIe read of the records) with the previous "
                        "analysis' results copied to pinned host memory meanwhile (counters, per-buffer counts, "
                        "object counters, page-cell rows)"}), flush=True)
            continue
        reps = []
        for r in range(a.reps + 1):
            eng.clear_buffers()
            eng.reset()
            eng.synchronize()
            t0 = time.perf_counter()
            if mode == "per_buffer":
                for rank, acc, data in lins:
                    eng.submit_buffer(data, rank, acc)
            elif mode == "batch":
                eng.submit_buffers(lins)
            elif mode == "zerocopy":
                eng.submit_arena(*zc_views)  # (pointers computed in numpy: no per-buffer list)
            else:
                eng.stream_begin(chunk_bytes=a.chunk_mb << 20, copy_threads=a.threads)
                for i in range(0, len(lins), a.batch):
                    eng.submit_buffers(lins[i:i + a.batch])
            t1 = time.perf_counter()
            if mode == "stream":
                eng.stream_end()  # (flushes the last chunk; the engine leaves streaming mode)
            eng.analyze()
            eng.synchronize()
            t2 = time.perf_counter()
            if a.report:  # the product's output stage: D2H of the counters + report files
                with tempfile.TemporaryDirectory() as d:
                    eng.report(os.path.join(d, "out"), os.path.join(d, "stdout.txt"))
            else:
                results()
            t3 = time.perf_counter()
            kern = float(np.sum(eng.launch_times(64 if mode == "stream" else 1))) / 1e3
            if r:
                reps.append((t1 - t0, t2 - t1, t3 - t2, kern))
        submit, tail, d2h, kern = np.median(np.array(reps), axis=0)
        total = submit + tail + d2h
        print(json.dumps({
            "workload": a.workload, "mode": mode, "records": int(nsamples), "bytes": int(nbytes),
            "copy_threads": a.threads if mode in ("batch", "stream") else (0 if mode == "zerocopy" else 1),
            "chunk_bytes": (a.chunk_mb << 20) if mode == "stream" else None,
            "submit_s": submit, "analyze_to_sync_s": tail,
            ("report_s" if a.report else "d2h_results_s"): d2h, "kernel_s": kern,
            "e2e_s": total, "e2e_samples_per_s": nsamples / total,
            "device_resident_samples_per_s": nsamples / kern if kern else None,
            "d2h_split_s": {k: float(np.median(v[1:] if len(v) > 1 else v)) for k, v in split.items()},
            **({"register_s": reg_s} if mode == "zerocopy" else {}),
        }), flush=True)
        split.clear()
    eng.close()


if __name__ == "__main__":
    main()
