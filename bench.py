#!/usr/bin/env python3
"""Benchmark: PEBS samples/s analysed (device-resident) on 1..8 MI355X.

One step = one full analysis pass over one batch of synthetic PEBS buffers
already resident in HBM: reset the counters, run the attribution kernel over
every buffer (the body of mem_sampling_finalize's loop, src/mem_sampling.c:
324-342) and its long-tail reduce, and, for N > 1, merge the per-rank
counters into rank 0 with RCCL reduces over xGMI.  Report printing is outside
the timed region.

Default workload (the north-star configuration, BASELINE.json configs[3]'s
per-GPU shard): 125M 40-byte PERF_RECORD_SAMPLE records per GPU in 128 KiB
per-thread buffers, 1M object intervals (+ 8 globals + [stack]), 8 threads.
Weak scaling: every rank analyses its own 125M-record shard against the same
table, so --gpus 8 is configs[3] (1B records).  configs[1] (10M records, 1k
intervals) and configs[2] (100M records, 100k intervals, per-page on) are measured
after it and reported in the same JSON line under "secondary".

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2|c3|k1m]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

RECORD_BYTES = 40
COMPACT_BYTES = 16  # partition-first path: compact record per routed sample
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MIN_TIMED_S = 1.0      # default --steps: enough steps for at least this much timed work

WORKLOADS = {
    "c2": dict(nb_samples=10_000_000, nb_intervals=1_000, desc="configs[1]: 10M PEBS records/GPU, 1k object intervals"),
    "c3": dict(nb_samples=100_000_000, nb_intervals=100_000, desc="configs[2]: 100M PEBS records/GPU, 100k intervals, per-page on"),
    "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024,
               desc="configs[3] per-GPU shard: 1B records / 8 GPUs, 1M intervals, per-page on"),
    "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024,
                desc="north-star table size, small batch: 10M PEBS records/GPU, 1M object intervals"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Workload:
    """One synthetic batch resident in HBM and an engine over it."""

    def __init__(self, name, rank, device, distributed):
        import torch

        from numamma_amd import _lib
        from numamma_amd.engine import Engine
        from numamma_amd.replay import SynthConfig, generate

        self.name = name
        wl = WORKLOADS[name]
        cfg_kw = {k: v for k, v in wl.items() if k != "desc"}
        self.cfg = SynthConfig(seed=1, sample_seed=1000 + rank, **cfg_kw)
        t0 = time.time()
        self.rp = generate(self.cfg)
        arena, offs, lens, ranks, acc = self.rp.packed()
        log(f"[rank {rank}] {name}: {self.rp.nb_records()} records in {len(lens)} buffers, "
            f"{arena.nbytes / 1e6:.0f} MB, generated in {time.time() - t0:.1f}s")
        self.d_arena = torch.from_numpy(arena).to(device)
        del arena
        self.nb_buf = len(lens)
        self.samples = int(lens.sum()) // RECORD_BYTES
        # (NMG_BENCH_DEBUG_FLAGS: internal ablation switches for counter
        # passes, tools/gpu_round.sh pmcx; never set for a reported number)
        dbg = int(os.environ.get("NMG_BENCH_DEBUG_FLAGS", "0"), 0)
        if dbg:
            os.environ["NMG_INTERNAL_FLAGS"] = "1"
        self.eng = Engine(device=device.index, flags=_lib.NMG_F_DEFAULT | dbg, nb_threads=self.rp.nb_threads)
        self.eng.set_objects(self.rp.table)
        # global analysis order: rank-major (seq_base)
        self.eng.set_device_buffers(self.d_arena.data_ptr(), offs, lens, ranks, acc, seq_base=rank * self.nb_buf)
        self.merge_bufs = []
        self.hist_packer = None
        self.obj_packer = None
        # per-step split of a distributed step (host clock): analysis (reset +
        # analyze + synchronize) and merge (exports, RCCL reduces / gathers,
        # imports, synchronized), and the counter bytes this rank contributes
        self.split = {"analysis_s": 0.0, "merge_s": 0.0, "steps": 0, "payload_bytes": 0}
        if distributed:  # merge buffers for the timed RCCL reduces (dense arrays)
            from numamma_amd.distributed import HistPacker, ObjPacker

            for which, dt in ((_lib.NMG_ARR_SUM64, torch.int64), (_lib.NMG_ARR_MIN64, torch.int64),
                              (_lib.NMG_ARR_MAX64, torch.int64)):
                n = self.eng.array_size(which)
                if n:
                    self.merge_bufs.append((which, torch.empty(n, dtype=dt, device=device)))
            # the page histogram (70 % of the payload) packed: bytes + overflow list;
            # the per-object count / weight rows as u32 words + overflow list
            self.hist_packer = HistPacker(self.eng, device)
            self.obj_packer = ObjPacker(self.eng, device)

    def step(self):
        import torch

        from numamma_amd import _lib
        from numamma_amd.distributed import GLOBAL_SUM_WORDS, reduce_u64

        t0 = time.perf_counter()
        self.eng.reset()
        self.eng.analyze()
        if self.merge_bufs:
            self.eng.synchronize()
            t1 = time.perf_counter()
            nbytes = 0
            for which, t in self.merge_bufs:
                self.eng.export_array(which, t.data_ptr())
                if which == _lib.NMG_ARR_SUM64 and self.obj_packer is not None:
                    got = self.obj_packer.merge(t, dst=0)
                    if got is not None:
                        reduce_u64(t[:GLOBAL_SUM_WORDS], "sum", dst=0)  # (the global sums as u64)
                        nbytes += got + 8 * GLOBAL_SUM_WORDS
                        continue
                reduce_u64(t, {0: "sum", 1: "min", 2: "max"}[which], dst=0)
                nbytes += 8 * t.numel()
            if self.hist_packer is not None:
                nbytes += self.hist_packer.merge(dst=0)
            torch.cuda.synchronize(self.d_arena.device)  # (the reduces ran on the collectives' stream)
            t2 = time.perf_counter()
            self.split["analysis_s"] += t1 - t0
            self.split["merge_s"] += t2 - t1
            self.split["steps"] += 1
            self.split["payload_bytes"] = nbytes


def timed_run(w, steps, warmup, barrier, agree=None):
    for _ in range(warmup):
        w.step()
    barrier()
    if steps <= 0:  # auto: one more step to size the timed region
        t = time.perf_counter()
        w.step()
        barrier()
        one = time.perf_counter() - t
        steps = int(min(2000, max(20, math.ceil(MIN_TIMED_S / max(one, 1e-6)))))
        if agree:  # every rank runs rank 0's count (the steps hold collectives)
            steps = agree(steps)
    if hasattr(w, "split"):  # (the timed steps only)
        w.split.update(analysis_s=0.0, merge_s=0.0, steps=0)
    t_start = time.perf_counter()
    for _ in range(steps):
        w.step()
    barrier()  # device sync; raises on a kernel-reported error
    return time.perf_counter() - t_start, steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="timed steps (0: enough for >= 1 s)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--secondary", default="c2,c3",
                    help="workloads measured after the main one, comma-separated (N=1; '' = none)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--handle", action="store_true",
                    help="without a launcher, drive the GPUs through one engine handle even for --gpus 1 "
                         "(host-staged buffers, as --gpus N > 1 does), so a 1 -> N curve compares one path")
    ap.add_argument("--cpu-records", type=int, default=100_000,
                    help="records in the reference-loop oracle's sample (its linear call-site list is quadratic)")
    ap.add_argument("--cpu-st-records", type=int, default=2_000_000,
                    help="records in the one-thread run of the multi-threaded restatement")
    ap.add_argument("--cpu-mt-records", type=int, default=62_500_000,
                    help="records in the multi-threaded baseline's sample (about 0.8 s a run on 16 threads: long "
                         "enough that the shared host's noise averages out within a run)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                    help="host threads of the multi-threaded CPU baseline (default: this job's CPU share, "
                         "OMP_NUM_THREADS, else every CPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and (args.gpus > 1 or args.handle):  # no launcher: one process drives every GPU through the C-ABI
        return main_one_process(args)
    # test hooks for the multi-rank path on a one-GPU box (never used by the driver):
    # NMG_BENCH_BACKEND=gloo, NMG_BENCH_SAME_GPU=1 (every rank on GPU 0)
    backend = os.environ.get("NMG_BENCH_BACKEND", "nccl")
    if os.environ.get("NMG_BENCH_SAME_GPU") == "1":
        local = 0
    if world != args.gpus:
        log(f"error: WORLD_SIZE={world} but --gpus={args.gpus}")
        sys.exit(2)
    distributed = world > 1
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)

    from numamma_amd.distributed import merge_engine

    w = Workload(args.workload, rank, device, distributed)

    def barrier():
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(device)
        w.eng.synchronize()

    def agree(n):
        if not distributed:
            return n
        t = torch.tensor([n], dtype=torch.int64, device=device if backend == "nccl" else "cpu")
        dist.broadcast(t, src=0)
        return int(t.item())

    elapsed, steps = timed_run(w, args.steps, args.warmup, barrier, agree)
    attr_ms, total_ms = w.eng.kernel_times(min(steps, 64))  # HIP events on the engine stream
    phases = w.eng.phase_times(min(steps, 64))
    if distributed:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed * 1e3 / steps
    value = w.samples * world / (elapsed / steps)

    # sanity: every record of the batch was decoded exactly once per step
    g, ns, nf = w.eng.global_counters()
    assert ns == w.samples or os.environ.get("NMG_BENCH_DEBUG_FLAGS"), (ns, w.samples)

    if distributed:
        merge_engine(w.eng, dst=0)  # full merge once (dense + gathers) for the report

    split = None
    if distributed and w.split["steps"]:  # the slowest rank's analysis / merge split per step
        sp = torch.tensor([w.split["analysis_s"], w.split["merge_s"]], dtype=torch.float64,
                          device=device if backend == "nccl" else "cpu")
        dist.all_reduce(sp, op=dist.ReduceOp.MAX)
        split = {"analysis_ms": float(sp[0]) * 1e3 / w.split["steps"], "merge_ms": float(sp[1]) * 1e3 / w.split["steps"],
                 "payload_bytes_per_rank": int(w.split["payload_bytes"]),
                 "note": "host clock per timed step, maximum over ranks: analysis = reset + analyze + synchronize; "
                         "merge = exports + RCCL reduces / gathers + imports, synchronized"}
    if rank == 0:
        out = result_line(args, w, world, steps, ms_per_step, value, attr_ms, total_ms, phases)
        if split:
            out["merge"] = split
        if world == 1 and args.secondary:
            out["secondary"] = {}
            for name in args.secondary.split(","):
                s = Workload(name, rank, device, False)

                def sbar():
                    torch.cuda.synchronize(device)
                    s.eng.synchronize()

                se, sn = timed_run(s, 0, 3, sbar)
                sa, st = s.eng.kernel_times(min(sn, 64))
                out["secondary"][s.name] = {
                    "workload": WORKLOADS[s.name]["desc"], "value": s.samples / (se / sn), "unit": "samples/s",
                    "ms_per_step": se * 1e3 / sn, "steps": sn,
                    "attribute_kernel_ms": float(np.mean(sa)), "launch_ms": float(np.mean(st)),
                    "roofline_frac": s.samples * RECORD_BYTES / (float(np.mean(sa)) * 1e-3) / 1e9 / HBM_PEAK_GBS}
                if s.name == "c2" and not args.no_cpu_baseline:
                    # BASELINE.md:34-38: the reference loop timed at configs[1], the whole workload
                    out["secondary"][s.name]["cpu_reference_loop"] = reference_loop_full(s.rp)
                s.eng.close()
                del s
        if world == 1 and not args.no_cpu_baseline:
            log(f"[rank 0] cpu baseline: first {args.cpu_records} records")
            out["cpu_baseline"] = cpu_baseline(w.rp, args.cpu_records, args.cpu_mt_records, args.cpu_threads,
                                         args.cpu_st_records)
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    w.eng.close()


def main_one_process(args):
    """--gpus N without a launcher: the reference's shape, one analysing
    process (mem_sampling.c:324-342), here driving N GPUs through one engine
    handle (nmg_options.nb_gpus): the buffers of N per-GPU shards are staged
    once, and a step is reset + nmg_analyze (every GPU analyses its
    byte-balanced contiguous range, RCCL reduces the counters over xGMI into
    GPU 0's handle) + the handle's per-buffer count gather.  Exits with status
    2 when fewer than N GPUs are visible."""
    import torch

    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    n = args.gpus
    visible = torch.cuda.device_count()
    same = os.environ.get("NMG_BENCH_SAME_GPU") == "1"  # (test hook: every worker on GPU 0, device merges)
    if visible < n and not same:
        log(f"error: --gpus {n} but {visible} GPU(s) visible")
        sys.exit(2)
    wl = WORKLOADS[args.workload]
    cfg = SynthConfig(seed=1, sample_seed=1000, **{k: v for k, v in wl.items() if k != "desc"})
    t0 = time.time()
    rp = generate(cfg)
    bufs = [b.linear() for b in rp.buffers]
    shard = sum(x.nbytes for x in bufs) // RECORD_BYTES
    log(f"[1 process, {n} GPUs] {args.workload}: shard of {shard} records in {len(bufs)} buffers, generated in "
        f"{time.time() - t0:.1f}s; every GPU analyses one copy of it")
    devices = [0] * n if same else list(range(n))
    eng = Engine(devices=devices, nb_threads=rp.nb_threads, copy_threads=16)
    eng.set_objects(rp.table)
    subs = [(b.thread_rank, b.access_type, x) for b, x in zip(rp.buffers, bufs) if x.shape[0]]
    for _ in range(n):  # N shards in analysis order; the handle cuts them into N byte-balanced ranges
        eng.submit_buffers(subs)

    class W:
        def step(self):
            eng.reset()
            eng.analyze()

    def barrier():
        eng.synchronize()
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    elapsed, steps = timed_run(W(), args.steps, args.warmup, barrier)
    merge_ms, payload = eng.merge_stats()  # (the last step's merge, GPU events on the root device)
    g, ns, nf = eng.global_counters()
    assert ns == n * shard, (ns, n * shard)
    ms_per_step = elapsed * 1e3 / steps
    out = {
        "metric": "PEBS samples/s analysed (device-resident)",
        "value": n * shard / (elapsed / steps),
        "unit": "samples/s",
        "n_gpus": n,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded SURVEY 8(d) generator); one per-GPU shard, analysed by every GPU",
        "config": {"workload": f"{args.workload}: {wl['desc']}", "records_per_gpu": shard,
                   "object_intervals": int(cfg.nb_intervals), "threads": rp.nb_threads,
                   "parallelism": (f"one process, nmg_options.nb_gpus={n}: buffers sharded over {n} GPUs, "
                                   "RCCL reduce of the counters" if n > 1 else
                                   "one process, one engine handle over host-staged buffers (the --gpus N path at N=1)")},
    }
    out["merge"] = {"merge_ms": merge_ms, "analysis_ms": ms_per_step - merge_ms, "payload_bytes_per_gpu": payload,
                    "note": ("GPU events on the root device around the last step's counter merge (end of worker 0's "
                             "analysis to the end of the reduces, waiting for the other workers included); analysis_ms "
                             "= ms_per_step - merge_ms" if n > 1 else "one GPU: no merge")
                            + ("; workers share GPU 0 (NMG_BENCH_SAME_GPU=1): device merges, not RCCL" if same else "")}
    # per GPU: its shard's 40 B records over the whole step (analysis, the
    # RCCL reduce of the counters into GPU 0's handle, the handle's gathers)
    achieved = shard * RECORD_BYTES / (ms_per_step * 1e-3) / 1e9
    out["roofline"] = {
        "bound": "hbm", "kernel": "whole step per GPU: nmg_analyze on every GPU + RCCL reduce + gathers",
        "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
        "traffic": None, "algorithmic_bytes_per_launch": shard * RECORD_BYTES,
        "note": "achieved = one GPU's shard (40 B per record, SURVEY 8(d)) / the step's wall time; the single-GPU "
                "line's kernel split and PMC traffic apply per GPU"}
    print(json.dumps(out), flush=True)
    eng.close()


def load_traffic(name):
    """HBM bytes per launch from profiles/pmc_<name>.json (tools/pmc_pipeline.py),
    or None with the reason when the file is missing or was measured on other
    kernel sources than this tree's (numamma_amd/srchash.py)."""
    from numamma_amd.srchash import kernel_source_hash

    path = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if not os.path.exists(path):
        return None, None, f"no profiles/pmc_{name}.json"
    try:
        pmc = json.load(open(path))
    except (OSError, ValueError) as e:
        return None, None, f"profiles/pmc_{name}.json unreadable: {e}"
    here = kernel_source_hash()
    if pmc.get("source_hash") != here:
        return None, None, (f"profiles/pmc_{name}.json was measured on kernel sources {pmc.get('source_hash')}, "
                            f"this tree is {here}: traffic not reported")
    return pmc.get("hbm_bytes_per_launch"), pmc, (f"profiles/pmc_{name}.json (sources {here}, "
                                                 f"commit {pmc.get('commit', '?')})")


def result_line(args, w, world, steps, ms_per_step, value, attr_ms, total_ms, phases):
    wl = WORKLOADS[w.name]
    avg_attr = float(np.mean(attr_ms))
    avg_total = float(np.mean(total_ms))
    first_ms, rest_ms = (float(np.mean(x)) if x else 0.0 for x in phases)
    algo = w.samples * RECORD_BYTES
    achieved = algo / (avg_attr * 1e-3) / 1e9
    traffic, pmc, traffic_src = load_traffic(w.name)
    routed = rest_ms > 0.0  # the partition-first path ran (tables > 1023 keys)
    kernels = {}
    route = "route2_kernel"  # the route pass
    if routed:
        # the route pass reads every 40 B record and writes a 16 B compact
        # record per sample (nmg_route.h XLayout); the local pass reads them back
        kernels[route] = {"avg_ms": first_ms, "algorithmic_bytes": w.samples * (RECORD_BYTES + COMPACT_BYTES)}
        kernels["overflow+count+plan+scatter+local_kernel"] = {"avg_ms": rest_ms,
                                                               "algorithmic_bytes": w.samples * COMPACT_BYTES}
    else:
        kernels["attribute_kernel"] = {"avg_ms": first_ms, "algorithmic_bytes": algo}
    for k, v in kernels.items():
        v["achieved_GBps"] = v["algorithmic_bytes"] / (v["avg_ms"] * 1e-3) / 1e9 if v["avg_ms"] else None
        v["frac"] = v["achieved_GBps"] / HBM_PEAK_GBS if v["achieved_GBps"] else None
        if pmc:
            names = [k] if k == route else [n for n in pmc["kernels"] if n not in ("route_kernel", "route2_kernel")
                                           and not n.startswith("reduce")]
            v["traffic"] = sum(pmc["kernels"][n]["hbm_read_bytes"] + pmc["kernels"][n]["hbm_write_bytes"]
                               for n in names if n in pmc["kernels"])
    return {
        "metric": "PEBS samples/s analysed (device-resident)",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded SURVEY 8(d) generator: Zipf objects, mem_lvl mix, 128 KiB buffers)",
        "config": {
            "workload": f"{w.name}: {wl['desc']}",
            "records_per_gpu": w.samples,
            "buffers_per_gpu": w.nb_buf,
            "object_intervals": int(w.cfg.nb_intervals),
            "table_entries": w.rp.table.nb_entries,
            "threads": w.rp.nb_threads,
            "parallelism": f"buffers sharded over {world} GPU(s), RCCL reduce of counters" if world > 1 else "1 GPU",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": (f"nmg attribution launch, partition-first: {route} -> overflow/count/plan/scatter -> "
                       "local_kernel" if routed else "nmg::attribute_kernel"),
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            # the HBM bytes the launch really moves (PMC, per launch) per second
            "traffic_GBps": (traffic / (avg_attr * 1e-3) / 1e9) if traffic else None,
            "algorithmic_bytes_per_launch": algo,
            "avg_kernel_ms": avg_attr,
            "avg_launch_ms": avg_total,
            "kernels": kernels,
            "note": "achieved = 40 B per record (SURVEY 8(d)) / attribution time, HIP events on the engine stream "
                    "around the kernels that attribute the records; the launch adds the long-tail reduce; "
                    f"kernels = the same events split after {route}; traffic: {traffic_src}",
        },
    }


def _sample_replay(rp, max_records):
    from numamma_amd.replay import Replay

    n, recs = 0, 0
    for b in rp.buffers:
        if recs >= max_records:
            break
        recs += b.linear().shape[0] // RECORD_BYTES
        n += 1
    return Replay(rp.nb_threads, rp.table, rp.buffers[:max(1, n)]), max(1, n)


def _rate_runs(fn, target_s, max_runs, tag):
    """fn() -> (records, seconds); repeated until about target_s seconds."""
    rates, secs, recs = [], 0.0, 0
    while len(rates) < max_runs and (not rates or secs < target_s):
        recs, t = fn()
        log(f"[rank 0] cpu baseline ({tag}) run {len(rates)}: {recs} records in {t:.2f}s")
        rates.append(recs / t)
        secs += t
    return float(np.median(rates)), rates, secs, recs


def reference_loop_full(rp, target_s=10.0, max_runs=5):
    """The single-threaded C restatement of the reference loop
    (oracle/nmg_oracle.c: mem_sampling_finalize's while(samples) loop,
    mem_sampling.c:311-346, with the reference's linear call-site and page
    lists) over a WHOLE workload (configs[1]: 10M records, 1k intervals),
    analysis loop timed, repeated to about target_s seconds; median rate."""
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "full.bin")
        rp.write(path)

        def run():
            t = pyoracle.run(path, os.path.join(d, "out"), os.path.join(d, "stdout.txt"))
            return t["nb_samples"], t["analysis_s"]

        v, rates, secs, recs = _rate_runs(run, target_s, max_runs, "reference loop, whole workload")
    return {"value": v, "unit": "samples/s", "cores": 1, "kind": "port", "runs": rates,
            "spread": [float(min(rates)), float(max(rates))],
            "sample": f"the whole workload ({recs} records, {len(rp.buffers)} buffers) analysed {len(rates)}x by the "
                      f"single-threaded restatement of the reference loop ({secs:.1f}s), median run; 1 core of "
                      f"{os.cpu_count()} (OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')})"}


def cpu_baseline(rp, max_records, mt_records, threads, st_records, target_s=20.0, max_runs=15):
    """CPU baselines timed on this host on bounded samples of the same
    workload (the first buffers of the batch, against the full object table);
    each is run repeatedly until about its share of `target_s` seconds of
    timed work and reports the MEDIAN per-run rate:

    * value: the multi-threaded bit-exact C++ restatement
      (oracle/nmg_cpu_mt.cpp) on `threads` host threads, first `mt_records`
      records; rate = records / (analysis + merge seconds);
    * single_thread: the same restatement on one thread, first `st_records`;
    * reference_loop_oracle: the single-threaded C restatement of the
      reference loop (oracle/nmg_oracle.c), which keeps the reference's
      linear call-site list (find_call_site, mem_analyzer.c:1302-1331, run at
      every object's first match) and linear page-block lists: with one call
      site per object its cost grows with the square of the objects touched,
      so its sample is `max_records` records (about 10 s)."""
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    def mt(path, nthreads):
        t = pyoracle.run_mt(path, None, threads=nthreads, levels=False)
        return t["nb_samples"], t["analysis_s"] + t["merge_s"]

    def st(path, d):
        t = pyoracle.run(path, os.path.join(d, "out"), os.path.join(d, "stdout.txt"))
        return t["nb_samples"], t["analysis_s"]

    host = (f"the host has {os.cpu_count()} CPUs, of which this job's share is OMP_NUM_THREADS="
            f"{os.environ.get('OMP_NUM_THREADS', 'unset')}")
    with tempfile.TemporaryDirectory() as d:
        sub, n = _sample_replay(rp, mt_records)
        path = os.path.join(d, "mt.bin")
        sub.write(path)
        del sub
        mt(path, threads)  # warm-up (first touch of the arrays)
        v, rates, secs, recs = _rate_runs(lambda: mt(path, threads), target_s, max_runs, f"{threads} threads")
        out = {
            "value": v,
            "unit": "samples/s",
            "cores": threads,
            "kind": "port",
            "sample": f"first {n} of {len(rp.buffers)} buffers ({recs} records, full object table) analysed "
                      f"{len(rates)}x by the multi-threaded bit-exact restatement (oracle/nmg_cpu_mt.cpp) on "
                      f"{threads} threads ({secs:.1f}s of analysis + merge), median run; {host}",
            "runs": rates,
            "spread": [float(min(rates)), float(max(rates))],
            # interquartile range relative to the median (the runs' spread without the outliers)
            "iqr_pct": float(100.0 * (np.percentile(rates, 75) - np.percentile(rates, 25)) / v),
        }
        os.remove(path)
        sub, n = _sample_replay(rp, st_records)
        path = os.path.join(d, "st.bin")
        sub.write(path)
        del sub
        v, rates, secs, recs = _rate_runs(lambda: mt(path, 1), target_s / 2, max_runs, "1 thread")
        out["single_thread"] = {
            "value": v, "cores": 1,
            "sample": f"first {n} buffers ({recs} records) analysed {len(rates)}x by oracle/nmg_cpu_mt.cpp on one "
                      f"thread ({secs:.1f}s), median run"}
        os.remove(path)
        sub, n = _sample_replay(rp, max_records)
        path = os.path.join(d, "ref.bin")
        sub.write(path)
        v, rates, secs, recs = _rate_runs(lambda: st(path, d), target_s / 4, max_runs, "reference loop")
        out["reference_loop_oracle"] = {
            "value": v, "cores": 1,
            "sample": f"first {n} buffers ({recs} records) analysed {len(rates)}x ({secs:.1f}s of analysis loop), "
                      "median run; single-threaded like the reference (global mutex, mem_analyzer.c:254), with its "
                      "linear call-site list (quadratic in the objects touched)"}
    return out


if __name__ == "__main__":
    main()
