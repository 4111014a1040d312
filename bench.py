#!/usr/bin/env python3
"""Benchmark: PEBS samples/s analysed (device-resident) on 1..8 MI355X.

One step = one full analysis pass over one batch of synthetic PEBS buffers
already resident in HBM: reset the counters, run the attribution kernel over
every buffer (the body of mem_sampling_finalize's loop, src/mem_sampling.c:
324-342) and, for N > 1, merge the per-rank counters into rank 0 with RCCL
reduces over xGMI.  Report printing is outside the timed region.

Workload (BASELINE.json configs[1], "c2"): 10M 40-byte PERF_RECORD_SAMPLE
records per GPU in 128 KiB per-thread buffers, 1k object intervals (+ 8
globals + [stack]), 8 threads.  Weak scaling: every rank analyses its own
10M-record shard against the same object table.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|k1m]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

RECORD_BYTES = 40
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    "c2": dict(nb_samples=10_000_000, nb_intervals=1_000, desc="configs[1]: 10M PEBS records/GPU, 1k object intervals"),
    "c3": dict(nb_samples=100_000_000, nb_intervals=100_000, desc="configs[2]: 100M PEBS records/GPU, 100k intervals, per-page on"),
    "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024,
               desc="configs[3] per-GPU shard: 1B records / 8 GPUs, 1M intervals"),
    "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024,
                desc="north-star table size: 10M PEBS records/GPU, 1M object intervals"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-frac", type=float, default=1.0)
    ap.add_argument("--verify", action="store_true", help="check the merged counters against the oracle")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # test hooks for the multi-rank path on a one-GPU box (never used by the driver):
    # NMG_BENCH_BACKEND=gloo, NMG_BENCH_SAME_GPU=1 (every rank on GPU 0)
    backend = os.environ.get("NMG_BENCH_BACKEND", "nccl")
    if os.environ.get("NMG_BENCH_SAME_GPU") == "1":
        local = 0
    if world != args.gpus:
        log(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    distributed = world > 1
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)

    from numamma_amd import _lib
    from numamma_amd.distributed import merge_engine, reduce_u32_sum, reduce_u64
    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    wl = WORKLOADS[args.workload]
    cfg_kw = {k: v for k, v in wl.items() if k != "desc"}
    cfg = SynthConfig(seed=1, sample_seed=1000 + rank, **cfg_kw)
    t0 = time.time()
    rp = generate(cfg)
    arena, offs, lens, ranks, acc = rp.packed()
    log(f"[rank {rank}] generated {rp.nb_records()} records in {len(lens)} buffers, "
        f"{arena.nbytes / 1e6:.0f} MB, {time.time() - t0:.1f}s")
    d_arena = torch.from_numpy(arena).to(device)
    nb_buf = len(lens)
    seq_base = rank * nb_buf  # global analysis order: rank-major

    eng = Engine(device=local, flags=_lib.NMG_F_DEFAULT, nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.set_device_buffers(d_arena.data_ptr(), offs, lens, ranks, acc, seq_base=seq_base)
    samples_per_rank = int(lens.sum()) // RECORD_BYTES

    # merge buffers for the timed RCCL reduces (dense arrays only; the tiny
    # variable-length gathers run once after timing)
    merge_bufs = []
    if distributed:
        for which, dt in ((_lib.NMG_ARR_SUM64, torch.int64), (_lib.NMG_ARR_MIN64, torch.int64),
                          (_lib.NMG_ARR_MAX64, torch.int64), (_lib.NMG_ARR_HIST32, torch.int32)):
            n = eng.array_size(which)
            if n:
                merge_bufs.append((which, torch.empty(n, dtype=dt, device=device)))

    def step():
        eng.reset()
        eng.analyze()
        if distributed:
            eng.synchronize()
            for which, t in merge_bufs:
                eng.export_array(which, t.data_ptr())
                if which == _lib.NMG_ARR_HIST32:
                    reduce_u32_sum(t, dst=0)
                else:
                    reduce_u64(t, {0: "sum", 1: "min", 2: "max"}[which], dst=0)

    def barrier():
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(device)
        eng.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()  # device sync; raises on a kernel-reported error
    elapsed = time.perf_counter() - t_start
    kernel_ms = eng.launch_times(min(args.steps, 64))  # HIP events on the engine stream
    if distributed:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed * 1e3 / args.steps
    total_samples = samples_per_rank * world
    value = total_samples / (elapsed / args.steps)

    # sanity: every record of the batch was decoded exactly once per step
    g, ns, nf = eng.global_counters()
    assert ns == samples_per_rank, (ns, samples_per_rank)

    if distributed:
        merge_engine(eng, dst=0)  # full merge once (dense + gathers) for the report

    if rank == 0:
        avg_kernel_ms = float(np.mean(kernel_ms))
        achieved = samples_per_rank * RECORD_BYTES / (avg_kernel_ms * 1e-3) / 1e9
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
        if os.path.exists(pmc_path):
            try:
                traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": "PEBS samples/s analysed (device-resident)",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded SURVEY 8(d) generator: Zipf objects, mem_lvl mix, 128 KiB buffers)",
            "config": {
                "workload": f"{args.workload}: {wl['desc']}",
                "records_per_gpu": samples_per_rank,
                "buffers_per_gpu": nb_buf,
                "object_intervals": int(cfg.nb_intervals),
                "table_entries": rp.table.nb_entries,
                "threads": rp.nb_threads,
                "parallelism": f"buffers sharded over {world} GPU(s), RCCL reduce of counters" if world > 1 else "1 GPU",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "nmg::attribute_kernel",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "avg_kernel_ms": avg_kernel_ms,
                "algorithmic_bytes_per_launch": samples_per_rank * RECORD_BYTES,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(rp, args.cpu_sample_frac)
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()


def cpu_baseline(rp, frac, target_s=10.0, max_runs=40):
    """The CPU oracle (a single-threaded C restatement of the reference's
    offline analysis loop, oracle/nmg_oracle.c) timed on this host on the
    same workload: the first `frac` of the buffers, analysed repeatedly until
    about `target_s` seconds of analysis time have accumulated (the whole c2
    batch takes well under a second), rate = records / analysis seconds."""
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    from numamma_amd.replay import Replay

    n = max(1, int(len(rp.buffers) * frac))
    sub = Replay(rp.nb_threads, rp.table, rp.buffers[:n])
    runs, samples, secs = 0, 0, 0.0
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "sample.bin")
        sub.write(path)
        while runs < max_runs and (runs == 0 or secs < target_s):
            t = pyoracle.run(path, os.path.join(d, "out"), os.path.join(d, "stdout.txt"))
            runs += 1
            samples += t["nb_samples"]
            secs += t["analysis_s"]
    return {
        "value": samples / secs,
        "unit": "samples/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n} of {len(rp.buffers)} buffers ({samples // runs} records) analysed {runs}x, "
                  f"{secs:.1f}s of analysis loop; single-threaded like the reference "
                  f"(global mutex, mem_analyzer.c:254); host has {os.cpu_count()} CPUs",
    }


if __name__ == "__main__":
    main()
