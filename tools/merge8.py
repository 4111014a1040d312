"""configs[3] as a whole on one GPU: `world` ranks (gloo, every one on GPU 0)
each analyse a configs[3]-sized shard (125M records by default, 1M
intervals; the shard rank r of bench.py, sample_seed 1000 + r), in the global
rank-major analysis order (seq_base = the buffers of the ranks before), then
merge through the product's one-process-per-GPU chain
(numamma_amd/distributed.py merge_engine: nmg_export_array -> reduce ->
nmg_import_array, the page histogram packed, sparse cells and per-buffer
counts gathered) -- the merge the 8-GPU bench runs over RCCL, here over gloo.

The check: every rank also analyses its shard with the bit-exact CPU
restatement (oracle/nmg_cpu_mt.cpp, pinned against the oracle in
tests/test_cpu_mt.py); rank 0 merges the restatement's raw results with
plain numpy (sums, minimums, maximums, page rows summed by key, per-buffer
counts concatenated, first-match ordinals shifted by seq_base) and compares
every counter of its merged engine with them.  The mem_sampling.c:324-342
loop over 1B records, sharded as configs[3] shards it.

Test tooling (the oracle restatement is the checker, never the product):
    python tools/merge8.py [--world 8] [--samples 125000000] > profiles/r5/merge8_c4.json
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def _worker(rank, world, port, shm, args, ret):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    try:
        import torch
        import torch.distributed as dist

        import pyoracle
        from numamma_amd.distributed import merge_engine
        from numamma_amd.engine import Engine
        from numamma_amd.replay import SynthConfig, generate

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        t0 = time.time()
        rp = generate(SynthConfig(seed=1, sample_seed=1000 + rank, nb_samples=args.samples,
                                  nb_intervals=args.intervals, size_max=64 * 1024))
        arena, offs, lens, ranks, acc = rp.packed()
        nbuf = [None] * world
        dist.all_gather_object(nbuf, len(lens))
        seq_base = int(sum(nbuf[:rank]))
        t_gen = time.time() - t0
        _log(f"rank {rank}: shard generated in {t_gen:.0f}s ({len(lens)} buffers)")
        # the bit-exact restatement of this shard (its own analysis order: seq
        # 0..), one rank at a time (host memory: a replay file in shm each)
        path = os.path.join(shm, f"shard{rank}.bin")
        raw = os.path.join(shm, f"shard{rank}_raw.bin")
        tm = None
        for turn in range(world):
            if turn == rank:
                rp.write(path)
                tm = pyoracle.run_mt(path, raw, threads=args.mt_threads, levels=False)
                os.remove(path)
                _log(f"rank {rank}: restatement {tm['analysis_s']:.1f}s")
            dist.barrier()
        dev = torch.device("cuda", 0)
        d_arena = torch.from_numpy(arena).to(dev)
        del arena
        eng = Engine(device=0, nb_threads=rp.nb_threads)
        eng.set_objects(rp.table)
        eng.set_device_buffers(d_arena.data_ptr(), offs, lens, ranks, acc, seq_base=seq_base)
        del rp
        steps = []
        nbytes = 0
        for rep in range(args.reps):
            dist.barrier()
            torch.cuda.synchronize(dev)
            ta = time.perf_counter()
            eng.reset()
            eng.analyze()
            eng.synchronize()
            tb = time.perf_counter()
            nbytes = merge_engine(eng, dst=0, device=dev, packed_hist=True)
            torch.cuda.synchronize(dev)
            dist.barrier()
            tc = time.perf_counter()
            steps.append((tb - ta, tc - tb))
            _log(f"rank {rank}: rep {rep} analyze {tb - ta:.3f}s merge {tc - tb:.3f}s")
        out = {"rank": rank, "seq_base": seq_base, "nb_buffers": len(lens), "gen_s": t_gen,
               "restatement_s": tm["analysis_s"], "payload_bytes": nbytes,
               "analyze_s": [s[0] for s in steps], "merge_s": [s[1] for s in steps]}
        if rank == 0:
            g, ns, nf = eng.global_counters()
            first, cw = eng.object_counters()
            bs, bf = eng.buffer_counts()
            np.savez(os.path.join(shm, "merged.npz"), g=g, ns=ns, nf=nf, first=first, cw=cw, bs=bs, bf=bf,
                     cells=eng.page_cells())
        eng.close()
        del d_arena
        dist.barrier()
        dist.destroy_process_group()
        ret.put((rank, out))
    except Exception:  # surfaced by the parent
        import traceback

        ret.put((rank, traceback.format_exc()))
        raise


def merge_restatements(raws, seq_bases):
    """The merge algebra over per-shard raw results (numamma_amd/results.py
    layout): what the product's reduce chain must give."""
    g = np.zeros((2, 75), dtype=np.uint64)
    mins = np.zeros(75, dtype=bool)
    maxs = np.zeros(75, dtype=bool)
    for b in range(18):  # struct count {count, min_weight, max_weight, sum_weight} (mem_analyzer.h:10-15)
        mins[3 + 4 * b + 1] = True
        maxs[3 + 4 * b + 2] = True
    sums = ~(mins | maxs)
    g[:, mins] = np.uint64(~np.uint64(0))
    first = None
    cw = None
    ns = nf = 0
    keys, vals = [], []
    for r, raw in enumerate(raws):
        gg = raw.global_counters
        g[:, sums] += gg[:, sums]
        g[:, mins] = np.minimum(g[:, mins], gg[:, mins])
        g[:, maxs] = np.maximum(g[:, maxs], gg[:, maxs])
        ns += raw.nb_samples
        nf += raw.nb_found
        fo = raw.first_ordinal.copy()
        ok = fo != np.uint64(~np.uint64(0))
        fo[ok] += np.uint64(seq_bases[r]) << np.uint64(32)
        first = fo if first is None else np.minimum(first, fo)
        c = raw.count_weight
        cw = c.copy() if cw is None else cw + c
        cl = raw.cells.astype(np.uint64)
        keys.append((cl[:, 0] << np.uint64(42)) | (cl[:, 1] << np.uint64(32)) | cl[:, 2])
        vals.append(cl[:, 3])
    k = np.concatenate(keys)
    v = np.concatenate(vals)
    u, inv = np.unique(k, return_inverse=True)
    s = np.bincount(inv, weights=v.astype(np.float64), minlength=u.shape[0]).astype(np.uint64)  # (sums < 2^53)
    cells = np.stack([u >> np.uint64(42), (u >> np.uint64(32)) & np.uint64(1023), u & np.uint64(0xFFFFFFFF),
                      s & np.uint64(0xFFFFFFFF)], axis=1).astype(np.uint32)
    bs = np.concatenate([raw.buf_samples for raw in raws])
    bf = np.concatenate([raw.buf_found for raw in raws])
    return g, ns, nf, first, cw, cells, bs, bf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--samples", type=int, default=125_000_000)
    ap.add_argument("--intervals", type=int, default=1_000_000)
    ap.add_argument("--mt-threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--shm", default="/dev/shm")
    args = ap.parse_args()
    import multiprocessing as mp

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    from numamma_amd.results import RawResults

    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    t0 = time.time()
    with tempfile.TemporaryDirectory(dir=args.shm) as shm:
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, args.world, port, shm, args, ret)) for r in range(args.world)]
        for p in procs:
            p.start()
        msgs = dict(ret.get(timeout=1800) for _ in procs)
        for p in procs:
            p.join(timeout=120)
        for r, m in msgs.items():
            if not isinstance(m, dict):
                raise SystemExit(f"rank {r} failed:\n{m}")
        ranks = [msgs[r] for r in range(args.world)]
        _log(f"ranks done in {time.time() - t0:.0f}s; merging the restatements")
        raws = [RawResults.read(os.path.join(shm, f"shard{r}_raw.bin")) for r in range(args.world)]
        g, ns, nf, first, cw, cells, bs, bf = merge_restatements(raws, [m["seq_base"] for m in ranks])
        m = np.load(os.path.join(shm, "merged.npz"))
        checks = {
            "global_counters": bool(np.array_equal(m["g"], g)),
            "nb_samples_found": (int(m["ns"]), int(m["nf"])) == (ns, nf),
            "first_ordinals": bool(np.array_equal(m["first"], first)),
            "count_weight": bool(np.array_equal(m["cw"], cw)),
            "page_cells": bool(np.array_equal(m["cells"], cells)),
            "buffer_counts": bool(np.array_equal(m["bs"], bs) and np.array_equal(m["bf"], bf)),
        }
    out = {"world": args.world, "records_per_rank": args.samples, "records_total": int(ns),
           "intervals": args.intervals, "matched_total": int(nf), "page_cells": int(cells.shape[0]),
           "bit_exact": all(checks.values()), "checks": checks,
           "payload_bytes_per_rank": [r["payload_bytes"] for r in ranks],
           "merge_s_rank0": ranks[0]["merge_s"], "analyze_s_rank0": ranks[0]["analyze_s"],
           "note": "all ranks share GPU 0 and merge over gloo (host staging): the timings are this "
                   "harness's, not an 8-GPU RCCL step; payload_bytes are what each rank sends",
           "ranks": ranks, "wall_s": time.time() - t0}
    print(json.dumps(out))
    if not out["bit_exact"]:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
