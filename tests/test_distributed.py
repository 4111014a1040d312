"""The merge algebra of the one-process-per-GPU path on CPU (world size 2 over
gloo, no GPU): each rank's partial counters for a contiguous, byte-balanced
shard (with its global seq_base) -- computed here by the oracle, since no
engine runs without a GPU -- are combined by the product's merge primitives
(reduce_u64 with the x ^ 2^63 order map for MIN/MAX, variable-length gathers,
merge_sparse) on rank 0, and the merged counters must give a report
byte-identical to a single unsharded run.  The same chain through the engine
itself (nmg_export_array -> reduce -> nmg_import_array) runs on the GPU in
tests/test_gpu_distributed.py."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, workdir, ret):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    import pyoracle
    from numamma_amd.distributed import gather_arrays, merge_sparse, reduce_u64, shard_ranges
    from numamma_amd.replay import Replay, SynthConfig, generate
    from numamma_amd.results import RawResults

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rp = generate(SynthConfig(nb_samples=60_000, nb_intervals=700, lost_frac=1e-3, seed=21))
    lens = [b.linear().shape[0] for b in rp.buffers]
    lo, hi = shard_ranges(lens, world)[rank]
    shard = Replay(rp.nb_threads, rp.table, rp.buffers[lo:hi])
    path = os.path.join(workdir, f"shard{rank}.bin")
    shard.write(path)
    pyoracle.run(path, os.path.join(workdir, f"o{rank}"), os.path.join(workdir, f"o{rank}.txt"),
                 os.path.join(workdir, f"raw{rank}.bin"))
    raw = RawResults.read(os.path.join(workdir, f"raw{rank}.bin"))
    E = raw.nb_entries
    first = raw.first_ordinal.copy()
    m = first != np.uint64(2**64 - 1)
    first[m] += np.uint64(lo) << np.uint64(32)  # shard-local -> global analysis position

    # the three u64 arrays, as an engine exports them
    g = raw.global_counters  # [2][75]: tc, tw, na, 18 x (count, min, max, sum)
    sums = [g[a, 0:3] for a in range(2)] + [np.stack([g[a, 3:][0::4], g[a, 3:][3::4]], axis=1).reshape(-1)
                                            for a in range(2)]
    sum64 = np.concatenate(sums + [raw.entries[:, 1:].reshape(-1)])
    min64 = np.concatenate([g[a, 3:][1::4] for a in range(2)] + [first])
    max64 = np.concatenate([g[a, 3:][2::4] for a in range(2)])
    t = {k: torch.from_numpy(v.astype(np.uint64).view(np.int64).copy()) for k, v in
         (("sum", sum64), ("min", min64), ("max", max64))}
    for op, tt in t.items():
        reduce_u64(tt, op, dst=0)
    cells = gather_arrays(raw.cells, dst=0)
    counts = gather_arrays(np.stack([raw.buf_samples, raw.buf_found]).astype(np.uint32), dst=0)
    if rank == 0:
        s = t["sum"].numpy().view(np.uint64)
        mn = t["min"].numpy().view(np.uint64)
        mx = t["max"].numpy().view(np.uint64)
        glob = np.zeros((2, 75), dtype=np.uint64)
        off = 0
        for a in range(2):
            glob[a, 0:3] = s[off:off + 3]
            off += 3
        for a in range(2):
            glob[a, 3:][0::4] = s[off:off + 36][0::2]
            glob[a, 3:][3::4] = s[off:off + 36][1::2]
            off += 36
            glob[a, 3:][1::4] = mn[18 * a:18 * a + 18]
            glob[a, 3:][2::4] = mx[18 * a:18 * a + 18]
        ent = np.zeros((E, 79), dtype=np.uint64)
        ent[:, 1:] = s[off:].reshape(E, 78)
        ent[:, 0] = mn[36:]
        # cells: merge as sparse (entry, thread, page) keys
        keys = [((c[:, 0].astype(np.uint64) << np.uint64(42)) | (c[:, 1].astype(np.uint64) << np.uint64(32))
                 | c[:, 2].astype(np.uint64), c[:, 3]) for c in cells]
        k, v = merge_sparse(keys)
        mc = np.stack([(k >> np.uint64(42)).astype(np.uint32), ((k >> np.uint64(32)) & np.uint64(0x3FF)).astype(np.uint32),
                       (k & np.uint64(0xFFFFFFFF)).astype(np.uint32), v], axis=1)
        allc = np.concatenate(counts, axis=1)
        merged = RawResults(E, allc.shape[1], raw.nb_threads, glob, 0, 0, allc[0], allc[1], ent, mc)
        ret.put(merged)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_merge_matches_single_run():
    import multiprocessing as mp

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import pyoracle
    from numamma_amd.replay import SynthConfig, generate
    from numamma_amd.results import report_host

    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, d, ret)) for r in range(2)]
        for p in procs:
            p.start()
        merged = ret.get(timeout=300)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        rp = generate(SynthConfig(nb_samples=60_000, nb_intervals=700, lost_frac=1e-3, seed=21))
        full = os.path.join(d, "full.bin")
        rp.write(full)
        pyoracle.run(full, os.path.join(d, "of"), os.path.join(d, "of.txt"), os.path.join(d, "of_raw.bin"))
        lens = np.array([x[2].shape[0] for x in rp.linear_buffers()], dtype=np.uint64)
        report_host(merged, rp.table, lens, os.path.join(d, "pm"), os.path.join(d, "pm.txt"))
        a = open(os.path.join(d, "of.txt"), "rb").read()
        b = open(os.path.join(d, "pm.txt"), "rb").read()
        if a != b:
            i = next((i for i in range(min(len(a), len(b))) if a[i] != b[i]), min(len(a), len(b)))
            pytest.fail(f"stdout differs at {i}:\n{a[max(0, i - 150):i + 80]!r}\n{b[max(0, i - 150):i + 80]!r}")
        for f in sorted(os.listdir(os.path.join(d, "of"))):
            a = open(os.path.join(d, "of", f), "rb").read()
            b = open(os.path.join(d, "pm", f), "rb").read()
            assert a == b, f


def test_shard_ranges_balanced_and_contiguous():
    from numamma_amd.distributed import shard_ranges

    rng = np.random.default_rng(0)
    lens = rng.integers(1000, 130_000, 500)
    for world in (1, 2, 3, 8):
        r = shard_ranges(lens, world)
        assert r[0][0] == 0 and r[-1][1] == 500
        assert all(r[i][1] == r[i + 1][0] for i in range(world - 1))
        tot = lens.sum()
        for lo, hi in r:
            assert abs(lens[lo:hi].sum() - tot / world) <= lens.max()


def test_u64_order_map():
    """MIN/MAX over uint64 through int64 reductions: x ^ 2^63 preserves order."""
    x = np.array([0, 1, 2**63 - 1, 2**63, 2**64 - 1, 12345], dtype=np.uint64)
    y = (x.view(np.int64) ^ np.int64(-(2**63)))
    order_u = np.argsort(x, kind="stable")
    order_i = np.argsort(y, kind="stable")
    assert np.array_equal(order_u, order_i)
