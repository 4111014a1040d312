"""The one-process-per-GPU merge through the product: two ranks (gloo, both on
GPU 0 of the test box) each analyse a contiguous byte-balanced shard of the
buffer list with its seq_base, then merge_engine runs the engine's
nmg_export_array -> reduce_u64 / reduce_u32_sum -> nmg_import_array chain and
the sparse / per-buffer gathers; rank 0 reports.  The merged counters and
every report file must equal the oracle's single unsharded run.  `packed`
merges the page histogram through nmg_hist_pack / nmg_hist_unpack (bytes of
the cells <= 255 / world summed as u8, the larger cells gathered)."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

CFGS = {
    "k700": dict(nb_samples=200_000, nb_intervals=700, lost_frac=1e-3, seed=21),
    # large-table path, hashed objects, cell log, [stack] sparse cells
    "k60k": dict(nb_samples=300_000, nb_intervals=60_000, seed=22),
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, workdir, cfg_name, ret, packed=False, before=None):
    """before: a configuration analysed and merged first on the same engines,
    whose table is then replaced by cfg_name's (a larger one: the merge's
    cached packers must be rebuilt for the new entry count)."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    try:
        import torch
        import torch.distributed as dist

        from numamma_amd.distributed import merge_engine, shard_ranges
        from numamma_amd.engine import Engine
        from numamma_amd.replay import SynthConfig, generate

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        eng = None
        keep = []
        for name in ([before] if before else []) + [cfg_name]:
            rp = generate(SynthConfig(**CFGS[name]))
            arena, offs, lens, ranks, acc = rp.packed()
            lo, hi = shard_ranges(lens, world)[rank]
            base = int(offs[lo]) if hi > lo else 0
            end = int(offs[hi - 1] + lens[hi - 1]) if hi > lo else 0
            d_arena = torch.from_numpy(arena[base:end].copy()).to(dev)
            keep.append(d_arena)
            if eng is None:
                eng = Engine(device=0, nb_threads=rp.nb_threads)
            else:
                eng.clear_buffers()
            eng.set_objects(rp.table)
            eng.set_device_buffers(d_arena.data_ptr(), offs[lo:hi] - base, lens[lo:hi], ranks[lo:hi], acc[lo:hi],
                                   seq_base=lo)
            for rep in range(2 if packed else 1):  # (packed: a second job on the same engines, reset in between
                if rep:                             # -- rank 0 drops the first merge's per-buffer counts)
                    eng.reset()
                eng.analyze()
                eng.synchronize()
                merge_engine(eng, dst=0, device=dev, packed_hist=packed)
            if name != cfg_name:
                eng.reset()
        if rank == 0:
            edir = os.path.join(workdir, "engine")
            eng.report(edir, os.path.join(workdir, "e.txt"))
            g, ns, nf = eng.global_counters()
            first, cw = eng.object_counters()
            np.savez(os.path.join(workdir, "merged.npz"), g=g, ns=ns, nf=nf, first=first, cw=cw,
                     cells=eng.page_cells())
        eng.close()
        dist.barrier()
        dist.destroy_process_group()
        ret.put((rank, "ok"))
    except Exception as e:  # surfaced by the parent
        import traceback

        ret.put((rank, traceback.format_exc()))
        raise


@pytest.mark.parametrize("packed", [False, True], ids=["dense", "packed"])
@pytest.mark.parametrize("cfg_name", sorted(CFGS))
def test_two_rank_engine_merge_matches_oracle(cfg_name, packed):
    _two_rank(cfg_name, packed)


def test_two_rank_packed_merge_after_table_grew():
    """Two packed merges on the same engines, the table grown from 700 to
    60k intervals in between (the per-object packer must follow
    the entry count, not write past its buffer)."""
    _two_rank("k60k", True, before="k700")


def _two_rank(cfg_name, packed, before=None):
    import multiprocessing as mp

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import pyoracle
    from numamma_amd.replay import SynthConfig, generate
    from numamma_amd.results import RawResults

    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, d, cfg_name, ret, packed, before)) for r in range(2)]
        for p in procs:
            p.start()
        msgs = [ret.get(timeout=240) for _ in procs]
        for p in procs:
            p.join(timeout=60)
        for rank, msg in msgs:
            assert msg == "ok", f"rank {rank}:\n{msg}"
        assert all(p.exitcode == 0 for p in procs)
        rp = generate(SynthConfig(**CFGS[cfg_name]))
        full = os.path.join(d, "full.bin")
        rp.write(full)
        pyoracle.run(full, os.path.join(d, "oracle"), os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"))
        raw = RawResults.read(os.path.join(d, "o_raw.bin"))
        m = np.load(os.path.join(d, "merged.npz"))
        assert np.array_equal(m["g"], raw.global_counters)
        assert (int(m["ns"]), int(m["nf"])) == (raw.nb_samples, raw.nb_found)
        assert np.array_equal(m["first"], raw.first_ordinal)
        assert np.array_equal(m["cw"], raw.count_weight)
        assert np.array_equal(m["cells"], raw.cells)
        assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
        for f in sorted(os.listdir(os.path.join(d, "oracle"))):
            assert open(os.path.join(d, "oracle", f), "rb").read() == \
                open(os.path.join(d, "engine", f), "rb").read(), f


@pytest.mark.parametrize("threshold,threads", [(0, 8), (1, 8), (31, 8), (127, 8), (255, 8), (1, 3), (31, 7)])
def test_hist_pack_round_trip(threshold, threads):
    """nmg_hist_pack then nmg_hist_unpack on one engine gives back every
    page cell (bytes <= threshold + overflow list, in cell order); a list
    longer than its capacity reports its full length.  Odd thread counts give
    cell counts that are not a multiple of 4 (the partial last quad)."""
    import torch

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    from numamma_amd import _lib
    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    rp = generate(SynthConfig(nb_samples=400_000, nb_intervals=20_000, nb_threads=threads, seed=23))
    eng = Engine(device=0, nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    cells = eng.array_size(_lib.NMG_ARR_HIST32)
    dev = torch.device("cuda", 0)
    before = torch.empty(cells, dtype=torch.int32, device=dev)
    eng.export_array(_lib.NMG_ARR_HIST32, before.data_ptr())
    ref = before.cpu().numpy().view(np.uint32)
    u8 = torch.empty(cells, dtype=torch.uint8, device=dev)
    ovf = torch.zeros(cells, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)  # (the fill is on torch's stream; hist_pack writes on the engine's)
    n = eng.hist_pack(threshold, u8.data_ptr(), ovf.data_ptr(), cells)
    assert n == int((ref > threshold).sum())
    b = u8.cpu().numpy()
    assert np.array_equal(b, np.where(ref <= threshold, ref, 0).astype(np.uint8))
    big = np.nonzero(ref > threshold)[0].astype(np.uint64)
    want = (big << np.uint64(32)) | ref[big].astype(np.uint64)
    assert np.array_equal(ovf[:n].cpu().numpy().view(np.uint64), want)
    if n > 1:
        assert eng.hist_pack(threshold, u8.data_ptr(), ovf.data_ptr(), n - 1) == n  # (capacity short)
        eng.hist_pack(threshold, u8.data_ptr(), ovf.data_ptr(), cells)
    eng.hist_unpack(u8.data_ptr(), ovf.data_ptr(), n)
    after = torch.empty(cells, dtype=torch.int32, device=dev)
    eng.export_array(_lib.NMG_ARR_HIST32, after.data_ptr())
    assert np.array_equal(after.cpu().numpy().view(np.uint32), ref)
    eng.close()


@pytest.mark.parametrize("threshold", [1, 7, 1000, 1 << 32])
def test_objcw_pack_round_trip(threshold):
    """nmg_objcw_pack then nmg_objcw_unpack on one sum64 image gives back the
    per-object count / weight rows: values below the threshold as u32 words,
    the others as (row word, value) pairs; a list longer than its capacity
    reports its full length; the global sums ahead of the rows are not
    touched."""
    import torch

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    from numamma_amd import _lib
    from numamma_amd.distributed import GLOBAL_SUM_WORDS
    from numamma_amd.engine import Engine
    from numamma_amd.replay import SynthConfig, generate

    rp = generate(SynthConfig(nb_samples=300_000, nb_intervals=20_000, seed=24))
    eng = Engine(device=0, nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    dev = torch.device("cuda", 0)
    n = eng.array_size(_lib.NMG_ARR_SUM64)
    t = torch.empty(n, dtype=torch.int64, device=dev)
    eng.export_array(_lib.NMG_ARR_SUM64, t.data_ptr())
    ref = t.cpu().numpy().view(np.uint64).copy()
    E = (n - GLOBAL_SUM_WORDS) // 4
    rows = ref[GLOBAL_SUM_WORDS:GLOBAL_SUM_WORDS + 4 * E]
    u32 = torch.empty(4 * E, dtype=torch.int32, device=dev)
    cap = 4 * E
    ovf = torch.empty(2 * cap, dtype=torch.int64, device=dev)
    nb = eng.objcw_pack(t.data_ptr(), threshold, u32.data_ptr(), ovf.data_ptr(), cap)
    big = rows >= np.uint64(threshold)
    assert nb == int(big.sum())
    assert np.array_equal(u32.cpu().numpy().view(np.uint32), np.where(big, 0, rows).astype(np.uint32))
    pairs = ovf[:2 * nb].cpu().numpy().view(np.uint64).reshape(-1, 2)
    order = np.argsort(pairs[:, 0])
    assert np.array_equal(pairs[order, 0], np.nonzero(big)[0].astype(np.uint64))
    assert np.array_equal(pairs[order, 1], rows[big])
    if nb > 1:
        assert eng.objcw_pack(t.data_ptr(), threshold, u32.data_ptr(), ovf.data_ptr(), nb - 1) == nb  # (short)
        eng.objcw_pack(t.data_ptr(), threshold, u32.data_ptr(), ovf.data_ptr(), cap)
    t[GLOBAL_SUM_WORDS:].fill_(-1)  # the rows rebuilt from the words and the list alone
    torch.cuda.synchronize(dev)
    eng.objcw_unpack(t.data_ptr(), u32.data_ptr(), ovf.data_ptr(), nb)
    assert np.array_equal(t.cpu().numpy().view(np.uint64), ref)
    eng.close()
