"""BASELINE configs at their stated sizes on one GPU, against the oracle.

* configs[2]: 100M records, 100k object intervals, per-page histogram on;
* configs[3]'s per-GPU shard: 125M records against the 1M-interval table
  (configs[3] is 1B records over 8 GPUs; a rank analyses 125M of them).

Both run the default product path (nmg_set_device_buffers + nmg_analyze,
flags NMG_F_DEFAULT) and compare with the oracle's raw dump: global
counters, per-buffer sample / match counts, every entry's first-match ordinal
and per-access count / weight, every non-zero (entry, thread, page) cell, and
the report files byte for byte.  At this size they also check the bounds the
small cases never reach (packed long-tail counters sized from the launch's
bytes, long-tail sub-log capacities, u32 per-buffer counts): any overflow
there would show up as a mismatch.  Size-independent properties are checked
as well: sum of per-entry counts == matched samples == sum of page cells.

The oracle's call-site sort is quadratic in the number of sites (it keeps the
reference's selection sort, mem_analyzer.c:1531-1557), so the configs use
fewer call sites than the generator's default."""
import os

import numpy as np
import pytest

import pyoracle
from numamma_amd import _lib
from numamma_amd.replay import SynthConfig, generate
from numamma_amd.results import RawResults

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _run(tmp_path, cfg):
    import torch
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(cfg)
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"))
    os.remove(path)
    raw = RawResults.read(os.path.join(d, "o_raw.bin"))
    arena, offs, lens, ranks, acc = rp.packed()
    dev = torch.from_numpy(arena).cuda()
    del arena
    eng = Engine(flags=_lib.NMG_F_DEFAULT, nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.set_device_buffers(dev.data_ptr(), offs, lens, ranks, acc)
    for _ in range(2):  # a second reset + analysis: nothing carries over
        eng.reset()
        eng.analyze()
    eng.synchronize()
    g, ns, nf = eng.global_counters()
    first, cw = eng.object_counters()
    nbs, nbf = eng.buffer_counts()
    cells = eng.page_cells()
    edir = os.path.join(d, "engine")
    eng.report(edir, os.path.join(d, "e.txt"))
    eng.close()
    assert ns == int(lens.sum()) // 40  # pure 40 B SAMPLE streams
    assert np.array_equal(g, raw.global_counters) and (ns, nf) == (raw.nb_samples, raw.nb_found)
    assert np.array_equal(nbs, raw.buf_samples) and np.array_equal(nbf, raw.buf_found)
    assert np.array_equal(first, raw.first_ordinal)
    assert np.array_equal(cw, raw.count_weight)
    assert np.array_equal(cells, raw.cells)
    # size-independent properties
    assert int(cw[:, :, 0].sum()) == nf
    assert int(cells[:, 3].astype(np.uint64).sum()) == nf  # every matched entry has dense cells here
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    fa, fb = sorted(os.listdir(odir)), sorted(os.listdir(edir))
    assert fa == fb
    for f in fa:
        assert open(os.path.join(odir, f), "rb").read() == open(os.path.join(edir, f), "rb").read(), f


def test_full_config3_bit_exact(tmp_path):
    """configs[2]: 100M records, 100k intervals, per-page histogram on."""
    _run(tmp_path, SynthConfig(nb_samples=100_000_000, nb_intervals=100_000, site_ratio=0.02, seed=43))


def test_config4_shard_bit_exact(tmp_path):
    """configs[3]'s per-GPU shard: 125M records, 1M intervals."""
    _run(tmp_path, SynthConfig(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024,
                               site_ratio=0.002, seed=44, sample_seed=1003))


def test_config4_shard_one_rank_rccl_handle(tmp_path):
    """The configs[3] shard through the multi-GPU handle's RCCL branch (a
    one-rank communicator on a one-GPU box, internal switch 0x40000): host
    buffers staged to the worker, the worker's analysis, the grouped
    ncclReduce of every dense array straight into the handle, the handle's
    gathers.  Every counter equals the bit-exact restatement
    (oracle/nmg_cpu_mt.cpp, pinned against the oracle in test_cpu_mt.py),
    after a reset + analysis as well as after the first one."""
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024,
                              site_ratio=0.002, seed=45, sample_seed=1004))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    pyoracle.run_mt(path, os.path.join(d, "mt_raw.bin"), threads=16, levels=False)
    os.remove(path)
    raw = RawResults.read(os.path.join(d, "mt_raw.bin"))
    eng = Engine(nb_threads=rp.nb_threads, flags=_lib.NMG_F_DEFAULT | 0x40000, copy_threads=16)
    eng.set_objects(rp.table)
    eng.submit_buffers(rp.linear_buffers())
    del rp
    for rep in range(2):
        eng.reset()
        eng.analyze()
        eng.synchronize()
        g, ns, nf = eng.global_counters()
        first, cw = eng.object_counters()
        nbs, nbf = eng.buffer_counts()
        cells = eng.page_cells()
        assert np.array_equal(g, raw.global_counters) and (ns, nf) == (raw.nb_samples, raw.nb_found), rep
        assert np.array_equal(nbs, raw.buf_samples) and np.array_equal(nbf, raw.buf_found), rep
        assert np.array_equal(first, raw.first_ordinal), rep
        assert np.array_equal(cw, raw.count_weight), rep
        assert np.array_equal(cells, raw.cells), rep
    eng.close()
