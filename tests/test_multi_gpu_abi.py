"""Multi-GPU behind the C-ABI (nmg_options.nb_gpus): one handle shards the
submitted buffers over several devices in contiguous byte-balanced ranges
(global analysis order kept through seq_base), replicates the table and merges
every worker's counters into the handle.  On a one-GPU box the workers share
the device, which takes the device-side merge; distinct devices take RCCL
reduces over xGMI (same arrays, same operators: u64 sum / min / max, u32 sum).
Reports and every counter equal the oracle's."""
import os

import numpy as np
import pytest

import pyoracle
from numamma_amd import _lib
from numamma_amd.replay import SynthConfig, generate
from numamma_amd.results import RawResults

pytestmark = pytest.mark.gpu


def _check(d, eng, rp, tag):
    raw = RawResults.read(os.path.join(d, "o_raw.bin"))
    g, ns, nf = eng.global_counters()
    first, cw = eng.object_counters()
    nbs, nbf = eng.buffer_counts()
    assert np.array_equal(g, raw.global_counters) and (ns, nf) == (raw.nb_samples, raw.nb_found), tag
    assert np.array_equal(nbs, raw.buf_samples) and np.array_equal(nbf, raw.buf_found), tag
    assert np.array_equal(first, raw.first_ordinal), tag
    assert np.array_equal(cw, raw.count_weight), tag
    assert np.array_equal(eng.page_cells(), raw.cells), tag


@pytest.mark.parametrize("nb_gpus,cfg", [
    (2, SynthConfig(nb_samples=200_000, nb_intervals=3_000, lost_frac=1e-3, wrap_one=True, seed=91)),
    (3, SynthConfig(nb_samples=150_000, nb_intervals=40_000, seed=92)),
    (4, SynthConfig(nb_samples=60_000, nb_intervals=400, seed=93)),
])
def test_multi_gpu_handle_bit_exact(tmp_path, nb_gpus, cfg):
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(cfg)
    path = os.path.join(d, "r.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"))
    eng = Engine(nb_threads=rp.nb_threads, devices=[0] * nb_gpus, hist_budget_bytes=(1 << 20) if nb_gpus == 4 else 0)
    eng.set_objects(rp.table)
    eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    _check(d, eng, rp, "first")
    eng.report(os.path.join(d, "e"), os.path.join(d, "e.txt"))
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    for f in sorted(os.listdir(os.path.join(d, "o"))):
        assert open(os.path.join(d, "o", f), "rb").read() == open(os.path.join(d, "e", f), "rb").read(), f
    eng.reset()  # reset + analyse again: the workers carry nothing over
    eng.analyze()
    eng.synchronize()
    _check(d, eng, rp, "second")
    # the merge of that analysis: timed on the root device, every counter array's bytes per worker
    from numamma_amd import _lib

    ms, payload = eng.merge_stats()
    assert ms > 0.0
    assert payload == 8 * sum(eng.array_size(a) for a in (_lib.NMG_ARR_SUM64, _lib.NMG_ARR_MIN64,
                                                         _lib.NMG_ARR_MAX64)) + 4 * eng.array_size(_lib.NMG_ARR_HIST32)
    eng.close()
    one = Engine(nb_threads=rp.nb_threads)  # a single-GPU engine merges nothing
    assert one.merge_stats() == (0.0, 0)
    one.close()


def test_multi_gpu_rejects_device_buffers():
    from numamma_amd.engine import Engine

    rp = generate(SynthConfig(nb_samples=1000, nb_intervals=10, seed=94))
    eng = Engine(nb_threads=rp.nb_threads, devices=[0, 0])
    eng.set_objects(rp.table)
    arena, offs, lens, ranks, acc = rp.packed()
    with pytest.raises(_lib.NmgError) as ei:
        eng.set_device_buffers(0x1000, offs, lens, ranks, acc)
    assert ei.value.code == -6  # NMG_ERR_STATE
    with pytest.raises(_lib.NmgError):
        eng.stream_begin()
    eng.close()


def _all(eng):
    g, ns, nf = eng.global_counters()
    first, cw = eng.object_counters()
    bs, bf = eng.buffer_counts()
    return [g, np.array([ns, nf]), first, cw, bs, bf, eng.page_cells()]


@pytest.mark.parametrize("devices,flags", [([0, 0], 0), (None, 0x40000)], ids=["two_shards", "one_rank_rccl"])
def test_multi_gpu_accumulates_like_one_engine(tmp_path, devices, flags):
    """Two analyses without a reset, then a third after nmg_synchronize: a
    multi-GPU handle accumulates every counter -- per-buffer sample / match
    counts included -- exactly like a one-GPU engine; after a reset one
    analysis equals the oracle.  `one_rank_rccl` (internal switch 0x40000) is
    a multi-GPU handle with one worker whose merge takes the distinct-device
    branch: librccl dlopen'ed, ncclCommInitAll over one device, the grouped
    ncclReduce of every array to the root, then the device add."""
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=150_000, nb_intervals=30_000, lost_frac=1e-3, seed=95))
    path = os.path.join(d, "r.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"))
    got = []
    for kind in ("multi", "single"):
        eng = (Engine(nb_threads=rp.nb_threads, devices=devices, flags=_lib.NMG_F_DEFAULT | flags) if kind == "multi"
               else Engine(nb_threads=rp.nb_threads))
        eng.set_objects(rp.table)
        eng.submit_replay(rp)
        eng.analyze()
        eng.analyze()
        eng.synchronize()
        eng.analyze()
        got.append(_all(eng))
        if kind == "multi":
            eng.reset()
            eng.analyze()
            eng.synchronize()
            _check(d, eng, rp, "after reset")
            eng.report(os.path.join(d, "e"), os.path.join(d, "e.txt"))
            assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
        eng.close()
    for a, b in zip(*got):
        assert np.array_equal(a, b)
    raw = RawResults.read(os.path.join(d, "o_raw.bin"))
    assert got[0][1][0] == 3 * raw.nb_samples and got[0][1][1] == 3 * raw.nb_found
