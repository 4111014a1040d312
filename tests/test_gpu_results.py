"""nmg_results_begin / nmg_results_end: the results snapshot copied to host
memory while the next analysis runs.  Its view must equal the synchronous
getters (themselves bit-exact against the oracle in the parity tests) at the
time of nmg_results_begin, even though the engine is reset and analyses
another workload before nmg_results_end."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from numamma_amd.replay import SynthConfig, generate  # noqa: E402

pytestmark = pytest.mark.gpu

CASES = {
    # attribute_kernel (small table)
    "k700": dict(nb_samples=200_000, nb_intervals=700, seed=21),
    # partition-first path, sparse cells of large objects and the [stack]
    "k60k": dict(nb_samples=300_000, nb_intervals=60_000, size_max=4 << 20, seed=22),
}


def _sync_results(eng):
    g, ns, nf = eng.global_counters()
    bs, bf = eng.buffer_counts()
    first, cw = eng.object_counters()
    return g, ns, nf, bs, bf, first, cw, eng.page_cells()


@pytest.mark.parametrize("case", sorted(CASES))
def test_results_snapshot_equals_getters(case):
    import torch
    from numamma_amd.engine import Engine

    rp = generate(SynthConfig(**CASES[case]))
    rp2 = generate(SynthConfig(**dict(CASES[case], seed=CASES[case]["seed"] + 100)))
    arena, offs, lens, ranks, acc = rp.packed()
    arena2, offs2, lens2, ranks2, acc2 = rp2.packed()
    d1 = torch.from_numpy(arena).cuda()
    d2 = torch.from_numpy(arena2).cuda()
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    for rep in range(3):  # (the second and third snapshots reuse the pinned buffers)
        eng.reset()
        eng.set_device_buffers(d1.data_ptr(), offs, lens, ranks, acc)
        eng.analyze()
        want = _sync_results(eng)
        eng.results_begin()
        # the next analysis at once: another workload on the same table
        eng.reset()
        eng.set_device_buffers(d2.data_ptr(), offs2, lens2, ranks2, acc2)
        eng.analyze()
        got = eng.results_end()
        names = ("global", "nb_samples", "nb_found", "buffer_samples", "buffer_found", "first_ordinal",
                 "count_weight", "cells")
        for name, x, y in zip(names, want, got):
            assert np.array_equal(np.asarray(x), np.asarray(y)), (rep, name)
        assert want[7].shape[0] > 0
    eng.synchronize()
    eng.close()


def test_page_cells_kept_buffers_across_tables():
    """The page-cell preparation keeps its device buffers across calls and
    tables (they only grow): one engine switched between a large and a small
    table must give the rows a fresh engine gives for each, and a repeated
    getter call the same rows again."""
    import torch
    from numamma_amd.engine import Engine

    rps = [generate(SynthConfig(**CASES[c])) for c in ("k60k", "k700", "k60k")]
    rps[2] = generate(SynthConfig(**dict(CASES["k60k"], seed=CASES["k60k"]["seed"] + 7)))
    nthr = max(rp.nb_threads for rp in rps)
    eng = Engine(nb_threads=nthr)
    for i, rp in enumerate(rps):
        arena, offs, lens, ranks, acc = rp.packed()
        d = torch.from_numpy(arena).cuda()
        eng.set_objects(rp.table)
        eng.reset()
        eng.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
        eng.analyze()
        got = eng.page_cells()
        again = eng.page_cells()
        fresh = Engine(nb_threads=nthr)
        fresh.set_objects(rp.table)
        fresh.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
        fresh.analyze()
        want = fresh.page_cells()
        fresh.close()
        assert want.shape[0] > 0, i
        assert np.array_equal(np.asarray(got), np.asarray(want)), i
        assert np.array_equal(np.asarray(again), np.asarray(want)), i
        eng.synchronize()
    eng.close()


def test_results_snapshot_errors_and_restart():
    """end without begin is a state error; a begin nobody ended is waited for
    by the next begin; a snapshot after set_buffer_counts (merged counts) is
    refused."""
    import torch
    from numamma_amd._lib import NmgError
    from numamma_amd.engine import Engine

    rp = generate(SynthConfig(**CASES["k700"]))
    arena, offs, lens, ranks, acc = rp.packed()
    d = torch.from_numpy(arena).cuda()
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
    with pytest.raises(NmgError):
        eng.results_end()
    eng.analyze()
    eng.results_begin()
    eng.results_begin()  # (the first one's copy waited for, its view dropped)
    got = eng.results_end()
    want = _sync_results(eng)
    assert all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(want, got))
    with pytest.raises(NmgError):
        eng.results_end()
    s, f = eng.buffer_counts()
    eng.set_buffer_counts(s, f, np.asarray(eng.buffer_bytes, dtype=np.uint64))
    with pytest.raises(NmgError):
        eng.results_begin()
    eng.close()


def test_results_snapshot_survives_table_switch():
    """A table switch between nmg_results_begin and nmg_results_end (ADVICE
    r5): the view is the begin-time analysis, its sparse rows placed with the
    begin-time table's sparse entries, even though nmg_set_objects replaced
    the table (different entry count and sparse entries) in between."""
    import torch
    from numamma_amd.engine import Engine

    rp = generate(SynthConfig(**CASES["k60k"]))
    rp2 = generate(SynthConfig(**dict(CASES["k60k"], nb_intervals=20_000, seed=123)))
    arena, offs, lens, ranks, acc = rp.packed()
    arena2, offs2, lens2, ranks2, acc2 = rp2.packed()
    d1 = torch.from_numpy(arena).cuda()
    d2 = torch.from_numpy(arena2).cuda()
    eng = Engine(nb_threads=max(rp.nb_threads, rp2.nb_threads))
    eng.set_objects(rp.table)
    eng.set_device_buffers(d1.data_ptr(), offs, lens, ranks, acc)
    eng.analyze()
    want = _sync_results(eng)
    assert want[7].shape[0] > 0
    eng.results_begin()
    eng.clear_buffers()
    eng.set_objects(rp2.table)
    eng.set_device_buffers(d2.data_ptr(), offs2, lens2, ranks2, acc2)
    eng.analyze()
    got = eng.results_end()
    names = ("global", "nb_samples", "nb_found", "buffer_samples", "buffer_found", "first_ordinal", "count_weight",
             "cells")
    for name, x, y in zip(names, want, got):
        assert np.array_equal(np.asarray(x), np.asarray(y)), name
    eng.synchronize()
    eng.close()
