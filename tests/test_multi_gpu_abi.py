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
    eng.close()


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
