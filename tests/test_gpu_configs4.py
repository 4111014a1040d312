"""BASELINE configs[4] at its stated size: the online --alarm streaming shape
(pinned-host staging -> async H2D overlapped with the attribution kernel) fed
with the configs[1] data, 10M records against 1k object intervals.

At every alarm the reference's __process_samples (mem_sampling.c:929-966)
collects each thread's read ring and write ring; here each alarm's 2 x
nb_threads buffers go to nmg_submit_buffers while nmg_stream_begin's chunks
are uploaded on the copy stream and analysed as they fill.  Offline analysis
order (the buffers as the replay lists them) is kept, so the oracle's offline
run is the reference: raw counters, per-buffer tallies, first-match ordinals,
page cells, stdout and every report file byte for byte.  (The online table
at each alarm is covered by tests/test_gpu_online.py, up to 1.2M records.)"""
import os

import numpy as np
import pytest

import pyoracle
from numamma_amd.replay import SynthConfig, generate
from numamma_amd.results import RawResults

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _same_dirs(a, b):
    fa, fb = sorted(os.listdir(a)), sorted(os.listdir(b))
    assert fa == fb
    for f in fa:
        assert open(os.path.join(a, f), "rb").read() == open(os.path.join(b, f), "rb").read(), f


@pytest.mark.parametrize("chunk_mb,copy_threads", [(4, 4), (64, 8)])
def test_config4_full_c2_streamed_at_alarm_cadence(tmp_path, chunk_mb, copy_threads):
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=10_000_000, nb_intervals=1_000, lost_frac=1e-4, wrap_one=True, seed=42))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"))
    os.remove(path)
    raw = RawResults.read(os.path.join(d, "o_raw.bin"))
    lins = rp.linear_buffers()
    alarm = 2 * rp.nb_threads  # one read ring and one write ring per thread
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.stream_begin(chunk_bytes=chunk_mb << 20, copy_threads=copy_threads)
    for i in range(0, len(lins), alarm):
        eng.submit_buffers(lins[i:i + alarm])
    eng.analyze()
    eng.stream_end()
    eng.synchronize()
    g, ns, nf = eng.global_counters()
    assert ns == raw.nb_samples and ns > 9_900_000  # (LOST records are not samples)
    assert np.array_equal(g, raw.global_counters) and nf == raw.nb_found
    s, f = eng.buffer_counts()
    assert np.array_equal(s, raw.buf_samples) and np.array_equal(f, raw.buf_found)
    first, cw = eng.object_counters()
    assert np.array_equal(first, raw.first_ordinal) and np.array_equal(cw, raw.count_weight)
    assert np.array_equal(eng.page_cells(), raw.cells)
    edir = os.path.join(d, "engine")
    eng.report(edir, os.path.join(d, "e.txt"))
    eng.close()
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)


@pytest.mark.parametrize("nb_samples,chunk_mb", [(10_000_000, 32), (125_000_000, 256)], ids=["k1m", "c4shard"])
def test_config4_streamed_large_table_route_path(tmp_path, nb_samples, chunk_mb):
    """configs[4]'s streaming shape against the 1M-interval table: every
    streamed chunk takes the partition-first passes (route, count, plan,
    scatter, local, and its per-buffer matched counts at once, before the next
    chunk reuses the chunk pool).  `c4shard` streams the whole configs[3]
    per-GPU shard (125M records) at alarm cadence.  Every counter equals the
    bit-exact restatement (oracle/nmg_cpu_mt.cpp)."""
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=nb_samples, nb_intervals=1_000_000, size_max=64 * 1024, site_ratio=0.002,
                              lost_frac=1e-5, seed=46))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    pyoracle.run_mt(path, os.path.join(d, "mt_raw.bin"), threads=16, levels=False)
    os.remove(path)
    raw = RawResults.read(os.path.join(d, "mt_raw.bin"))
    lins = rp.linear_buffers()
    alarm = 2 * rp.nb_threads
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    del rp
    eng.stream_begin(chunk_bytes=chunk_mb << 20, copy_threads=16)
    for i in range(0, len(lins), alarm):
        eng.submit_buffers(lins[i:i + alarm])
    eng.analyze()
    eng.stream_end()
    eng.synchronize()
    g, ns, nf = eng.global_counters()
    assert ns == raw.nb_samples
    assert np.array_equal(g, raw.global_counters) and nf == raw.nb_found
    s, f = eng.buffer_counts()
    assert np.array_equal(s, raw.buf_samples) and np.array_equal(f, raw.buf_found)
    first, cw = eng.object_counters()
    assert np.array_equal(first, raw.first_ordinal) and np.array_equal(cw, raw.count_weight)
    assert np.array_equal(eng.page_cells(), raw.cells)
    _, rest = eng.phase_times(8)  # (the local pass ran after every recent chunk's route pass)
    assert rest and all(r > 0 for r in rest)
    eng.close()
