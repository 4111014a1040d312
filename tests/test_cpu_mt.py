"""The multi-threaded C++ restatement (oracle/nmg_cpu_mt.cpp, bench.py's CPU
baseline) against the single-threaded oracle: byte-identical raw-results
dumps (global counters, per-buffer counts, per-entry counters and level
buckets, first-match ordinals, page cells) over the edge cases the GPU parity
tests use -- LOST records, a wrapped ring, reused and realloc'd addresses,
short buffers, 1 interval, 64 threads, huge ([stack]-sized) sparse objects --
for several thread counts (the split into buffer ranges must not matter)."""
import os

import pytest

import pyoracle
from numamma_amd.replay import SynthConfig, generate

CASES = [
    SynthConfig(nb_samples=60_000, nb_intervals=1_000, lost_frac=1e-3, wrap_one=True, seed=81),
    SynthConfig(nb_samples=40_000, nb_intervals=20, nb_threads=64, site_ratio=1.0, seed=82),
    SynthConfig(nb_samples=50_000, nb_intervals=3_000, reuse_frac=0.4, realloc_frac=0.2, frac_gap=0.3,
                buffer_records=97, seed=83),
    SynthConfig(nb_samples=20_000, nb_intervals=1, nb_globals=0, with_stack=False, buffer_records=10_000, seed=84),
    SynthConfig(nb_samples=30_000, nb_intervals=200_000, size_min=8, size_max=512, seed=85),
    # objects of 64 MiB - 4 GiB: page histograms beyond the dense limit (sparse cells)
    SynthConfig(nb_samples=30_000, nb_intervals=50, size_min=64 << 20, size_max=4 << 30, nb_threads=16, seed=86),
]


@pytest.mark.parametrize("cfg", CASES, ids=[f"mt{i}" for i in range(len(CASES))])
@pytest.mark.parametrize("threads", [1, 5])
def test_mt_restatement_matches_oracle(tmp_path, cfg, threads):
    d = str(tmp_path)
    path = os.path.join(d, "r.bin")
    generate(cfg).write(path)
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"))
    t = pyoracle.run_mt(path, os.path.join(d, "m_raw.bin"), threads=threads)
    assert t["nb_samples"] > 0
    assert open(os.path.join(d, "o_raw.bin"), "rb").read() == open(os.path.join(d, "m_raw.bin"), "rb").read()
