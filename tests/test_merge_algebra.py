"""The shard-merge algebra tools/merge8.py checks the 8-rank merge against:
per-shard oracle results merged in numpy (sums, minimums, maximums, page
rows summed by key, per-buffer counts concatenated, first-match ordinals
shifted by the shard's seq_base) equal the oracle's one run over every
shard's buffers in rank-major order (mem_sampling.c:324-342 over the whole
list).  CPU only: this pins the checker, the GPU run is the tool's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "oracle")]

import pyoracle  # noqa: E402
from merge8 import merge_restatements  # noqa: E402
from numamma_amd.replay import Replay, SynthConfig, generate  # noqa: E402
from numamma_amd.results import RawResults  # noqa: E402


def test_merge_restatements_equals_unsharded_oracle(tmp_path):
    d = str(tmp_path)
    shards = [generate(SynthConfig(nb_samples=60_000, nb_intervals=4_000, lost_frac=1e-3, seed=5, sample_seed=s))
              for s in (11, 12, 13)]
    raws, bases, buffers = [], [], []
    for i, rp in enumerate(shards):
        path = os.path.join(d, f"s{i}.bin")
        rp.write(path)
        pyoracle.run(path, os.path.join(d, f"o{i}"), os.path.join(d, f"o{i}.txt"), os.path.join(d, f"o{i}_raw.bin"))
        raws.append(RawResults.read(os.path.join(d, f"o{i}_raw.bin")))
        bases.append(len(buffers))
        buffers.extend(rp.buffers)
    whole = Replay(nb_threads=shards[0].nb_threads, table=shards[0].table, buffers=buffers)
    path = os.path.join(d, "whole.bin")
    whole.write(path)
    pyoracle.run(path, os.path.join(d, "ow"), os.path.join(d, "ow.txt"), os.path.join(d, "ow_raw.bin"))
    ref = RawResults.read(os.path.join(d, "ow_raw.bin"))
    g, ns, nf, first, cw, cells, bs, bf = merge_restatements(raws, bases)
    assert np.array_equal(g, ref.global_counters)
    assert (ns, nf) == (ref.nb_samples, ref.nb_found)
    assert np.array_equal(first, ref.first_ordinal)
    assert np.array_equal(cw, ref.count_weight)
    assert np.array_equal(cells, ref.cells)
    assert np.array_equal(bs, ref.buf_samples) and np.array_equal(bf, ref.buf_found)
