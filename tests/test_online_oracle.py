"""CPU checks of the --online-analysis restatement (no GPU): replay.table_at
and the oracle's alarm mode."""
import os

import numpy as np

import pyoracle
from numamma_amd.replay import SynthConfig, generate, online_alarms, table_at
from numamma_amd.results import RawResults


def test_table_at_snapshots():
    rp = generate(SynthConfig(nb_samples=2_000, nb_intervals=500, reuse_frac=0.3, with_stack=False, seed=81))
    t = rp.table
    ent = t.entries
    late = int(ent["free_date"].max()) + 1
    keys, off, ids, ent4 = table_at(t, late)  # everything allocated and freed
    assert np.array_equal(keys, t.keys) and np.array_equal(off, t.entry_off)
    assert np.array_equal(ids, np.arange(t.nb_entries))
    assert np.array_equal(ent4[:, 3], ent["free_date"])
    early = int(np.sort(ent["alloc_date"][ent["alloc_date"] > 0])[10])
    keys, off, ids, ent4 = table_at(t, early)
    assert np.all(ent["alloc_date"][ids] <= early)
    assert np.all(ent4[:, 3][ent["free_date"][ids] > early] == 0)  # alive: free_date 0
    assert np.all(np.diff(keys.astype(np.int64)) > 0) and off[-1] == ids.shape[0]
    for k in range(keys.shape[0]):  # newest-first order kept within each key
        assert np.all(np.diff(ids[off[k]:off[k + 1]].astype(np.int64)) > 0)


def test_oracle_single_final_alarm_counts_like_offline(tmp_path):
    """One alarm whose table is the final one: the same counters as the
    offline analysis (only the report's online form differs)."""
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=30_000, nb_intervals=800, with_stack=False, seed=82))
    path = os.path.join(d, "r.bin")
    rp.write(path)
    t = rp.table
    ent4 = np.stack([t.entries[f] for f in ("buffer_addr", "buffer_size", "alloc_date", "free_date")], axis=1)
    pyoracle.run(path, os.path.join(d, "off"), os.path.join(d, "off.txt"), os.path.join(d, "off.bin"))
    pyoracle.run(path, os.path.join(d, "on"), os.path.join(d, "on.txt"), os.path.join(d, "on.bin"),
                 alarms=[(len(rp.buffers), t.keys, t.entry_off, np.arange(t.nb_entries), ent4)])
    assert open(os.path.join(d, "off.bin"), "rb").read() == open(os.path.join(d, "on.bin"), "rb").read()
    on = open(os.path.join(d, "on.txt")).read()
    assert "Analyzing" not in on and "bytes processed" not in on
    assert "MEM ANALYZER" in on


def test_oracle_alarms_match_only_freed_objects(tmp_path):
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=40_000, nb_intervals=300, nb_threads=4, with_stack=False, reuse_frac=0.3,
                              buffer_records=300, seed=83))
    rp.buffers.reverse()
    snaps = [(be,) + table_at(rp.table, t) for be, t in online_alarms(rp, 4)]
    path = os.path.join(d, "r.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "on"), os.path.join(d, "on.txt"), os.path.join(d, "on.bin"), alarms=snaps)
    pyoracle.run(path, os.path.join(d, "off"), os.path.join(d, "off.txt"), os.path.join(d, "off.bin"))
    on, off = RawResults.read(os.path.join(d, "on.bin")), RawResults.read(os.path.join(d, "off.bin"))
    assert on.nb_samples == off.nb_samples
    assert 0 < on.nb_found < off.nb_found
    assert np.array_equal(on.global_counters, off.global_counters)  # update_counters does not depend on the table
