"""--online-analysis parity (mem_sampling.c:929-966, branch :953-954): every
alarm's rings are attributed against the object table as it stands at that
alarm -- objects not yet allocated are absent, live ones carry free_date 0 and
never match (quirk Q3) -- and the counters accumulate across alarms; the
report is ma_finalize's online one (no finalize lines, every object reaches
update_call_sites).  The engine gets each alarm's table through
nmg_update_objects while it streams; the oracle replays the same alarms
(replay.table_at).  Bit-exact: raw counters, per-buffer tallies, page cells,
stdout, call_sites.log and every callsite_counters_<id>.dat."""
import os

import numpy as np
import pytest

import pyoracle
from numamma_amd import _lib
from numamma_amd.replay import SynthConfig, generate, online_alarms, table_at
from numamma_amd.results import RawResults

pytestmark = pytest.mark.gpu

CASES = [
    # small table (LDS Eytzinger path), address reuse: entries appear and are freed mid-run
    (SynthConfig(nb_samples=120_000, nb_intervals=400, nb_threads=4, with_stack=False, reuse_frac=0.3,
                 buffer_records=300, seed=71), 6, 1 << 20),
    # large table (fences + directory), one chunk per alarm and several
    (SynthConfig(nb_samples=200_000, nb_intervals=30_000, nb_threads=8, with_stack=False, reuse_frac=0.2,
                 realloc_frac=0.05, buffer_records=500, seed=72), 5, 256 << 10),
    # a single alarm at the end: every object freed by then matches as offline would
    (SynthConfig(nb_samples=60_000, nb_intervals=2_000, nb_threads=2, with_stack=False, buffer_records=400,
                 seed=73), 1, 4 << 20),
    # configs[4] scale: 1.2M records over 48 alarms, 20k intervals (large-table lookup), reuse + realloc
    (SynthConfig(nb_samples=1_200_000, nb_intervals=20_000, nb_threads=8, with_stack=False, reuse_frac=0.2,
                 realloc_frac=0.05, buffer_records=1_000, seed=76), 48, 1 << 20),
]


def _ent_objs(ent4):
    objs = np.zeros(ent4.shape[0], dtype=[("a", "<u8"), ("s", "<u8"), ("al", "<u8"), ("fr", "<u8")])
    objs["a"], objs["s"], objs["al"], objs["fr"] = ent4[:, 0], ent4[:, 1], ent4[:, 2], ent4[:, 3]
    return objs


def _same_dirs(a, b):
    fa, fb = sorted(os.listdir(a)), sorted(os.listdir(b))
    assert fa == fb
    for f in fa:
        assert open(os.path.join(a, f), "rb").read() == open(os.path.join(b, f), "rb").read(), f


@pytest.mark.parametrize("cfg,nb_alarms,chunk", CASES, ids=["k400", "k30k", "one_alarm", "m1_48_alarms"])
def test_online_analysis_bit_exact(tmp_path, cfg, nb_alarms, chunk):
    from numamma_amd.engine import Engine, table_objects

    d = str(tmp_path)
    rp = generate(cfg)
    rp.buffers.reverse()  # online: rings are analysed as they are collected, oldest first
    alarms = online_alarms(rp, nb_alarms)
    snaps = [(be,) + table_at(rp.table, t) for be, t in alarms]
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"), alarms=snaps)
    raw = RawResults.read(os.path.join(d, "o_raw.bin"))
    assert raw.nb_found > 0  # objects freed before an alarm did match

    eng = Engine(flags=_lib.NMG_F_DEFAULT, nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)  # the final table: ids, page cells, report metadata
    eng.stream_begin(chunk_bytes=chunk, copy_threads=2)
    b0 = 0
    for be, keys, off, ids, ent4 in snaps:
        eng.update_objects(keys, off, ids, _ent_objs(ent4))
        for b in rp.buffers[b0:be]:
            eng.submit_ring(b.ring, b.data_tail, b.data_head, b.thread_rank, b.access_type)
        b0 = be
    eng.analyze()
    eng.stream_end()
    eng.synchronize()
    if cfg.nb_intervals > 10_000:  # large alarm tables take the partition-first path
        assert eng.route_count() > 0
    # at exit: the table ma_finalize walks (the report's objects and order)
    t = rp.table
    eng.update_objects(t.keys, t.entry_off, np.arange(t.nb_entries, dtype=np.uint32), table_objects(t))
    g, ns, nf = eng.global_counters()
    assert np.array_equal(g, raw.global_counters) and (ns, nf) == (raw.nb_samples, raw.nb_found)
    s, f = eng.buffer_counts()
    assert np.array_equal(s, raw.buf_samples) and np.array_equal(f, raw.buf_found)
    first, cw = eng.object_counters()
    assert np.array_equal(first, raw.first_ordinal)
    assert np.array_equal(cw, raw.count_weight)
    assert np.array_equal(eng.page_cells(), raw.cells)
    edir = os.path.join(d, "engine")
    eng.report(edir, os.path.join(d, "e.txt"), online=True)
    eng.close()
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)


def test_online_table_updates_keep_counters(tmp_path):
    """Updating to the same table between analyses changes nothing: the
    counters of one stream equal those of the stream split by updates."""
    from numamma_amd.engine import Engine, table_objects

    rp = generate(SynthConfig(nb_samples=80_000, nb_intervals=3_000, seed=74))
    t = rp.table
    lins = rp.linear_buffers()
    res = []
    for split in (False, True):
        eng = Engine(nb_threads=rp.nb_threads)
        eng.set_objects(t)
        eng.stream_begin(chunk_bytes=1 << 20, copy_threads=1)
        for i, (r, a, data) in enumerate(lins):
            if split and i % 7 == 0:
                eng.update_objects(t.keys, t.entry_off, np.arange(t.nb_entries, dtype=np.uint32), table_objects(t))
            eng.submit_buffer(data, r, a)
        eng.analyze()
        eng.stream_end()
        eng.synchronize()
        res.append((eng.global_counters()[0], eng.object_counters()[1], eng.page_cells()))
        eng.close()
    for a, b in zip(*res):
        assert np.array_equal(a, b)


def test_update_objects_rejects_bad_tables(tmp_path):
    from numamma_amd.engine import Engine, table_objects

    rp = generate(SynthConfig(nb_samples=1_000, nb_intervals=50, seed=75))
    t = rp.table
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(t)
    ids = np.arange(t.nb_entries, dtype=np.uint32)
    objs = table_objects(t)
    bad = ids.copy()
    bad[3] = t.nb_entries + 1  # a new id, but not the next one (t.nb_entries is missing)
    with pytest.raises(RuntimeError):
        eng.update_objects(t.keys, t.entry_off, bad, objs)
    bad = ids.copy()
    bad[3] = bad[4]  # one id twice
    with pytest.raises(RuntimeError):
        eng.update_objects(t.keys, t.entry_off, bad, objs)
    big = objs.copy()
    big["s"][5] += 1 << 20  # larger than its page cells: they move to a larger range
    eng.update_objects(t.keys, t.entry_off, ids, big)
    eng.update_objects(t.keys[:0], np.zeros(1, dtype=np.uint32), ids[:0], objs[:0])  # empty table at an alarm
    with pytest.raises(RuntimeError):  # dump modes read the NULL `samples` list online in the reference
        eng.report(str(tmp_path), os.path.join(str(tmp_path), "x.txt"), dump_flags=_lib.NMG_DUMP_ALL, online=True)
    eng.close()


def _creation_ids(table):
    """Live ids: objects numbered in creation order (alloc date, then table
    position), as _init_mem_info's next_mem_info_id hands them out
    (mem_analyzer.c:567-568); cid[table position] = id."""
    ent = table.entries
    order = np.lexsort((np.arange(table.nb_entries), ent["alloc_date"]))
    cid = np.empty(table.nb_entries, dtype=np.uint32)
    cid[order] = np.arange(table.nb_entries, dtype=np.uint32)
    return cid


LIVE_CASES = [
    (SynthConfig(nb_samples=150_000, nb_intervals=600, nb_threads=4, with_stack=False, reuse_frac=0.3,
                 buffer_records=300, seed=81), 7, 1 << 20),
    # hashed object counters (> 2048 entries by the end) and the large-table lookup
    (SynthConfig(nb_samples=400_000, nb_intervals=20_000, nb_threads=8, with_stack=False, reuse_frac=0.2,
                 realloc_frac=0.05, buffer_records=800, seed=82), 12, 512 << 10),
]


@pytest.mark.parametrize("cfg,nb_alarms,chunk", LIVE_CASES, ids=["k600", "k20k"])
def test_online_live_tables_bit_exact(tmp_path, cfg, nb_alarms, chunk):
    """A live host: the engine never sees the final
    table before the last alarm.  It starts from an empty table; each alarm's
    table brings the objects created since (ids in creation order, counters
    from creation) and objects that grew (every third object is half its
    final size until it is freed: ma_record_free stamps the final size,
    mem_analyzer.c:1287); at exit the finalize table gives the report its
    objects and order.  The oracle replays the same alarm tables with
    final-table ids: reports byte-identical, raw counters equal through the
    id map."""
    from numamma_amd.engine import Engine, table_objects
    from numamma_amd.replay import ObjectTable

    d = str(tmp_path)
    rp = generate(cfg)
    rp.buffers.reverse()
    alarms = online_alarms(rp, nb_alarms)
    final = rp.table
    grows = (np.arange(final.nb_entries) % 3) == 0
    snaps = []
    for be, t in alarms:
        keys, off, ids, ent4 = table_at(final, t)
        ent4 = ent4.copy()
        live = (ent4[:, 3] == 0) & grows[ids]
        ent4[live, 1] = ent4[live, 1] // 2  # size before ma_record_free
        snaps.append((be, keys, off, ids, ent4))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"), alarms=snaps)
    raw = RawResults.read(os.path.join(d, "o_raw.bin"))
    assert raw.nb_found > 0

    cid = _creation_ids(final)
    eng = Engine(flags=_lib.NMG_F_DEFAULT, nb_threads=rp.nb_threads)
    eng.set_objects(ObjectTable.empty())  # no objects yet
    eng.stream_begin(chunk_bytes=chunk, copy_threads=2)
    b0 = 0
    for be, keys, off, ids, ent4 in snaps:
        eng.update_objects(keys, off, cid[ids], _ent_objs(ent4))
        for b in rp.buffers[b0:be]:
            eng.submit_ring(b.ring, b.data_tail, b.data_head, b.thread_rank, b.access_type)
        b0 = be
    eng.analyze()
    eng.stream_end()
    eng.synchronize()
    if cfg.nb_intervals > 10_000:  # partitions over ids in creation order (an id map)
        assert eng.route_count() > 0
    eng.update_objects(final.keys, final.entry_off, cid, table_objects(final))  # ma_finalize's table
    eng.table = final  # the report's metadata, in the finalize table's order
    g, ns, nf = eng.global_counters()
    assert np.array_equal(g, raw.global_counters) and (ns, nf) == (raw.nb_samples, raw.nb_found)
    s, f = eng.buffer_counts()
    assert np.array_equal(s, raw.buf_samples) and np.array_equal(f, raw.buf_found)
    first, cw = eng.object_counters()
    assert np.array_equal(first[cid], raw.first_ordinal)
    assert np.array_equal(cw[cid], raw.count_weight)
    cells = eng.page_cells().copy()
    pos = np.empty_like(cid)
    pos[cid] = np.arange(cid.shape[0], dtype=np.uint32)
    cells[:, 0] = pos[cells[:, 0]]
    cells = cells[np.lexsort((cells[:, 2], cells[:, 1], cells[:, 0]))]
    assert np.array_equal(cells, raw.cells)
    edir = os.path.join(d, "engine")
    eng.report(edir, os.path.join(d, "e.txt"), online=True)
    eng.close()
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)


def test_failed_growth_keeps_state(tmp_path):
    """nmg_update_objects that would grow an object past the page-histogram
    budget fails with NMG_ERR_CAPACITY and leaves the engine as it was: the
    analysis after it, nmg_get_page_cells and nmg_report equal an engine that
    never saw the update."""
    from numamma_amd.engine import Engine, table_objects

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=60_000, nb_intervals=2_000, with_stack=False, seed=78))
    t = rp.table
    ids = np.arange(t.nb_entries, dtype=np.uint32)
    objs = table_objects(t)
    cells = int((t.entries["buffer_size"] // 4096 + 1).sum())
    budget = (cells + 8) * rp.nb_threads * 4  # every object dense, no room to grow one by 1 MiB
    outs = []
    for fail_first in (True, False):
        eng = Engine(nb_threads=rp.nb_threads, hist_budget_bytes=budget)
        eng.set_objects(t)
        if fail_first:
            big = objs.copy()
            big["s"][5] += 1 << 20
            with pytest.raises(_lib.NmgError) as ei:
                eng.update_objects(t.keys, t.entry_off, ids, big)
            assert ei.value.code == -8  # NMG_ERR_CAPACITY
        eng.submit_replay(rp)
        eng.analyze()
        eng.synchronize()
        edir = os.path.join(d, f"e{int(fail_first)}")
        eng.report(edir, os.path.join(d, f"e{int(fail_first)}.txt"))
        outs.append((eng.page_cells().copy(), eng.object_counters()[1].copy(), edir))
        eng.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert open(os.path.join(d, "e1.txt"), "rb").read() == open(os.path.join(d, "e0.txt"), "rb").read()
    _same_dirs(outs[0][2], outs[1][2])


def test_partial_update_after_permuted_table(tmp_path):
    """A live table listing every entry in a non-identity order, then a
    partial table that brings new objects: the report walks the known entries
    in the first table's order and the new ones after them (the walk order
    always covers every entry)."""
    from numamma_amd.engine import Engine, table_objects
    from numamma_amd.replay import ObjectTable

    rp = generate(SynthConfig(nb_samples=40_000, nb_intervals=500, with_stack=False, seed=79))
    t = rp.table
    E = t.nb_entries
    objs = table_objects(t)
    perm = np.random.default_rng(79).permutation(E).astype(np.uint32)
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(ObjectTable.empty())
    eng.update_objects(t.keys, t.entry_off, perm, objs)  # every entry, ids permuted
    # two new objects past the table (ids E, E + 1), one key each
    top = int(t.keys[-1]) + (1 << 30)
    keys = np.array([top, top + (1 << 20)], dtype=np.uint64)
    new = np.zeros(2, dtype=objs.dtype)
    new["a"], new["s"], new["al"], new["fr"] = keys, 4096, 1, 2
    eng.update_objects(keys, np.array([0, 1, 2], dtype=np.uint32), np.array([E, E + 1], dtype=np.uint32), new)
    eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    # the report's metadata in walk order: the table's entries, then the two new objects
    ent = np.concatenate([t.entries, t.entries[:2].copy()])
    ent["buffer_addr"][E:] = keys
    ent["buffer_size"][E:] = 4096
    ent["initial_buffer_size"][E:] = 4096
    ent["alloc_date"][E:], ent["free_date"][E:] = 1, 2
    eng.table = ObjectTable(np.concatenate([t.keys, keys]), np.concatenate([t.entry_off, [E + 1, E + 2]]).astype(np.uint32),
                            ent, t.callstack_pool, t.string_pool)
    eng.report(str(tmp_path), os.path.join(str(tmp_path), "x.txt"), online=True)
    assert os.path.exists(os.path.join(str(tmp_path), "call_sites.log"))
    g, ns, nf = eng.global_counters()
    assert ns > 0
    eng.close()


def test_online_route_matches_single_pass():
    """A large table given through nmg_update_objects with permuted ids (a
    partition's table positions map to scattered entry ids and page cells):
    the partition-first path and the single-pass kernel give the same
    counters, page cells and per-buffer counts, older entries of reused
    addresses included."""
    from numamma_amd.engine import Engine, table_objects
    from numamma_amd.replay import ObjectTable

    rp = generate(SynthConfig(nb_samples=400_000, nb_intervals=60_000, reuse_frac=0.3, realloc_frac=0.1, seed=83))
    t = rp.table
    perm = np.random.default_rng(83).permutation(t.nb_entries).astype(np.uint32)
    out = []
    for flags in (_lib.NMG_F_DEFAULT, _lib.NMG_F_DEFAULT | 0x10000):  # (internal 0x10000: no partition-first path)
        eng = Engine(flags=flags, nb_threads=rp.nb_threads)
        eng.set_objects(ObjectTable.empty())
        eng.update_objects(t.keys, t.entry_off, perm, table_objects(t))
        eng.submit_replay(rp)
        eng.analyze()
        eng.synchronize()
        g, ns, nf = eng.global_counters()
        first, cw = eng.object_counters()
        bs, bf = eng.buffer_counts()
        out.append(((g, ns, nf, first, cw, bs, bf, eng.page_cells().copy()), eng.route_count()))
        eng.close()
    (a, na), (b, nb) = out
    assert na > 0 and nb == 0
    assert a[2] > 0
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x), np.asarray(y))
