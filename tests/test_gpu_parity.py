"""Parity of the HIP engine (through the C-ABI) with the CPU oracle.

Bit-exact: every counter of the canonical raw-results dump, the stdout
report, call_sites.log and every callsite_counters_<id>.dat -- on seeded
synthetic replays (edge cases included), on the README fixture, at the full
configs[1] size (10M samples, 1k intervals), through the device-resident
entry point, and through a sharded two-engine merge."""
import os

import numpy as np
import pytest

import pyoracle
import readme_fixture
from numamma_amd import _lib
from numamma_amd.replay import RECORD_DTYPE, SynthConfig, generate
from numamma_amd.results import RawResults, report_host

pytestmark = pytest.mark.gpu


def _oracle(rp, d):
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "oracle_stdout.txt"), os.path.join(d, "oracle_raw.bin"))
    return path, odir


def _engine_replay(path, d, flags=_lib.NMG_F_DEFAULT):
    from numamma_amd.engine import run_replay

    edir = os.path.join(d, "engine")
    run_replay(path, edir, os.path.join(d, "engine_stdout.txt"), os.path.join(d, "engine_raw.bin"), flags=flags)
    return edir


def _same_dirs(a, b):
    fa, fb = sorted(os.listdir(a)), sorted(os.listdir(b))
    assert fa == fb
    for f in fa:
        assert open(os.path.join(a, f), "rb").read() == open(os.path.join(b, f), "rb").read(), f


def _assert_raw_equal(pa, pb):
    a, b = RawResults.read(pa), RawResults.read(pb)
    assert np.array_equal(a.global_counters, b.global_counters)
    assert (a.nb_samples, a.nb_found) == (b.nb_samples, b.nb_found)
    assert np.array_equal(a.buf_samples, b.buf_samples) and np.array_equal(a.buf_found, b.buf_found)
    assert np.array_equal(a.entries, b.entries)
    assert np.array_equal(a.cells, b.cells)
    assert open(pa, "rb").read() == open(pb, "rb").read()


CONFIGS = [
    SynthConfig(nb_samples=200_000, nb_intervals=1_000, seed=1),
    SynthConfig(nb_samples=100_000, nb_intervals=5_000, nb_threads=5, lost_frac=1e-3, wrap_one=True, seed=2),
    SynthConfig(nb_samples=50_000, nb_intervals=20, nb_threads=64, site_ratio=1.0, seed=3),
    SynthConfig(nb_samples=80_000, nb_intervals=3_000, reuse_frac=0.4, realloc_frac=0.2, frac_gap=0.3,
                buffer_records=97, seed=4),
    SynthConfig(nb_samples=30_000, nb_intervals=1, nb_globals=0, with_stack=False, buffer_records=10_000, seed=5),
    SynthConfig(nb_samples=60_000, nb_intervals=200_000, size_min=8, size_max=512, seed=6),
    # 1M intervals (configs[3]'s table): fences + per-bucket directory lookup.
    # Few call sites: the reference's site list and sort are quadratic (the oracle keeps that cost)
    SynthConfig(nb_samples=300_000, nb_intervals=1_000_000, size_max=64 * 1024, site_ratio=0.002, seed=12),
    # kernel table modes: dense objects + hashed page cells (large objects) ...
    SynthConfig(nb_samples=150_000, nb_intervals=1_500, size_min=64 * 1024, size_max=1024 * 1024, seed=13),
    # ... hashed objects + dense u16 page cells (many small objects) ...
    SynthConfig(nb_samples=100_000, nb_intervals=5_000, size_max=4096, seed=14),
    # ... and 4 MiB buffers: > 62 windows per workgroup, so the dense page
    # counts are flushed on their cadence, not only at stream ends
    SynthConfig(nb_samples=3_000_000, nb_intervals=800, buffer_records=100_000, seed=15),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=[f"cfg{i}" for i in range(len(CONFIGS))])
def test_engine_bit_exact_vs_oracle(tmp_path, cfg):
    d = str(tmp_path)
    path, odir = _oracle(generate(cfg), d)
    edir = _engine_replay(path, d)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    assert open(os.path.join(d, "oracle_stdout.txt"), "rb").read() == open(os.path.join(d, "engine_stdout.txt"), "rb").read()
    _same_dirs(odir, edir)


def test_readme_block_on_gpu(tmp_path):
    d = str(tmp_path)
    path, odir = _oracle(readme_fixture.build(), d)
    _engine_replay(path, d)
    got = readme_fixture.normalize(open(os.path.join(d, "engine_stdout.txt"), newline="").read())
    assert got == readme_fixture.expected_lines()
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))


def test_full_config2_bit_exact(tmp_path):
    """BASELINE configs[1] at full size: 10M records, 1k intervals."""
    d = str(tmp_path)
    path, odir = _oracle(generate(SynthConfig(nb_samples=10_000_000, nb_intervals=1_000, seed=42)), d)
    edir = _engine_replay(path, d)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    _same_dirs(odir, edir)


@pytest.mark.parametrize("nb_intervals", [300, 6_000])
def test_large_weights_bit_exact(tmp_path, nb_intervals):
    """Weights at and above the kernel's packing limits (2^23 per lane, 2^26
    per wave sum, the packed long-tail limit 2^28, 2^32, up to 2^63): the unpacked LDS / global paths of the
    dense (<= 2048 entries) and hashed table modes must agree with the oracle,
    including u64 wrap-around of the weight sums (mem_sampling.c:531)."""
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=200_000, nb_intervals=nb_intervals, seed=16))
    rng = np.random.default_rng(16)
    # (2^28: the hashed mode's packed long-tail limit at 200k records, 2^(64 - 2 * 18))
    big = np.array([(1 << 23) - 1, 1 << 23, (1 << 26) + 5, (1 << 28) - 1, 1 << 28, (1 << 32) - 1, 1 << 32,
                    (1 << 40) + 7, (1 << 63) + 3, (1 << 64) - 1], dtype=np.uint64)
    for b in rp.buffers:
        rec = b.ring.view(RECORD_DTYPE)  # pure 40 B SAMPLE streams (lost_frac = 0, no wrap)
        pick = rng.random(rec.shape[0]) < 0.05
        rec["weight"][pick] = big[rng.integers(0, big.shape[0], int(pick.sum()))]
    path, odir = _oracle(rp, d)
    edir = _engine_replay(path, d)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    assert open(os.path.join(d, "oracle_stdout.txt"), "rb").read() == open(os.path.join(d, "engine_stdout.txt"), "rb").read()
    _same_dirs(odir, edir)


@pytest.mark.parametrize("dbg", [0, 0x2000, 0x2000 | 0x4000])
def test_long_tail_paths_bit_exact(tmp_path, dbg):
    """Hashed object mode's three long-tail paths: the per-range log summed by
    tlog_reduce_kernel, its overflow through packed atomics (internal switch
    0x2000: sub-logs of 2 records) and through plain atomics (0x4000: no
    packing); weights on both sides of the packing limit (2^(64 - 2 * 18) =
    2^28 at 200k records) and past 2^32."""
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=200_000, nb_intervals=20_000, seed=17))
    rng = np.random.default_rng(17)
    big = np.array([(1 << 28) - 1, 1 << 28, (1 << 32) + 3, (1 << 63) + 1], dtype=np.uint64)
    for b in rp.buffers:
        rec = b.ring.view(RECORD_DTYPE)
        pick = rng.random(rec.shape[0]) < 0.02
        rec["weight"][pick] = big[rng.integers(0, big.shape[0], int(pick.sum()))]
    path, odir = _oracle(rp, d)
    edir = _engine_replay(path, d, flags=_lib.NMG_F_DEFAULT | dbg)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    assert open(os.path.join(d, "oracle_stdout.txt"), "rb").read() == open(os.path.join(d, "engine_stdout.txt"), "rb").read()
    _same_dirs(odir, edir)


def test_no_match_mode(tmp_path):
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=40_000, nb_intervals=100, seed=8))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "oracle"), os.path.join(d, "o.txt"), os.path.join(d, "oracle_raw.bin"),
                 match_samples=False)
    _engine_replay(path, d, flags=_lib.NMG_F_PAGE_HIST)
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "engine_stdout.txt"), "rb").read()


def test_sparse_histogram_path(tmp_path):
    """Every object's page histogram forced sparse (hashed cells)."""
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=100_000, nb_intervals=400, seed=9))
    path, odir = _oracle(rp, d)
    eng = Engine(flags=_lib.NMG_F_DEFAULT, nb_threads=rp.nb_threads, hist_budget_bytes=4, sparse_capacity=1 << 16)
    eng.set_objects(rp.table)
    eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    edir = os.path.join(d, "engine")
    eng.report(edir, os.path.join(d, "e.txt"))
    assert open(os.path.join(d, "oracle_stdout.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)
    raw = RawResults.read(os.path.join(d, "oracle_raw.bin"))
    assert np.array_equal(eng.page_cells(), raw.cells)


def test_device_resident_buffers(tmp_path):
    """nmg_set_device_buffers on a torch-allocated HBM arena == staged path."""
    import torch
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=150_000, nb_intervals=2_000, lost_frac=1e-3, seed=10))
    path, odir = _oracle(rp, d)
    arena, offs, lens, ranks, acc = rp.packed()
    dev = torch.from_numpy(arena).cuda()
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.set_device_buffers(dev.data_ptr(), offs, lens, ranks, acc)
    for _ in range(3):  # reset + analyse repeatedly: no state leaks between steps
        eng.reset()
        eng.analyze()
    eng.synchronize()
    edir = os.path.join(d, "engine")
    eng.report(edir, os.path.join(d, "e.txt"))
    assert open(os.path.join(d, "oracle_stdout.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)
    raw = RawResults.read(os.path.join(d, "oracle_raw.bin"))
    first, cw = eng.object_counters()
    assert np.array_equal(first, raw.first_ordinal)
    assert np.array_equal(cw, raw.count_weight)
    g, ns, nf = eng.global_counters()
    assert np.array_equal(g, raw.global_counters) and (ns, nf) == (raw.nb_samples, raw.nb_found)


def test_two_shard_merge_matches_single(tmp_path):
    """The multi-GPU scheme on one device: two engines, contiguous shards with
    seq_base, merged (sum / min / max / gathers) -> identical report."""
    import torch
    from numamma_amd.distributed import merge_sparse, shard_ranges
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=200_000, nb_intervals=3_000, seed=11))
    path, odir = _oracle(rp, d)
    arena, offs, lens, ranks, acc = rp.packed()
    dev = torch.from_numpy(arena).cuda()
    engines = []
    for lo, hi in shard_ranges(lens, 2):
        e = Engine(nb_threads=rp.nb_threads, hist_budget_bytes=4, sparse_capacity=1 << 18)
        e.set_objects(rp.table)
        e.set_device_buffers(dev.data_ptr(), offs[lo:hi], lens[lo:hi], ranks[lo:hi], acc[lo:hi], seq_base=lo)
        e.analyze()
        e.synchronize()
        engines.append(e)
    # merge into engine 0 exactly as merge_engine does over RCCL
    for which, op in ((_lib.NMG_ARR_SUM64, "sum"), (_lib.NMG_ARR_MIN64, "min"), (_lib.NMG_ARR_MAX64, "max")):
        n = engines[0].array_size(which)
        ts = []
        for e in engines:
            t = torch.empty(n, dtype=torch.int64, device="cuda")
            e.export_array(which, t.data_ptr())
            ts.append(t)
        if op == "sum":
            m = ts[0] + ts[1]
        else:
            f = [t ^ torch.tensor(-(1 << 63), dtype=torch.int64, device="cuda") for t in ts]
            m = (torch.minimum(*f) if op == "min" else torch.maximum(*f)) ^ torch.tensor(-(1 << 63), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        engines[0].import_array(which, m.data_ptr())
    parts = [e.sparse_export() for e in engines]
    for k, _ in parts:  # (export order: ascending keys, reproducible)
        assert np.all(k[1:] > k[:-1])
    assert all(np.array_equal(a[0], b[0]) for a, b in zip(parts, [e.sparse_export() for e in engines]))
    engines[0].sparse_import(*merge_sparse(parts))
    cs = [e.buffer_counts() for e in engines]
    engines[0].set_buffer_counts(np.concatenate([c[0] for c in cs]), np.concatenate([c[1] for c in cs]),
                                 np.concatenate([np.array(e.buffer_bytes, dtype=np.uint64) for e in engines]))
    edir = os.path.join(d, "engine")
    engines[0].report(edir, os.path.join(d, "e.txt"))
    assert open(os.path.join(d, "oracle_stdout.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)


def _one_buffer_replay(raw_bytes):
    from numamma_amd.replay import Buffer, Replay

    rp = generate(SynthConfig(nb_samples=100, nb_intervals=10, seed=1))
    rp.buffers = [Buffer(0, 0, np.frombuffer(raw_bytes, dtype=np.uint8).copy(), 0, len(raw_bytes))]
    return rp


@pytest.mark.parametrize("case,code", [("zero_size", -4), ("truncated", -5), ("odd_size", -9)])
def test_error_codes(tmp_path, case, code):
    """Malformed records: the reference abort()s (size 0, mem_sampling.c:857)
    or reads out of bounds (truncated SAMPLE, :865-879); the engine returns
    the matching NMG_ERR_* code instead."""
    from numamma_amd.engine import Engine

    rec = np.zeros(20, dtype=RECORD_DTYPE)
    rec["type"] = 9
    rec["size"] = 40
    raw = bytearray(rec.tobytes())
    if case == "zero_size":
        raw[40 * 7 + 6:40 * 7 + 8] = b"\0\0"
    elif case == "truncated":
        raw = raw[:-16]
    else:
        raw[40 * 3 + 6:40 * 3 + 8] = (44).to_bytes(2, "little")
    rp = _one_buffer_replay(bytes(raw))
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.submit_replay(rp)
    eng.analyze()
    with pytest.raises(_lib.NmgError) as ei:
        eng.synchronize()
    assert ei.value.code == code


def test_empty_inputs(tmp_path):
    """No buffers at all, and an empty object table."""
    from numamma_amd.engine import Engine
    from numamma_amd.replay import ObjectTable

    rp = generate(SynthConfig(nb_samples=1000, nb_intervals=10, seed=1))
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.analyze()
    eng.synchronize()
    g, ns, nf = eng.global_counters()
    assert ns == 0 and nf == 0
    empty = ObjectTable(np.zeros(0, np.uint64), np.zeros(1, np.uint32), rp.table.entries[:0],
                        np.zeros(0, np.uint64), b"")
    eng2 = Engine(nb_threads=rp.nb_threads)
    eng2.set_objects(empty)
    eng2.submit_replay(rp)
    eng2.analyze()
    eng2.synchronize()
    g, ns, nf = eng2.global_counters()
    assert ns == rp.nb_records() and nf == 0


def _edge_replay(nkeys, seed, cluster=0):
    """A table of exactly `nkeys` keys (a generated table cut down) and samples
    at every lookup boundary: each key, key - 1, end - 1, end, the
    alloc / free dates themselves and one tick outside, address 0 and the
    top of the address space.  `cluster` > 0 moves every run of `cluster`
    consecutive keys (with their objects) 2^40 bytes further up than the
    previous run: buckets spanning a huge gap, many keys per directory slot."""
    from numamma_amd.replay import Buffer, ObjectTable, Replay

    rp = generate(SynthConfig(nb_samples=1000, nb_intervals=nkeys + 50, reuse_frac=0.2, seed=seed))
    t = rp.table
    assert t.nb_keys >= nkeys
    ne = int(t.entry_off[nkeys])
    tab = ObjectTable(t.keys[:nkeys].copy(), t.entry_off[:nkeys + 1].copy(), t.entries[:ne].copy(),
                      t.callstack_pool, t.string_pool)
    if cluster:
        shift = (np.arange(nkeys, dtype=np.uint64) // np.uint64(cluster)) << np.uint64(40)
        tab.keys += shift
        per_entry = np.repeat(shift, np.diff(tab.entry_off).astype(np.int64))
        tab.entries["buffer_addr"] += per_entry
    rng = np.random.default_rng(seed)
    e = tab.entries
    first = tab.entry_off[:-1]
    addrs, tss = [], []
    for k in range(nkeys):
        x = e[first[k]]
        a, end = int(x["buffer_addr"]), int(x["buffer_addr"]) + int(x["buffer_size"])
        al, fr = int(x["alloc_date"]), int(x["free_date"])
        for ad in (int(tab.keys[k]), int(tab.keys[k]) - 1, a, end - 1, end):
            for ts in (al, fr, max(al - 1, 0), min(fr + 1, 2**64 - 1), (al + fr) // 2):
                addrs.append(ad % 2**64)
                tss.append(ts)
    for ad in (0, 1, 2**64 - 1, 2**64 - 2, 2**63):
        for ts in (0, 2**64 - 1, int(e["alloc_date"][0])):
            addrs.append(ad)
            tss.append(ts)
    n = len(addrs)
    rec = np.zeros(n, dtype=RECORD_DTYPE)
    rec["type"] = 9
    rec["size"] = 40
    rec["timestamp"] = np.array(tss, dtype=np.uint64)
    rec["addr"] = np.array(addrs, dtype=np.uint64)
    rec["weight"] = rng.integers(0, 2000, n)
    rec["data_src"] = (np.uint64(0x42) << np.uint64(5))  # L1 hit
    perm = rng.permutation(n)
    rec = rec[perm]
    bufs = []
    for s in range(0, n, 1500):
        raw = np.frombuffer(rec[s:s + 1500].tobytes(), dtype=np.uint8).copy()
        bufs.append(Buffer(int(rng.integers(0, rp.nb_threads)), int(rng.integers(0, 2)), raw, 0, raw.shape[0]))
    return Replay(rp.nb_threads, tab, bufs)


@pytest.mark.parametrize("nkeys,cluster", [(1, 0), (2, 0), (1022, 0), (1023, 0), (1024, 0), (1025, 0),
                                          (4095, 0), (4096, 0), (8191, 0), (40_000, 0),
                                          (20_000, 300), (20_000, 7)])
def test_lookup_boundaries_bit_exact(tmp_path, nkeys, cluster):
    """Every lookup layout: <= 1023 keys use the LDS Eytzinger tree with node
    records; up to 4095 keys are all fences; larger tables add the per-bucket
    directory (1 to 2^16 keys per bucket), whose slots can hold many keys or
    be skipped for a binary search when a bucket spans a huge gap (`cluster`).
    Each crossover is covered on both sides."""
    d = str(tmp_path)
    path, odir = _oracle(_edge_replay(nkeys, 100 + nkeys, cluster), d)
    edir = _engine_replay(path, d)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    _same_dirs(odir, edir)


@pytest.mark.parametrize("nkeys,cluster", [(40_000, 0), (20_000, 7)])
def test_lookup_without_directory_bit_exact(tmp_path, nkeys, cluster):
    """Large-table buckets with no directory (internal switch 0x8000, the
    layout of tables beyond 4095 << 16 keys): fence search, then a binary
    search of the bucket's keys."""
    d = str(tmp_path)
    path, odir = _oracle(_edge_replay(nkeys, 200 + nkeys, cluster), d)
    edir = _engine_replay(path, d, flags=_lib.NMG_F_DEFAULT | 0x8000)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    _same_dirs(odir, edir)


def _short_sample_replay(n=200_000, seed=61):
    """One buffer of n PERF_RECORD_SAMPLE records whose header size is 16 B
    (the reference's byte cursor accepts them, mem_sampling.c:862-918: the
    32 B of struct mem_sample are read after the header whatever the size),
    then two 40 B records.  Record i reads ts = its own second word, addr =
    the next header (0x0010000000000009), weight = the next record's second
    word: every sample hits one object, and a launch holds 2.5x more samples
    than nbytes / 40."""
    from numamma_amd.replay import Buffer, ObjectTable, Replay

    rp = generate(SynthConfig(nb_samples=1000, nb_intervals=3000, seed=seed))
    t = rp.table
    special = np.zeros(1, dtype=t.entries.dtype)
    special[0] = t.entries[t.entry_off[-2]]  # a heap entry as the template
    special["buffer_addr"] = 0x0010000000000000
    special["buffer_size"] = special["initial_buffer_size"] = 4096
    special["alloc_date"] = 0
    special["free_date"] = 1 << 62
    special["id"] = t.nb_entries + 1
    # (2^52 + 9: above every heap, global and [stack] key)
    tab = ObjectTable(np.concatenate([t.keys, np.array([0x0010000000000000], np.uint64)]),
                      np.concatenate([t.entry_off, [t.entry_off[-1] + 1]]).astype(np.uint32),
                      np.concatenate([t.entries, special]), t.callstack_pool, t.string_pool)
    rng = np.random.default_rng(seed)
    words = np.zeros(2 * n, dtype=np.uint64)
    words[0::2] = np.uint64(9) | (np.uint64(16) << np.uint64(48))
    words[1::2] = rng.integers(1, 2000, n).astype(np.uint64)
    tail = np.zeros(2, dtype=RECORD_DTYPE)
    tail["type"], tail["size"], tail["timestamp"], tail["addr"], tail["weight"] = 9, 40, 5, 1, 7
    raw = np.concatenate([np.frombuffer(words.tobytes(), np.uint8), np.frombuffer(tail.tobytes(), np.uint8)])
    return Replay(rp.nb_threads, tab, [Buffer(0, 0, raw.copy(), 0, raw.shape[0])])


@pytest.mark.parametrize("dbg", [0, 0x2000])
def test_short_sample_records_bit_exact(tmp_path, dbg):
    """SAMPLE records shorter than 40 B in the hashed object mode: they stay
    out of the packed long-tail counters (whose bound counts 40 B records);
    0x2000 (sub-logs of 2 records) drives every contribution to the overflow
    paths."""
    d = str(tmp_path)
    path, odir = _oracle(_short_sample_replay(), d)
    edir = _engine_replay(path, d, flags=_lib.NMG_F_DEFAULT | dbg)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    _same_dirs(odir, edir)


# ---- batch submit and streaming (configs[4]): same results as one nmg_analyze
STREAM_CASES = [
    # (replay config, NMG_REPLAY_STREAM = chunk_bytes:copy_threads:batch)
    (SynthConfig(nb_samples=120_000, nb_intervals=2_000, lost_frac=1e-3, wrap_one=True, seed=31), "0:4:16"),
    (SynthConfig(nb_samples=120_000, nb_intervals=2_000, lost_frac=1e-3, wrap_one=True, seed=32), "262144:1:7"),
    (SynthConfig(nb_samples=400_000, nb_intervals=5_000, seed=33), "1048576:4:64"),
    (SynthConfig(nb_samples=50_000, nb_intervals=300, seed=34), "65536:2:1"),  # ~one buffer per chunk
    # buffers larger than a chunk, > 62 windows per workgroup in a chunk
    (SynthConfig(nb_samples=2_000_000, nb_intervals=900, buffer_records=100_000, seed=35), "1048576:3:4"),
    # large table in a stream
    (SynthConfig(nb_samples=200_000, nb_intervals=60_000, seed=36), "2097152:8:32"),
]


@pytest.mark.parametrize("cfg,mode", STREAM_CASES, ids=[f"stream{i}" for i in range(len(STREAM_CASES))])
def test_streaming_bit_exact_vs_oracle(tmp_path, monkeypatch, cfg, mode):
    """nmg_submit_buffers (copy threads) and nmg_stream_begin chunks (uploaded
    and analysed while submission continues) give byte-identical reports and raw
    results: analysis order, per-buffer counts and first-match ordinals span
    the chunks (mem_sampling.c:953-957 online branch fed per alarm)."""
    d = str(tmp_path)
    path, odir = _oracle(generate(cfg), d)
    monkeypatch.setenv("NMG_REPLAY_STREAM", mode)
    edir = _engine_replay(path, d)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    assert open(os.path.join(d, "oracle_stdout.txt"), "rb").read() == open(os.path.join(d, "engine_stdout.txt"), "rb").read()
    _same_dirs(odir, edir)


ZERO_COPY_CASES = [
    # (replay config, NMG_REPLAY_STREAM: "" = nmg_submit_ring per buffer, "0:4:16" = nmg_submit_buffers batches)
    (SynthConfig(nb_samples=150_000, nb_intervals=2_000, lost_frac=1e-3, wrap_one=True, seed=41), ""),
    (SynthConfig(nb_samples=150_000, nb_intervals=2_000, lost_frac=1e-3, wrap_one=True, seed=42), "0:4:16"),
    (SynthConfig(nb_samples=300_000, nb_intervals=60_000, lost_frac=1e-3, seed=43), "0:4:64"),  # partition-first
    (SynthConfig(nb_samples=100_000, nb_intervals=3_000, buffer_records=97, seed=44), ""),  # odd buffer sizes
]


@pytest.mark.parametrize("cfg,mode", ZERO_COPY_CASES, ids=[f"zc{i}" for i in range(len(ZERO_COPY_CASES))])
def test_zero_copy_bit_exact_vs_oracle(tmp_path, monkeypatch, cfg, mode):
    """nmg_register_host over the loaded replay: unwrapped buffers that start
    16-byte aligned are read in place by the kernels over PCIe, the rest
    (wrapped rings, unaligned starts) are staged; byte-identical to the
    oracle either way."""
    d = str(tmp_path)
    path, odir = _oracle(generate(cfg), d)
    monkeypatch.setenv("NMG_REPLAY_REGISTER", "1")
    if mode:
        monkeypatch.setenv("NMG_REPLAY_STREAM", mode)
    edir = _engine_replay(path, d)
    _assert_raw_equal(os.path.join(d, "oracle_raw.bin"), os.path.join(d, "engine_raw.bin"))
    assert open(os.path.join(d, "oracle_stdout.txt"), "rb").read() == open(os.path.join(d, "engine_stdout.txt"), "rb").read()
    _same_dirs(odir, edir)


def test_register_host_api(tmp_path):
    """Registration rules: overlapping ranges are refused, a range holding
    submitted buffers cannot be unregistered before nmg_clear_buffers, and
    a registered engine gives the same counters as a copying one, its buffers
    given as views or as (arena, offsets, lengths) arrays (Engine.submit_arena)."""
    from numamma_amd.engine import Engine
    from numamma_amd.replay import RECORD_DTYPE

    rp = generate(SynthConfig(nb_samples=100_000, nb_intervals=1_500, seed=45))
    lins = rp.linear_buffers()
    # one arena, buffers at 16-byte aligned offsets (one deliberately at +8: staged)
    offs, o = [], 0
    for i, (_, _, b) in enumerate(lins):
        o = (o + 15) // 16 * 16 + (8 if i == 3 else 0)
        offs.append(o)
        o += b.shape[0]
    from numamma_amd.engine import page_aligned_empty

    arena = page_aligned_empty(o + 64)
    arena[:] = 0
    for (_, _, b), off in zip(lins, offs):
        arena[off:off + b.shape[0]] = b
    views = [(r, a, arena[off:off + b.shape[0]]) for (r, a, b), off in zip(lins, offs)]
    out = []
    for register, as_arena in ((False, False), (True, False), (True, True)):
        eng = Engine(nb_threads=rp.nb_threads)
        eng.set_objects(rp.table)
        if register:
            eng.register_host(arena)
            with pytest.raises(_lib.NmgError):
                eng.register_host(arena[4096:])  # overlap
            with pytest.raises(_lib.NmgError):
                eng.register_host(arena[100:])  # not page-aligned
        if as_arena:
            lens = np.array([b.shape[0] for _, _, b in lins], dtype=np.uint64)
            ranks = np.array([r for r, _, _ in lins], dtype=np.uint32)
            accs = np.array([a for _, a, _ in lins], dtype=np.uint32)
            with pytest.raises(ValueError):
                eng.submit_arena(arena, offs, lens, ranks[:-1], accs)
            with pytest.raises(ValueError):
                eng.submit_arena(arena[:offs[-1]], offs, lens, ranks, accs)  # past the arena
            neg = np.asarray(offs, dtype=np.int64).copy()
            neg[0] = -16  # (wraps to 2^64 - 16 unsigned: before the arena)
            with pytest.raises(ValueError):
                eng.submit_arena(arena, neg, lens, ranks, accs)
            eng.submit_arena(arena, offs, lens, ranks, accs)
        else:
            eng.submit_buffers(views)
        eng.analyze()
        eng.synchronize()
        g, ns, nf = eng.global_counters()
        first, cw = eng.object_counters()
        bs, bf = eng.buffer_counts()
        out.append((g, ns, nf, first, cw, bs, bf, eng.page_cells()))
        if register:
            with pytest.raises(_lib.NmgError):
                eng.unregister_host(arena)  # buffers still submitted
            eng.clear_buffers()
            eng.unregister_host(arena)
        eng.close()
    for o in out[1:]:
        for x, y in zip(out[0], o):
            assert np.array_equal(np.asarray(x), np.asarray(y))
    assert out[0][1] == sum(int((b.view(RECORD_DTYPE)["type"] == 9).sum()) for _, _, b in lins)


def test_streaming_python_api_repeat(tmp_path):
    """Engine.stream_begin + submit_buffers in alarm-sized batches, analysed,
    then cleared and streamed again on the same engine (state reuse), equal to
    a single device-resident analysis of the same buffers."""
    from numamma_amd.engine import Engine

    rp = generate(SynthConfig(nb_samples=300_000, nb_intervals=1_500, seed=37))
    lins = rp.linear_buffers()
    ref = Engine(nb_threads=rp.nb_threads)
    ref.set_objects(rp.table)
    for r, a, data in lins:
        ref.submit_buffer(data, r, a)
    ref.analyze()
    ref.synchronize()
    want = (ref.global_counters(), ref.buffer_counts(), ref.object_counters(), ref.page_cells())
    ref.close()
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    for rnd in range(2):
        eng.clear_buffers()
        eng.reset()
        eng.stream_begin(chunk_bytes=512 << 10, copy_threads=3)
        for i in range(0, len(lins), 23):
            eng.submit_buffers(lins[i:i + 23])
        eng.analyze()
        eng.synchronize()
        got = (eng.global_counters(), eng.buffer_counts(), eng.object_counters(), eng.page_cells())
        for a, b in zip(want, got):
            for x, y in zip(a if isinstance(a, tuple) else (a,), b if isinstance(b, tuple) else (b,)):
                assert np.array_equal(np.asarray(x), np.asarray(y)), rnd
    eng.close()


def test_sparse_table_reset_cycles():
    """The sparse (object, thread, page) table is cleared by a reset only when
    an analysis inserted into it since the previous reset (two parity flags):
    accumulate without reset, reset, reset twice in a row, re-analyse."""
    from numamma_amd.engine import Engine

    rp = generate(SynthConfig(nb_samples=60_000, nb_intervals=300, seed=38))
    eng = Engine(flags=_lib.NMG_F_DEFAULT, nb_threads=rp.nb_threads, hist_budget_bytes=4, sparse_capacity=1 << 16)
    eng.set_objects(rp.table)
    eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    once = eng.page_cells()
    assert once.shape[0] > 0
    eng.analyze()  # counters accumulate
    eng.synchronize()
    twice = eng.page_cells()
    assert np.array_equal(twice[:, :3], once[:, :3]) and np.array_equal(twice[:, 3], 2 * once[:, 3])
    for resets in (1, 2, 1):
        for _ in range(resets):
            eng.reset()
        eng.synchronize()
        assert eng.page_cells().shape[0] == 0
        eng.analyze()
        eng.synchronize()
        assert np.array_equal(eng.page_cells(), once)
    eng.close()


# ---- dump modes: -d / -D / -u and callsite_summary_<id>.dat
MAPS = ("00400000-00452000 r-xp 00000000 08:02 173521 /usr/bin/app\n"
        "555500000000-555600000000 rw-p 00000000 00:00 0 [heap]\n"
        "7ffd0000-7ffd1000 rw-p 00000000 00:00 0 [stack]\n")
# dladdr() view for all_memory_objects.dat (frames past 0x4f0000: no module)
DUMP_MODULES = [(0x400000, 0x480000, 0x400000, "/usr/bin/app"), (0x480000, 0x4F0000, 0x470000, "/usr/lib/libfoo.so.1")]


@pytest.mark.parametrize("dump,dump_all,unmatched,single,resident", [
    (1, 0, 0, 1, False), (0, 1, 0, 1, False), (1, 1, 1, 1, False), (0, 0, 1, 1, True),
    (1, 1, 1, 0, True), (1, 1, 1, 1, True)])
def test_dump_modes_bit_exact(tmp_path, dump, dump_all, unmatched, single, resident):
    """Every dump file byte-identical to the oracle's: callsite_dump_<id>.dat,
    callsite_summary_<id>.dat for the sort's predecessor sites (Q10),
    all_memory_accesses.dat, all_memory_objects.dat, unmatched_samples.log with the maps header
    (last line repeated by the reference's feof loop); staged and
    device-resident buffers."""
    import torch
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=40_000, nb_intervals=300, lost_frac=2e-3, wrap_one=True, seed=51))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), dump_single_items=bool(single), dump=bool(dump),
                 dump_all=bool(dump_all), dump_unmatched=bool(unmatched), maps_path="/proc/4242/maps", maps_text=MAPS,
                 modules=DUMP_MODULES)
    flags = _lib.NMG_F_DEFAULT | _lib.NMG_F_SAMPLE_MATCHES | _lib.NMG_F_OBJECT_LEVELS
    eng = Engine(flags=flags, nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    keep = None
    if resident:
        arena, offs, lens, ranks, acc = rp.packed()
        keep = torch.from_numpy(arena).cuda()
        eng.set_device_buffers(keep.data_ptr(), offs, lens, ranks, acc)
    else:
        eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    edir = os.path.join(d, "engine")
    dflags = ((_lib.NMG_DUMP_CALLSITES if dump else 0) | (_lib.NMG_DUMP_ALL if dump_all else 0)
              | (_lib.NMG_DUMP_UNMATCHED if unmatched else 0))
    eng.report(edir, os.path.join(d, "e.txt"), dump_single_items=single, dump_flags=dflags,
               maps_path="/proc/4242/maps", maps_text=MAPS, modules=DUMP_MODULES)
    eng.close()
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    names = sorted(os.listdir(odir))
    assert any(n.startswith("callsite_summary_") for n in names) == bool((dump or dump_all) and single)
    assert ("all_memory_objects.dat" in names) == bool(dump_all)
    _same_dirs(odir, edir)


def test_replay_helper_dump_modes(tmp_path, monkeypatch):
    """The out-of-process helper path (nmg_run_replay, NMG_REPLAY_DUMP=7) with
    the replay's context section (module table, maps file): every dump file,
    all_memory_objects.dat included, byte-identical to the oracle's."""
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=40_000, nb_intervals=300, lost_frac=2e-3, wrap_one=True, seed=52))
    rp.modules, rp.maps_path, rp.maps_text = DUMP_MODULES, "/proc/4242/maps", MAPS
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), dump=True, dump_all=True, dump_unmatched=True,
                 maps_path=rp.maps_path, maps_text=MAPS, modules=DUMP_MODULES)
    monkeypatch.setenv("NMG_REPLAY_DUMP", str(_lib.NMG_DUMP_CALLSITES | _lib.NMG_DUMP_ALL | _lib.NMG_DUMP_UNMATCHED))
    from numamma_amd.engine import run_replay

    edir = os.path.join(d, "engine")
    run_replay(path, edir, os.path.join(d, "e.txt"))
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    assert "all_memory_objects.dat" in os.listdir(edir)
    _same_dirs(odir, edir)
