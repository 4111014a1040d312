"""The partition-first path for large tables (nmg_route.h) against the oracle
and against the single-pass kernel: every raw counter, the reports.

Large tables (> 1023 keys) take the partition-first passes by default; these
tests pin the parts the other parity tests do not reach on purpose:

* the pool-overflow path (internal switch 0x20000: private pools of two
  chunks, so nearly every record goes through the overflow list and
  overflow_kernel's global lookups);
* analyses that accumulate without a reset (the per-buffer match counts of
  one analysis are summed before the next one reuses the chunk pool);
* the route pass's partition directory over clustered address spaces;
* partition shapes: many threads (page cells of a partition too many for
  LDS: global atomics), objects larger than a partition's LDS cells, heavily
  reused addresses (older entries), tiny buffers (more buffers than windows);
* the route pass's LDS line stage: with it, without it (every record stored
  to its slot), and with every partition's line given up at its first record
  ahead of the lap (the given-up path and the end-of-launch write-out of
  incomplete lines);
* NMG_F_SINGLE_PASS gives the same results."""
import os

import numpy as np
import pytest

import pyoracle
from numamma_amd import _lib
from numamma_amd.replay import SynthConfig, generate
from numamma_amd.results import RawResults

pytestmark = pytest.mark.gpu

NO_ROUTE = 0x10000
TINY_POOL = 0x20000
TINY_OVF = 0x80000  # (internal, with TINY_POOL) an overflow list of 64 records: the rest attributed in the route pass
NO_LINES = 0x20000000  # (internal) route pass without the LDS line stage: every record stored to its slot
LAP_NOWAIT = 0x100000  # (internal) a partition's LDS line given up at its first record ahead of the lap


def _oracle(rp, d):
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "oracle_stdout.txt"), os.path.join(d, "oracle_raw.bin"))
    return path, odir


def _engine(path, d, flags, tag):
    from numamma_amd.engine import run_replay

    edir = os.path.join(d, f"engine_{tag}")
    raw = os.path.join(d, f"engine_{tag}_raw.bin")
    run_replay(path, edir, os.path.join(d, f"engine_{tag}_stdout.txt"), raw, flags=flags)
    return edir, raw


def _same(a, b):
    assert open(a, "rb").read() == open(b, "rb").read(), (a, b)


def _same_dirs(a, b):
    fa, fb = sorted(os.listdir(a)), sorted(os.listdir(b))
    assert fa == fb
    for f in fa:
        _same(os.path.join(a, f), os.path.join(b, f))


ROUTE_CASES = [
    # LOST records, a wrapped ring, 8 threads
    SynthConfig(nb_samples=400_000, nb_intervals=50_000, lost_frac=1e-3, wrap_one=True, seed=71),
    # 64 threads: partitions' page cells exceed LDS (global cell atomics)
    SynthConfig(nb_samples=300_000, nb_intervals=20_000, nb_threads=64, seed=72),
    # objects up to 4 MiB: single keys with more cells than a partition's LDS
    SynthConfig(nb_samples=300_000, nb_intervals=3_000, size_min=1 << 20, size_max=4 << 20, seed=73),
    # heavy address reuse and reallocs: older entries of a node
    SynthConfig(nb_samples=300_000, nb_intervals=10_000, reuse_frac=0.5, realloc_frac=0.2, seed=74),
    # tiny buffers: more buffers than windows, windows across many buffers
    SynthConfig(nb_samples=200_000, nb_intervals=5_000, buffer_records=7, seed=75),
    # 10 heap arenas 1 TiB apart (+ globals, stack): more clusters than the
    # route directory's 8 segments, so some segments span a gap and their
    # slots hold many partition starts (saturated slot counts)
    SynthConfig(nb_samples=400_000, nb_intervals=400_000, size_max=4096, heap_clusters=10, seed=77),
    # 3 arenas: a segment each, dense slots
    SynthConfig(nb_samples=300_000, nb_intervals=60_000, heap_clusters=3, cluster_gap=1 << 36, seed=78),
    # chains of 4 entries on 30 % of the keys: up to ~900 older entries per
    # partition, so keys past the local pass's LDS list (kOldLds) walk the
    # chain in global memory
    SynthConfig(nb_samples=300_000, nb_intervals=20_000, reuse_frac=0.3, reuse_depth=4, seed=80),
]


@pytest.mark.parametrize("cfg", ROUTE_CASES, ids=[f"case{i}" for i in range(len(ROUTE_CASES))])
@pytest.mark.parametrize("flags", [0, TINY_POOL, TINY_POOL | TINY_OVF, _lib.NMG_F_SINGLE_PASS, NO_LINES,
                                   NO_LINES | TINY_POOL, LAP_NOWAIT, LAP_NOWAIT | TINY_POOL | TINY_OVF],
                         ids=["route", "tinypool", "tinyovf", "single", "nolines", "nolinestiny", "lapnowait",
                              "lapnowaittinyovf"])
def test_route_bit_exact(tmp_path, cfg, flags):
    d = str(tmp_path)
    path, odir = _oracle(generate(cfg), d)
    edir, raw = _engine(path, d, _lib.NMG_F_DEFAULT | flags, "e")
    _same(os.path.join(d, "oracle_raw.bin"), raw)
    _same(os.path.join(d, "oracle_stdout.txt"), os.path.join(d, "engine_e_stdout.txt"))
    _same_dirs(odir, edir)


def _results(eng):
    g, ns, nf = eng.global_counters()
    first, cw = eng.object_counters()
    bs, bf = eng.buffer_counts()
    return g, ns, nf, first, cw, bs, bf, eng.page_cells()


@pytest.mark.parametrize("extra", [0, TINY_POOL, NO_LINES, LAP_NOWAIT])
def test_route_accumulates_like_single_pass(extra):
    """analyze, analyze (no reset), synchronize, analyze: the route path and
    the single-pass kernel accumulate the same counters, per-buffer match
    counts included; then a reset and one analysis equals the oracle run."""
    import torch
    from numamma_amd.engine import Engine

    rp = generate(SynthConfig(nb_samples=500_000, nb_intervals=80_000, lost_frac=5e-4, seed=76))
    arena, offs, lens, ranks, acc = rp.packed()
    dev = torch.from_numpy(arena).cuda()
    out = []
    for flags in (_lib.NMG_F_DEFAULT | extra, _lib.NMG_F_DEFAULT | NO_ROUTE):
        eng = Engine(flags=flags, nb_threads=rp.nb_threads)
        eng.set_objects(rp.table)
        eng.set_device_buffers(dev.data_ptr(), offs, lens, ranks, acc)
        eng.analyze()
        eng.analyze()
        eng.synchronize()
        eng.analyze()
        res = _results(eng)
        eng.reset()
        eng.analyze()
        out.append((res, _results(eng)))
        eng.close()
    (a3, a1), (b3, b1) = out
    for x, y in zip(a3 + a1, b3 + b1):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    assert a3[1] == 3 * a1[1] and a3[2] == 3 * a1[2]


def test_route_escaped_records_bit_exact(tmp_path):
    """Compact records that cannot hold a sample (nmg_route.h XLayout) carry
    the escape mark and the local pass re-reads the raw record: timestamps
    before the table's first allocation (some still match the globals, alloc
    date 0) or 2^41 ns past it, addresses 2^40 bytes and more above their
    partition's first key, weights past the 14-bit field."""
    from numamma_amd.replay import RECORD_DTYPE, T0

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=300_000, nb_intervals=30_000, seed=79))
    rng = np.random.default_rng(79)
    for b in rp.buffers:
        rec = b.ring.view(RECORD_DTYPE)  # pure 40 B SAMPLE streams (lost_frac = 0, no wrap)
        u = rng.random(rec.shape[0])
        early, late = u < 0.03, (u >= 0.03) & (u < 0.05)
        far, heavy = (u >= 0.05) & (u < 0.07), (u >= 0.07) & (u < 0.08)
        rec["timestamp"][early] = rng.integers(1, T0, int(early.sum()), dtype=np.uint64)
        rec["timestamp"][late] += np.uint64(1 << 41)
        rec["addr"][far] = np.uint64(0x600000000000) + rng.integers(0, 1 << 41, int(far.sum()), dtype=np.uint64)
        rec["weight"][heavy] = rng.integers(1 << 14, 1 << 20, int(heavy.sum()), dtype=np.uint64)
    path, odir = _oracle(rp, d)
    for tag, flags in (("route", 0), ("tiny", TINY_POOL), ("nolines", NO_LINES), ("lapnowait", LAP_NOWAIT)):
        edir, raw = _engine(path, d, _lib.NMG_F_DEFAULT | flags, tag)
        _same(os.path.join(d, "oracle_raw.bin"), raw)
        _same(os.path.join(d, "oracle_stdout.txt"), os.path.join(d, f"engine_{tag}_stdout.txt"))
        _same_dirs(odir, edir)


def test_route_settled_partitions_keep_timestamp_zero(tmp_path):
    """Partitions whose entries all have free_date 0 (the [stack] range after
    warn_non_freed_buffers, quirk Q4; RouteParams::pdead) are matched only by
    timestamp-0 samples (alloc <= ts <= free, mem_analyzer.c:148-149): the route
    pass drops their other samples and keeps those.  Here 20 % of the [stack]
    samples carry timestamp 0 and must match the stack entry (a call site of
    their own, page cells in the sparse table), and a cluster of objects
    allocated at 0 and never freed (free_date 0) forms partitions of its own,
    hit by timestamp-0 samples too."""
    from numamma_amd.replay import RECORD_DTYPE, STACK_BASE

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=300_000, nb_intervals=30_000, heap_clusters=3, cluster_gap=1 << 36,
                              seed=81))
    t = rp.table
    # the highest heap cluster's objects: allocated at 0, never freed
    keys = np.asarray(t.keys, dtype=np.uint64)
    heap = keys[keys < np.uint64(STACK_BASE)]
    hi = heap[-1] - np.uint64(1 << 35)
    ent = t.entries
    live = (ent["buffer_addr"] >= hi) & (ent["buffer_addr"] < np.uint64(STACK_BASE)) & (ent["alloc_date"] > 0)
    ent["alloc_date"][live] = 0
    ent["free_date"][live] = 0
    assert live.sum() > 3000  # (several partitions of them)
    rng = np.random.default_rng(81)
    nz = 0
    for b in rp.buffers:
        rec = b.ring.view(RECORD_DTYPE)  # pure 40 B SAMPLE streams
        sel = ((rec["addr"] >= np.uint64(STACK_BASE)) | (rec["addr"] >= hi)) & (rng.random(rec.shape[0]) < 0.2)
        rec["timestamp"][sel] = 0
        nz += int(sel.sum())
    assert nz > 1000
    path, odir = _oracle(rp, d)
    raw = RawResults.read(os.path.join(d, "oracle_raw.bin"))
    assert raw.nb_found > 0
    for tag, flags in (("route", 0), ("tiny", TINY_POOL), ("single", _lib.NMG_F_SINGLE_PASS)):
        edir, eraw = _engine(path, d, _lib.NMG_F_DEFAULT | flags, tag)
        _same(os.path.join(d, "oracle_raw.bin"), eraw)
        _same(os.path.join(d, "oracle_stdout.txt"), os.path.join(d, f"engine_{tag}_stdout.txt"))
        _same_dirs(odir, edir)


def test_route_hot_page_cell_past_u16(tmp_path):
    """One cell taking most of an item's records: a Zipf(3) hot object of one
    page, one thread, so a work item of the local pass puts far more than
    2^16 samples on one u16 LDS page cell when items hold more than 2^16
    records (kPageCarry: the cell moves kCarryMove to global memory at
    kCarryAt); the counts must still equal the oracle's, and the hot cell
    must be past 2^16."""
    d = str(tmp_path)
    cfg = SynthConfig(nb_samples=600_000, nb_intervals=3_000, nb_threads=1, size_min=64, size_max=4000, zipf_s=3.0,
                      frac_gap=0.0, frac_stack=0.0, frac_global=0.0, reuse_frac=0.0, realloc_frac=0.0, seed=82)
    path, odir = _oracle(generate(cfg), d)
    raw = RawResults.read(os.path.join(d, "oracle_raw.bin"))
    assert int(raw.cells[:, 3].max()) > 3 * 65536
    for tag, flags in (("route", 0), ("nolines", NO_LINES)):
        edir, eraw = _engine(path, d, _lib.NMG_F_DEFAULT | flags, tag)
        _same(os.path.join(d, "oracle_raw.bin"), eraw)
        _same(os.path.join(d, "oracle_stdout.txt"), os.path.join(d, f"engine_{tag}_stdout.txt"))
        _same_dirs(odir, edir)
