"""Replays that reproduce three more output blocks of the reference README.

* readme_call_sites.log -- README.md:115-123, the `call_sites.log` of a
  mat_mul run: 7 call sites (six size-12000 malloc lines of test/mat_mul.c
  plus [stack]), their buffer counts, read counts, read weights and write
  counts;
* readme_callsite_counters_3.dat -- README.md:127-131, `callsite_counters_3.dat`
  of the same run: site 3 (mat_mul.c:74) per page (3 pages of a 12000-byte
  object) and per thread (4 threads).  Its 12 cells sum to 5539404 = the
  5498814 reads + 40590 writes of site 3 in call_sites.log, so both blocks
  come from one run and one replay reproduces both;
* readme_callsite_summary.dat -- README.md:159-175, a `callsite_summary_<id>.dat`
  of the dump mode (-d): one site's read counters per memory level (L1, L2,
  L3, LFB, local RAM hits, with their total weights) and 12040 L1 write hits;
* readme_callsite_dump.dat -- README.md:141-148, a `callsite_dump_<id>.dat` of
  the dump mode: six samples of one site, one row each (thread, timestamp,
  offset in the object, get_data_src_level string, weight).  The README
  predates the trailing access_type column that _dump_call_site prints
  (mem_sampling.c:792-804), so the first five columns and the header without
  that column are compared (dump_rows).

Everything these blocks print is a per-site aggregate, so any sample stream
with those aggregates reproduces them; the builders below choose one
deterministically (seeded): per (site, thread, access, page) sample counts,
read weights base/base+1 so each site's (or level's) total weight is exact,
first matches in the README's id order (ids are given at a site's first
match, mem_analyzer.c:1333-1378 via __match_sample, mem_sampling.c:594-673).
What they pin beyond readme_fixture.py: the `(size=%zu) - %d buffers` line
of 12000-byte sites with 1..339 objects, the %f average weight, the weight
sort of 7 sites, __plot_counters' page rows x thread columns
(mem_analyzer.c:1559-1583), and __print_counters' per-level lines with the
integer average (mem_analyzer.c:1438-1487).  The README was rendered by a
terminal (tabs expanded), so comparisons collapse whitespace
(readme_fixture.normalize).

Sizes: the call-site replay holds 58.9M records (2.35 GB of PEBS records),
the summary replay 6.28M."""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from numamma_amd.replay import (  # noqa: E402
    ENTRY_DTYPE, LVL_HIT, LVL_L1, LVL_L2, LVL_L3, LVL_LFB, LVL_LOC_RAM, MEM_DYNAMIC, MEM_STACK, MEM_OP_LOAD,
    MEM_OP_STORE, RECORD_DTYPE, STACK_BASE, STACK_END, Buffer, ObjectTable, Replay)

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/home/trahay/Soft/opt/numamma/test/mat_mul.c"
CALL_SITES = os.path.join(HERE, "readme_call_sites.log")
COUNTERS_3 = os.path.join(HERE, "readme_callsite_counters_3.dat")
SUMMARY = os.path.join(HERE, "readme_callsite_summary.dat")
DUMP = os.path.join(HERE, "readme_callsite_dump.dat")

READ, WRITE = 0, 1
PAGE = 4096
OBJ_SIZE = 12000
REC_PER_BUF = 3276  # 128 KiB sample buffers
ALLOC, FREE = 1_000_000_000, 3_000_000_000

# heap sites in README id order (id 1 is [stack]): line, objects, reads, read weight, writes
HEAP_SITES = [
    ("70", 38, 6_873_841, 58_451_985, 40_590),
    ("74", 160, 5_498_814, 1_305_315_950, 40_590),
    ("78", 339, 5_818_196, 1_088_387_205, 14_656_019),
    ("76", 1, 10_830_555, 80_991_250, 0),
    ("72", 1, 6_453_238, 52_071_167, 0),
    ("68", 1, 6_836_348, 48_885_993, 0),
]
STACK_SITE = (1_819_616, 14_471_352, 4_946)
# callsite_counters_3.dat: [page][thread] reads + writes of site 3 (mat_mul.c:74)
SITE3_CELLS = np.array([[58570, 0, 5352336, 58], [58570, 0, 0, 0], [27042, 0, 42828, 0]], dtype=np.int64)
SITE3_WRITES = {(0, 0): 20_000, (1, 0): 20_590}  # the 40590 writes: (page, thread) -> count
NB_THREADS = 4


def _table(sites, obj_size):
    """Object table: the objects of each heap site at 16 KiB strides (one
    call stack per site, frames 3.. distinct), then [stack]."""
    strings = bytearray()
    caller_off = []
    for line, *_ in sites:
        caller_off.append(len(strings))
        strings += f"{SRC}:{line}(main)".encode() + b"\0"
    heap = [(si, j) for si, s in enumerate(sites) for j in range(s[1])]
    K = len(heap) + 1
    ent = np.zeros(K, dtype=ENTRY_DTYPE)
    keys = np.zeros(K, dtype=np.uint64)
    pool = []
    first = []
    addr = 0x555555560000
    for e, (si, j) in enumerate(heap):
        if j == 0:
            first.append(e)
        r = ent[e]
        keys[e] = addr
        r["buffer_addr"] = addr
        r["buffer_size"] = obj_size
        r["initial_buffer_size"] = obj_size
        r["alloc_date"] = ALLOC
        r["free_date"] = FREE
        r["caller_rip"] = 0x555555555000 + 0x10 * si
        r["mem_type"] = MEM_DYNAMIC
        r["caller_off"] = caller_off[si]
        cs = [0x7F0000001000 + e, 0x7F0000002000 + e, 0x7F0000003000 + e,  # interposer frames
              0x555555555000 + 0x10 * si, 0x555555556000, 0x7F0000004000]
        r["has_callstack"] = 1
        r["callstack_size"] = len(cs)
        r["callstack_off"] = 6 * e
        pool.append(np.array(cs, dtype=np.uint64))
        addr += 0x4000
    s = ent[K - 1]
    keys[K - 1] = STACK_BASE
    s["buffer_addr"] = STACK_BASE
    s["buffer_size"] = STACK_END - STACK_BASE
    s["initial_buffer_size"] = STACK_END - STACK_BASE
    s["mem_type"] = MEM_STACK
    s["caller_off"] = len(strings)
    strings += b"[stack]\0"
    ent["id"] = np.arange(1, K + 1)
    table = ObjectTable(keys, np.arange(K + 1, dtype=np.uint32), ent, np.concatenate(pool), bytes(strings))
    return table, first


def _weights(rng, n, total):
    """n read weights summing to total: base = total // n, the remainder +1."""
    if n == 0:
        return np.zeros(0, dtype=np.uint64)
    base = total // n
    w = np.full(n, base, dtype=np.uint64)
    w[rng.choice(n, total - base * n, replace=False)] += 1
    return w


class _Lists:
    """Per (thread, access) sample columns."""

    def __init__(self):
        self.cols = {}

    def add(self, th, acc, addr, ts, w, lvl):
        self.cols.setdefault((th, acc), []).append((addr, ts, w, lvl))

    def records(self, th, acc, rng, front=None):
        parts = self.cols.get((th, acc), [])
        if not parts:
            return np.zeros(0, dtype=RECORD_DTYPE)
        cols = [np.concatenate([p[k] for p in parts]) for k in range(4)]
        n = cols[0].shape[0]
        perm = rng.permutation(n)
        if front is not None:  # these rows first, in this order (first matches)
            perm = np.concatenate([front, perm[~np.isin(perm, front)]])
        rec = np.zeros(n, dtype=RECORD_DTYPE)
        rec["type"] = 9  # PERF_RECORD_SAMPLE
        rec["misc"] = 2
        rec["size"] = 40
        rec["addr"] = cols[0][perm]
        rec["timestamp"] = cols[1][perm]
        rec["weight"] = cols[2][perm]
        rec["data_src"] = (cols[3][perm] << np.uint64(5)) | np.uint64(MEM_OP_LOAD if acc == READ else MEM_OP_STORE)
        return rec


def _buffers(rec, th, acc):
    raw = rec.view(np.uint8).reshape(-1)
    step = REC_PER_BUF * 40
    return [Buffer(th, acc, raw[o:o + step], 0, min(step, raw.shape[0] - o)) for o in range(0, raw.shape[0], step)]


def _heap_cell(rng, keys, objs, page, n, cover):
    """n samples on `page` of objects drawn from `objs` (every one of them
    when cover)."""
    o = rng.integers(0, len(objs), n)
    if cover:
        o[:len(objs)] = np.arange(len(objs))
    lo = page * PAGE
    hi = min(OBJ_SIZE, lo + PAGE)
    addr = keys[np.asarray(objs)[o]] + rng.integers(lo, hi, n).astype(np.uint64)
    ts = rng.integers(ALLOC + 100_000_000, FREE - 100_000_000, n).astype(np.uint64)
    return addr, ts


def build_call_sites() -> Replay:
    """README.md:115-131: call_sites.log + callsite_counters_3.dat."""
    rng = np.random.default_rng(115)
    table, first = _table(HEAP_SITES, OBJ_SIZE)
    keys = table.keys
    L = _Lists()
    hit = np.uint64(LVL_HIT)
    read_lvls = np.array([LVL_L1, LVL_L2, LVL_L3, LVL_LFB], dtype=np.uint64) | hit
    pages = (OBJ_SIZE + PAGE - 1) // PAGE
    for si, (line, nobj, nr, wr_total, nw) in enumerate(HEAP_SITES):
        objs = list(range(first[si], first[si] + nobj))
        # (page, thread) cells: site 3 as README.md:127-131, the others multinomial
        if line == "74":
            tot = SITE3_CELLS
        else:
            tot = rng.multinomial(nr + nw, np.full(pages * NB_THREADS, 1.0 / (pages * NB_THREADS))).reshape(
                pages, NB_THREADS)
        wcell = np.zeros_like(tot)
        if line == "74":
            for (p, t), c in SITE3_WRITES.items():
                wcell[p, t] = c
        elif nw:
            wcell = rng.multinomial(nw, tot.reshape(-1) / tot.sum()).reshape(tot.shape)
            wcell = np.minimum(wcell, tot)
            wcell[0, 0] += nw - wcell.sum()  # (cells are millions: stays <= tot)
        rcell = tot - wcell
        assert rcell.sum() == nr and wcell.sum() == nw and (rcell >= 0).all()
        wts = _weights(rng, nr, wr_total)
        big = np.unravel_index(np.argmax(tot), tot.shape)
        k = 0
        for p in range(pages):
            for t in range(NB_THREADS):
                for acc, cnt in ((READ, int(rcell[p, t])), (WRITE, int(wcell[p, t]))):
                    if not cnt:
                        continue
                    addr, ts = _heap_cell(rng, keys, objs, p, cnt, cover=(acc == READ and (p, t) == big))
                    if acc == READ:
                        w, k = wts[k:k + cnt], k + cnt
                        lvl = read_lvls[rng.integers(0, len(read_lvls), cnt)]
                    else:
                        w = np.zeros(cnt, dtype=np.uint64)
                        lvl = np.full(cnt, LVL_L1 | LVL_HIT, dtype=np.uint64)
                    L.add(t, acc, addr, ts, w, lvl)
    nr, wr_total, nw = STACK_SITE
    wts = _weights(rng, nr, wr_total)
    for acc, n, w in ((READ, nr, wts), (WRITE, nw, np.zeros(nw, dtype=np.uint64))):
        th = rng.integers(0, NB_THREADS, n)
        # a 192 KiB stack window: the [stack] object's page blocks are a sorted
        # list per thread (ma_get_block, mem_analyzer.c:494-534), so the pages
        # a real stack touches stay few
        addr = (0x7FFFFFFD0000 + 8 * rng.integers(0, 24576, n)).astype(np.uint64)
        for t in range(NB_THREADS):
            m = th == t
            c = int(m.sum())
            # [stack]: alloc = free = 0, so only timestamp-0 samples match (quirk Q4)
            L.add(t, acc, addr[m], np.zeros(c, dtype=np.uint64), w[m],
                  np.full(c, LVL_L1 | LVL_HIT, dtype=np.uint64))
    # first matches in id order, all in the first buffer (thread 0, reads):
    # [stack], then the heap sites as listed
    cols = L.cols[(0, READ)]
    offs = np.cumsum([0] + [p[0].shape[0] for p in cols])
    front = []
    st = table.keys[-1]
    allad = np.concatenate([p[0] for p in cols])
    allts = np.concatenate([p[1] for p in cols])
    front.append(int(np.flatnonzero((allad >= st) & (allts == 0))[0]))
    for si in range(len(HEAP_SITES)):
        lo = keys[first[si]]
        hi = keys[first[si] + HEAP_SITES[si][1] - 1] + np.uint64(OBJ_SIZE)
        front.append(int(np.flatnonzero((allad >= lo) & (allad < hi))[0]))
    del allad, allts, offs
    buffers = _buffers(L.records(0, READ, rng, np.array(front)), 0, READ)
    for t in range(NB_THREADS):
        for acc in (READ, WRITE):
            if (t, acc) != (0, READ):
                buffers += _buffers(L.records(t, acc, rng), t, acc)
    return Replay(NB_THREADS, table, buffers, {"fixture": "README.md:115-131"})


# callsite_summary (README.md:159-175): level -> (count, total weight) of the reads
SUMMARY_READS = [(LVL_L1, 44_461, 533_532), (LVL_L2, 336_434, 12_716_280), (LVL_L3, 5_094_515, 311_692_351),
                 (LVL_LFB, 43_375, 6_593_000), (LVL_LOC_RAM, 746_880, 167_736_693)]
SUMMARY_WRITES = 12_040


def build_summary() -> Replay:
    """README.md:159-175: one heap site (id 1) of 4 objects on one thread;
    analysed in dump mode (-d) it gets callsite_summary_1.dat."""
    rng = np.random.default_rng(159)
    table, first = _table([("74", 4, 0, 0, 0)], OBJ_SIZE)
    objs = list(range(4))
    L = _Lists()
    for lvl, n, wt in SUMMARY_READS:
        addr, ts = _heap_cell(rng, table.keys, objs, int(rng.integers(0, 3)), n, cover=True)
        L.add(0, READ, addr, ts, _weights(rng, n, wt), np.full(n, lvl | LVL_HIT, dtype=np.uint64))
    addr, ts = _heap_cell(rng, table.keys, objs, 0, SUMMARY_WRITES, cover=False)
    L.add(0, WRITE, addr, ts, np.zeros(SUMMARY_WRITES, dtype=np.uint64),
          np.full(SUMMARY_WRITES, LVL_L1 | LVL_HIT, dtype=np.uint64))
    buffers = _buffers(L.records(0, READ, rng), 0, READ) + _buffers(L.records(0, WRITE, rng), 0, WRITE)
    return Replay(1, table, buffers, {"fixture": "README.md:159-175"})


# callsite_dump (README.md:141-148): thread 0, (timestamp, offset, level, weight) in analysis order
DUMP_ROWS = [(14087247746057, 5864, LVL_L1, 0), (14087248615826, 3872, LVL_L1, 0), (14087249526638, 1888, LVL_L1, 0),
             (14087250387561, 7912, LVL_L1, 0), (14088660667040, 5776, LVL_L3, 50), (14088923322555, 6376, LVL_L2, 46)]


def build_dump() -> Replay:
    """README.md:141-148: one 12000-byte object of one heap site, six read
    samples of thread 0 in one buffer; analysed in dump mode (-d) the site
    (id 1: the first and only one matched) gets callsite_dump_1.dat."""
    table, _ = _table([("74", 1, 0, 0, 0)], OBJ_SIZE)
    table.entries["alloc_date"][0] = 14_000_000_000_000
    table.entries["free_date"][0] = 14_100_000_000_000
    base = np.uint64(table.keys[0])
    rec = np.zeros(len(DUMP_ROWS), dtype=RECORD_DTYPE)
    rec["type"] = 9  # PERF_RECORD_SAMPLE
    rec["misc"] = 2
    rec["size"] = 40
    for i, (ts, off, lvl, w) in enumerate(DUMP_ROWS):
        rec["timestamp"][i] = ts
        rec["addr"][i] = base + np.uint64(off)
        rec["weight"][i] = w
        rec["data_src"][i] = (np.uint64(lvl | LVL_HIT) << np.uint64(5)) | np.uint64(MEM_OP_LOAD)
    return Replay(1, table, _buffers(rec, 0, READ), {"fixture": "README.md:141-148"})


def dump_rows(path):
    """A callsite_dump file as the README shows it: the header without
    ' access_type', each row's first five columns."""
    lines = [x for x in open(path).read().splitlines() if x.strip()]
    head = lines[0].replace(" access_type", "")
    return [head] + [" ".join(x.split()[:5]) for x in lines[1:]]


def expected(path):
    from readme_fixture import normalize

    lines = normalize(open(path).read())
    while lines and lines[0] == "":
        lines.pop(0)
    return lines


def produced(path):
    """A produced file, normalised like the README block it is compared with
    (blank lines at either end dropped)."""
    return expected(path)
