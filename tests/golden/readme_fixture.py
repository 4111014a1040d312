"""Replay that reproduces the reference README's example report.

tests/golden/readme_report.txt holds the report block printed in the
reference README (README.md:80-107: a run of test/mat_mul.c under numamma).
Every number in it is internally consistent (74698 samples = 7293 reads +
67405 writes, 72793 matched = the call sites' read + write accesses, 2987920
bytes = 74698 x 40 B), so a replay can be built whose analysis must print
exactly that block.  Building it here (instead of committing a 3 MB binary)
keeps the fixture small; the construction is deterministic.

What the block pins: the __print_counters / print_call_site_summary /
mem_sampling_statistics formats, the progress line, call-site grouping by
(size, callstack[3..]), first-match id order, the weight sort with id
tie-break, nb_mallocs counting, and the [stack] entry (alloc = free = 0)
matching only timestamp-0 samples (quirk Q4).  The README was rendered by a
terminal (tabs expanded, "\\r" progress lines overwritten), so comparisons
collapse whitespace and keep the text after the last "\\r" of each line.
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from numamma_amd.replay import (  # noqa: E402
    ENTRY_DTYPE, LVL_HIT, LVL_L1, MEM_DYNAMIC, MEM_STACK, RECORD_DTYPE, STACK_BASE, STACK_END,
    Buffer, ObjectTable, Replay)

HERE = os.path.dirname(os.path.abspath(__file__))
EXPECTED = os.path.join(HERE, "readme_report.txt")
SRC = "/home/trahay/Soft/opt/numamma/test/mat_mul.c"


def normalize(text: str):
    """Terminal rendering of the report: text after the last '\\r' of each
    line, whitespace runs collapsed."""
    out = []
    for line in text.split("\n"):
        line = line.split("\r")[-1]
        out.append(" ".join(line.split()))
    while out and out[-1] == "":
        out.pop()
    return out


def build() -> Replay:
    rng = np.random.default_rng(2024)
    # ---- object table: call sites 2..5 are size-800 mallocs from four lines
    # of mat_mul.c, told apart by their call stacks (test/mat_mul.c:68-78)
    sites = [("70", 2), ("74", 2), ("78", 100), ("68", 1)]
    heap = []
    strings = bytearray()
    pool = []
    caller_off = {}
    for line, _ in sites:
        caller_off[line] = len(strings)
        strings += f"{SRC}:{line}(main)".encode() + b"\0"
    addr = 0x555555560000
    for si, (line, n) in enumerate(sites):
        for j in range(n):
            heap.append((addr, line, si))
            addr += 0x400
    K = len(heap) + 1
    ent = np.zeros(K, dtype=ENTRY_DTYPE)
    keys = np.zeros(K, dtype=np.uint64)
    for e, (a, line, si) in enumerate(heap):
        r = ent[e]
        keys[e] = a
        r["buffer_addr"] = a
        r["buffer_size"] = 800
        r["initial_buffer_size"] = 800
        r["alloc_date"] = 1_000_000_000
        r["free_date"] = 3_000_000_000
        r["caller_rip"] = 0x555555555000 + 0x10 * si
        r["mem_type"] = MEM_DYNAMIC
        r["caller_off"] = caller_off[line]
        cs = [0x7F0000001000 + e, 0x7F0000002000 + e, 0x7F0000003000 + e,  # interposer frames
              0x555555555000 + 0x10 * si, 0x555555556000, 0x7F0000004000]
        r["has_callstack"] = 1
        r["callstack_size"] = len(cs)
        r["callstack_off"] = sum(len(c) for c in pool)
        pool.append(np.array(cs, dtype=np.uint64))
    s = ent[K - 1]
    keys[K - 1] = STACK_BASE
    s["buffer_addr"] = STACK_BASE
    s["buffer_size"] = STACK_END - STACK_BASE
    s["initial_buffer_size"] = STACK_END - STACK_BASE
    s["mem_type"] = MEM_STACK
    s["caller_off"] = len(strings)
    strings += b"[stack]\0"
    ent["id"] = np.arange(1, K + 1)
    table = ObjectTable(keys, np.arange(K + 1, dtype=np.uint32), ent,
                        np.concatenate(pool), bytes(strings))
    first = {0: 0, 1: 2, 2: 4, 3: 104}  # first entry of each heap site

    # ---- samples: (addr, ts, weight, level)
    L1 = LVL_HIT | LVL_L1

    def stack(n, w):
        return [(int(rng.integers(0x7FFC00000000, 0x7FFF00000000)), 0, w, L1) for _ in range(n)]

    def obj(site, n, w):
        nobj = sites[site][1]
        out = []
        for i in range(n):
            e = first[site] + (i % nobj)
            out.append((int(keys[e]) + int(rng.integers(0, 800)), int(rng.integers(1_100_000_000, 2_900_000_000)), w, L1))
        return out

    def unmatched(n, w, lvl):
        return [(0x1000 + 8 * int(rng.integers(0, 512)), 2_000_000_000, w, lvl) for _ in range(n)]

    # sites[] order: 0 = :70, 1 = :74, 2 = :78 (100 objects), 3 = :68
    def shuffled(x):
        rng.shuffle(x)
        return x

    # first matches in analysis order give the README ids: [stack] 1, :70 2,
    # :74 3, :78 4 (all in the first, write, buffer), then :68 5 (first read buffer)
    writes = stack(1, 0) + obj(0, 1, 0) + obj(1, 1, 0) + obj(2, 1, 0) + shuffled(
        stack(3481, 0) + obj(2, 62015, 0) + obj(0, 607, 0) + obj(1, 607, 0) +
        unmatched(387, 0, L1) + unmatched(304, 0, 0))
    reads = obj(3, 1, 7) + shuffled(
        stack(3951, 7) + stack(912, 8) + obj(2, 608, 13) + obj(3, 607, 7) +
        unmatched(1207, 9, L1) + unmatched(2, 14, L1) + unmatched(5, 7, L1))
    assert len(writes) == 67405 and len(reads) == 7293

    # ---- 1214 buffers; the last 4 hold 8 samples (progress "1210/1214 ... 74690")
    tail_r, tail_w = reads[-4:], writes[-4:]
    reads, writes = reads[:-4], writes[:-4]
    nr, nw = 110, 1100
    rparts = np.array_split(np.arange(len(reads)), nr)
    wparts = np.array_split(np.arange(len(writes)), nw)
    order = []  # (access, list)
    ri = wi = 0
    for b in range(nr + nw):
        if b == 0 or (b % 11 != 1 and wi < nw) or ri >= nr:
            order.append((1, [writes[j] for j in wparts[wi]]))
            wi += 1
        else:
            order.append((0, [reads[j] for j in rparts[ri]]))
            ri += 1
    order += [(0, tail_r[:2]), (1, tail_w[:2]), (0, tail_r[2:]), (1, tail_w[2:])]
    buffers = []
    for b, (acc, recs) in enumerate(order):
        rec = np.zeros(len(recs), dtype=RECORD_DTYPE)
        rec["type"] = 9
        rec["misc"] = 2
        rec["size"] = 40
        rec["addr"] = [x[0] for x in recs]
        rec["timestamp"] = [x[1] for x in recs]
        rec["weight"] = [x[2] for x in recs]
        rec["data_src"] = [(x[3] << 5) | (0x2 if acc == 0 else 0x4) for x in recs]
        raw = np.frombuffer(rec.tobytes(), dtype=np.uint8).copy()
        buffers.append(Buffer(b % 4, acc, raw, 0, raw.shape[0]))
    assert len(buffers) == 1214
    return Replay(4, table, buffers, {"fixture": "README.md:80-107"})


def expected_lines():
    return normalize(open(EXPECTED).read())


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "readme_replay.bin"
    build().write(out)
    print("wrote", out)
