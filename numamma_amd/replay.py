"""Replay format and synthetic PEBS workload generator.

A *replay* is what NumaMMa's offline analysis consumes at exit
(src/mem_sampling.c:311-346 + src/mem_analyzer.c:1802-1884):

* the object table -- the AVL tree of ``mem_analyzer.c`` after
  ``warn_non_freed_buffers`` and ``ma_register_stack``, flattened into sorted
  unique keys, each owning a newest-first (LIFO) list of entries
  (tools/hash.c:108-114);
* the ``samples`` list of captured perf ring segments in *analysis* order
  (the list is LIFO, so newest capture first, mem_sampling.c:729-730), each
  as ``struct sample_list`` (mem_sampling.c:61-71): thread rank, access type,
  ring bytes, ``data_tail``/``data_head``.

File layout (little endian, DESIGN.md "Replay format")::

    header 64 B: "NMGRPLY1", u32 version=1, u32 nb_threads, u32 nb_keys,
                 u32 nb_entries, u32 nb_buffers, u32 0, u64 callstack_pool_len,
                 u64 string_pool_bytes, u64 0, u64 0
    u64 keys[nb_keys]
    u32 entry_off[nb_keys+1]                       (padded to 8)
    entry[nb_entries] (72 B, ENTRY_DTYPE)
    u64 callstack_pool[]
    char string_pool[]                             (padded to 8)
    per buffer: u32 thread_rank, u32 access_type, u64 data_tail,
                u64 data_head, u64 ring_size, ring bytes (padded to 8)
    optional context (dump modes): "NMGMODS1", u32 nb_modules, u32 names_bytes,
                u32 maps_path_bytes, u32 maps_text_bytes, u64 0; per module
                u64 lo, u64 hi, u64 fbase, u32 name_off, u32 0; names pool,
                maps path, maps text (each padded to 8)

The generator follows SURVEY.md section 8(d): log-uniform object sizes with
gaps, ~3 % address reuse (same key, disjoint lifetimes), ~0.5 % realloc'd
objects (key != buffer_addr), 8 equal-size globals, the [stack] shadow range,
Zipf(1.1) object popularity, a fixed mem_lvl mix, integer read weights in
[1, 2000] and write weight 0.
"""
from __future__ import annotations

import dataclasses
import struct
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

MAX_THREADS = 1024  # src/numamma.h.in:9
PERF_RECORD_SAMPLE = 9
PERF_RECORD_LOST = 2
RECORD_BYTES = 40  # perf_event_header (8) + struct mem_sample (32), mem_analyzer.h:98-105
STACK_BASE = 0x7FA000000000  # ma_register_stack, mem_analyzer.c:639-641
STACK_END = 0x7FFFFFFFFFFF
HEAP_BASE = 0x555500000000
GLOBAL_BASE = 0x555400000000

# enum mem_type (mem_analyzer.h:58-64)
MEM_NONE, MEM_GLOBAL, MEM_STACK, MEM_DYNAMIC, MEM_LIB = range(5)

# PERF_MEM_LVL_* (linux/perf_event.h:1250-1263)
LVL_NA, LVL_HIT, LVL_MISS = 0x01, 0x02, 0x04
LVL_L1, LVL_LFB, LVL_L2, LVL_L3, LVL_LOC_RAM = 0x08, 0x10, 0x20, 0x40, 0x80
LVL_REM_RAM1, LVL_REM_RAM2, LVL_REM_CCE1, LVL_REM_CCE2 = 0x100, 0x200, 0x400, 0x800
LVL_IO, LVL_UNC = 0x1000, 0x2000
MEM_OP_LOAD, MEM_OP_STORE = 0x02, 0x04

ENTRY_DTYPE = np.dtype(
    [
        ("buffer_addr", "<u8"),
        ("buffer_size", "<u8"),
        ("initial_buffer_size", "<u8"),
        ("alloc_date", "<u8"),
        ("free_date", "<u8"),
        ("caller_rip", "<u8"),
        ("mem_type", "<u4"),
        ("id", "<u4"),
        ("callstack_off", "<u4"),
        ("callstack_size", "<i4"),
        ("caller_off", "<u4"),
        ("has_callstack", "<u4"),
    ]
)
assert ENTRY_DTYPE.itemsize == 72

RECORD_DTYPE = np.dtype(
    [
        ("type", "<u4"),
        ("misc", "<u2"),
        ("size", "<u2"),
        ("timestamp", "<u8"),
        ("addr", "<u8"),
        ("weight", "<u8"),
        ("data_src", "<u8"),
    ]
)
assert RECORD_DTYPE.itemsize == RECORD_BYTES

NO_CALLER = 0xFFFFFFFF


def _pad8(n: int) -> int:
    return (n + 7) & ~7


def flatten_insertions(keys_in_insertion_order):
    """Flatten a sequence of ht_insert(key) calls (tools/hash.c:204-231) the
    way the AVL tree stores them: unique keys ascending, each key's entries
    newest-first (__ht_new_entry pushes at the list head, hash.c:108-114).

    Returns (keys, entry_off, order) with order[flat position] = insertion
    index, i.e. the FOREACH_HASH visiting order (hash.h:75-78)."""
    k = np.asarray(keys_in_insertion_order, dtype=np.uint64)
    idx = np.arange(k.shape[0], dtype=np.int64)
    order = np.lexsort((-idx, k))  # key ascending, then insertion descending
    sk = k[order]
    uniq, first = np.unique(sk, return_index=True)
    entry_off = np.append(first, sk.shape[0]).astype(np.uint32)
    return uniq, entry_off, order


@dataclass
class ObjectTable:
    keys: np.ndarray  # u64[K] ascending, unique
    entry_off: np.ndarray  # u32[K+1]
    entries: np.ndarray  # ENTRY_DTYPE[E], per key newest-first
    callstack_pool: np.ndarray  # u64[]
    string_pool: bytes

    @property
    def nb_keys(self) -> int:
        return int(self.keys.shape[0])

    @property
    def nb_entries(self) -> int:
        return int(self.entries.shape[0])

    def caller(self, e: int) -> Optional[str]:
        off = int(self.entries["caller_off"][e])
        if off == NO_CALLER:
            return None
        end = self.string_pool.index(b"\0", off)
        return self.string_pool[off:end].decode()

    @classmethod
    def empty(cls) -> "ObjectTable":
        """No objects (a live host's table before the first allocation)."""
        return cls(keys=np.zeros(0, dtype=np.uint64), entry_off=np.zeros(1, dtype=np.uint32),
                   entries=np.zeros(0, dtype=ENTRY_DTYPE), callstack_pool=np.zeros(0, dtype=np.uint64),
                   string_pool=b"")

    def validate(self) -> None:
        k = self.keys
        if k.shape[0] > 1 and not np.all(k[1:] > k[:-1]):
            raise ValueError("keys must be strictly ascending")
        off = self.entry_off.astype(np.int64)
        if off[0] != 0 or off[-1] != self.nb_entries or np.any(off[1:] <= off[:-1]):
            raise ValueError("bad entry offsets")


@dataclass
class Buffer:
    """One ``struct sample_list`` (mem_sampling.c:61-71) before __copy_buffer."""

    thread_rank: int
    access_type: int
    ring: np.ndarray  # u8
    data_tail: int
    data_head: int

    def linear(self) -> np.ndarray:
        """__copy_buffer (mem_sampling.c:675-738): linearise [tail, head)."""
        t, h, r = self.data_tail, self.data_head, self.ring
        if h == t:
            return r[:0]
        if h < t:
            return np.concatenate([r[t:], r[:h]])
        return r[t:h]


CONTEXT_MAGIC = b"NMGMODS1"


def _context_section(modules, maps_path, maps_text) -> bytes:
    names = bytearray()
    mods = bytearray()
    for lo, hi, fb, fn in modules:
        mods += struct.pack("<QQQII", lo, hi, fb, len(names), 0)
        names += fn.encode() + b"\0"
    path = (maps_path or "").encode()
    text = (maps_text or "").encode()
    out = bytearray(CONTEXT_MAGIC + struct.pack("<IIIIQ", len(modules), len(names), len(path), len(text), 0))
    out += mods
    for part in (bytes(names), path, text):
        out += part + b"\0" * (_pad8(len(part)) - len(part))
    return bytes(out)


@dataclass
class Replay:
    nb_threads: int
    table: ObjectTable
    buffers: List[Buffer]
    meta: dict = field(default_factory=dict)
    # dump-mode context of the traced process: dladdr() module table
    # [(lo, hi, fbase, fname)] and /proc/<pid>/maps (path, text)
    modules: list = field(default_factory=list)
    maps_path: Optional[str] = None
    maps_text: Optional[str] = None

    # ------------------------------------------------------------------
    def write(self, path: str) -> None:
        t = self.table
        t.validate()
        with open(path, "wb") as f:
            hdr = struct.pack(
                "<8sIIIIIIQQQQ",
                b"NMGRPLY1",
                1,
                self.nb_threads,
                t.nb_keys,
                t.nb_entries,
                len(self.buffers),
                0,
                int(t.callstack_pool.shape[0]),
                len(t.string_pool),
                0,
                0,
            )
            assert len(hdr) == 64
            f.write(hdr)
            f.write(t.keys.astype("<u8").tobytes())
            eo = t.entry_off.astype("<u4").tobytes()
            f.write(eo + b"\0" * (_pad8(len(eo)) - len(eo)))
            f.write(t.entries.tobytes())
            f.write(t.callstack_pool.astype("<u8").tobytes())
            f.write(t.string_pool + b"\0" * (_pad8(len(t.string_pool)) - len(t.string_pool)))
            for b in self.buffers:
                ring = np.ascontiguousarray(b.ring, dtype=np.uint8)
                f.write(struct.pack("<IIQQQ", b.thread_rank, b.access_type, b.data_tail, b.data_head, ring.shape[0]))
                f.write(ring.tobytes())
                f.write(b"\0" * (_pad8(ring.shape[0]) - ring.shape[0]))
            if self.modules or self.maps_path or self.maps_text:
                f.write(_context_section(self.modules, self.maps_path, self.maps_text))

    @staticmethod
    def read(path: str) -> "Replay":
        data = np.fromfile(path, dtype=np.uint8)
        raw = data.tobytes()
        magic, ver, nthr, nk, ne, nb, _, cs_len, str_len, _, _ = struct.unpack_from("<8sIIIIIIQQQQ", raw, 0)
        if magic != b"NMGRPLY1" or ver != 1:
            raise ValueError("not a replay file")
        off = 64
        keys = np.frombuffer(raw, "<u8", nk, off).copy()
        off += 8 * nk
        entry_off = np.frombuffer(raw, "<u4", nk + 1, off).copy()
        off += _pad8(4 * (nk + 1))
        entries = np.frombuffer(raw, ENTRY_DTYPE, ne, off).copy()
        off += 72 * ne
        pool = np.frombuffer(raw, "<u8", cs_len, off).copy()
        off += 8 * cs_len
        strings = raw[off : off + str_len]
        off += _pad8(str_len)
        bufs = []
        for _ in range(nb):
            rank, acc, tail, head, ring = struct.unpack_from("<IIQQQ", raw, off)
            off += 32
            bufs.append(Buffer(rank, acc, data[off : off + ring].copy(), tail, head))
            off += _pad8(ring)
        rp = Replay(nthr, ObjectTable(keys, entry_off, entries, pool, strings), bufs)
        if off + 32 <= len(raw) and raw[off : off + 8] == CONTEXT_MAGIC:
            nm, nn, npath, ntext = struct.unpack_from("<IIII", raw, off + 8)
            off += 32
            mods = [struct.unpack_from("<QQQI", raw, off + 32 * i) for i in range(nm)]
            off += 32 * nm
            names = raw[off : off + nn]
            off += _pad8(nn)
            rp.maps_path = raw[off : off + npath].decode() if npath else None
            off += _pad8(npath)
            rp.maps_text = raw[off : off + ntext].decode() if ntext else None
            rp.modules = [(lo, hi, fb, names[no : names.index(b"\0", no)].decode()) for lo, hi, fb, no in mods]
        return rp

    # ------------------------------------------------------------------
    def linear_buffers(self):
        """Buffers as the analysis loop sees them (empty rings dropped)."""
        out = []
        for b in self.buffers:
            lin = b.linear()
            if lin.shape[0]:
                out.append((b.thread_rank, b.access_type, lin))
        return out

    def packed(self, align: int = 16):
        """Concatenate the linearised buffers into one arena (16-byte aligned
        offsets) for nmg_set_device_buffers: (arena u8, offsets, lengths,
        thread_ranks, access_types)."""
        lins = self.linear_buffers()
        lens = np.array([x[2].shape[0] for x in lins], dtype=np.uint64)
        padded = (lens + (align - 1)) // align * align
        offsets = np.zeros(len(lins), dtype=np.uint64)
        if len(lins):
            offsets[1:] = np.cumsum(padded)[:-1]
        total = int(padded.sum()) + 64
        arena = np.zeros(total, dtype=np.uint8)
        for (_, _, lin), o in zip(lins, offsets):
            arena[int(o) : int(o) + lin.shape[0]] = lin
        ranks = np.array([x[0] for x in lins], dtype=np.uint32)
        acc = np.array([x[1] for x in lins], dtype=np.uint32)
        return arena, offsets, lens, ranks, acc

    def nb_records(self) -> int:
        return int(sum(x[2].shape[0] for x in self.linear_buffers()) // RECORD_BYTES)


# ----------------------------------------------------------------------
# synthetic workload


@dataclass
class SynthConfig:
    nb_samples: int = 100_000
    nb_intervals: int = 1_000
    nb_threads: int = 8
    size_min: int = 64
    size_max: int = 256 * 1024
    reuse_frac: float = 0.03
    reuse_depth: int = 2  # entries per reused key (LIFO chain, disjoint lifetimes)
    realloc_frac: float = 0.005
    nb_globals: int = 8
    global_size: int = 8192
    with_stack: bool = True
    site_ratio: float = 0.1
    null_callstack_frac: float = 0.05
    zipf_s: float = 1.1
    frac_gap: float = 0.10
    frac_stack: float = 0.05
    frac_global: float = 0.02
    read_frac: float = 0.7
    buffer_records: int = 3276  # 128 KiB ring / 40 B (mem_sampling.c:298)
    lost_frac: float = 0.0
    wrap_one: bool = False
    seed: int = 1
    sample_seed: Optional[int] = None  # None: continue the table's stream
    # heap keys in `heap_clusters` runs, each `cluster_gap` bytes above the
    # previous one (mmap'd arenas far apart: the route pass's directory
    # segments); 1 = one contiguous heap
    heap_clusters: int = 1
    cluster_gap: int = 1 << 40


# named configurations from BASELINE.json "configs"
CONFIGS = {
    "c1": SynthConfig(nb_samples=100_000, nb_intervals=200, nb_threads=4),
    "c2": SynthConfig(nb_samples=10_000_000, nb_intervals=1_000),
    "c3": SynthConfig(nb_samples=100_000_000, nb_intervals=100_000),
    "c4": SynthConfig(nb_samples=1_000_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
}

_LVL_MIX = [
    (LVL_HIT | LVL_L1, 0.60),
    (LVL_HIT | LVL_L2, 0.10),
    (LVL_HIT | LVL_L3, 0.10),
    (LVL_HIT | LVL_LFB, 0.05),
    (LVL_HIT | LVL_LOC_RAM, 0.08),
    (LVL_HIT | LVL_REM_RAM1, 0.02),
    (LVL_MISS | LVL_L3, 0.02),
    (LVL_NA, 0.02),
    (0, 0.01),
]

T0 = 1_000_000_000_000  # ns; timestamps never 0 (so [stack] never matches, quirk Q4)
HORIZON = 10_000_000_000


def make_table(cfg: SynthConfig, rng: np.random.Generator) -> ObjectTable:
    K = cfg.nb_intervals
    G = max(1, int(round(K * cfg.site_ratio)))
    # call-site groups: one size, caller_rip and callstack tail each
    lo, hi = np.log(cfg.size_min), np.log(cfg.size_max)
    gsize = (np.exp(rng.uniform(lo, hi, G)).astype(np.uint64) + 7) // 8 * 8
    grip = rng.integers(0x555555554000, 0x555555600000, G, dtype=np.uint64)
    gnull = rng.random(G) < cfg.null_callstack_frac
    gdepth = rng.integers(4, 13, G)
    group = rng.integers(0, G, K)
    size = gsize[group]
    gap = (rng.random(K) * (size + 1)).astype(np.uint64) // 16 * 16
    stride = (size + 15) // 16 * 16 + gap
    keys = np.empty(K, dtype=np.uint64)
    keys[0] = HEAP_BASE
    if K > 1:
        keys[1:] = HEAP_BASE + np.cumsum(stride[:-1], dtype=np.uint64)
    if cfg.heap_clusters > 1:
        keys += (np.arange(K, dtype=np.uint64) * np.uint64(cfg.heap_clusters) // np.uint64(K)) * np.uint64(cfg.cluster_gap)
    reused = rng.random(K) < cfg.reuse_frac
    realloc = (rng.random(K) < cfg.realloc_frac) & ~reused

    # call stacks: frames [0..2] are interposer frames (random per object),
    # frames [3..] identify the call path (per group)
    pool = []
    pool_off = 0
    cs_off = np.zeros(K + 1, dtype=np.uint32)
    strings = bytearray()
    g_caller_off = np.zeros(G, dtype=np.uint32)
    for g in range(G):
        g_caller_off[g] = len(strings)
        strings += f"app.c:{100 + g}(func_{g % 97})".encode() + b"\0"
    g_tail = [rng.integers(0x400000, 0x500000, int(gdepth[g]) - 3, dtype=np.uint64) for g in range(G)]

    nper = np.where(reused, max(2, int(cfg.reuse_depth)), 1)
    nent = int(nper.sum())
    ent = np.zeros(nent, dtype=ENTRY_DTYPE)
    head_frames = rng.integers(0x7F0000000000, 0x7F0000100000, (nent, 3), dtype=np.uint64)
    alloc_jit = rng.integers(0, HORIZON // 100, (K, 2))
    # entries in key order, newest first (vectorised; the only random draws
    # inside the per-key walk are the realloc'd keys' offsets, taken in key
    # order as the scalar walk did)
    entry_off = np.zeros(K + 1, dtype=np.uint32)
    entry_off[1:] = np.cumsum(nper)
    ek = np.repeat(np.arange(K), nper)               # entry -> key
    ej = np.arange(nent) - entry_off[ek].astype(np.int64)  # 0 = newest
    eg = group[ek]
    ent["initial_buffer_size"] = size[ek]
    ent["buffer_addr"] = keys[ek]
    ent["buffer_size"] = size[ek]
    for k in np.flatnonzero(realloc):  # (never reused: one entry)
        e = int(entry_off[k])
        ent["buffer_addr"][e] = keys[k] + np.uint64(16 * int(rng.integers(1, 64)))
        ent["buffer_size"][e] = size[k] + np.uint64(16 * int(rng.integers(0, 512)))
    j0, j1 = alloc_jit[ek, 0].astype(np.uint64), alloc_jit[ek, 1].astype(np.uint64)
    # a key's d entries split the horizon: entry ej (0 = newest) lives in
    # slice d - 1 - ej (d = 1: the whole horizon)
    d = nper[ek].astype(np.uint64)
    seg = np.uint64(HORIZON) // d
    sl = d - np.uint64(1) - ej.astype(np.uint64)
    ent["alloc_date"] = np.uint64(T0) + j0 + sl * seg
    ent["free_date"] = np.uint64(T0) + (sl + np.uint64(1)) * seg - j1
    ent["caller_rip"] = grip[eg]
    ent["mem_type"] = MEM_DYNAMIC
    ent["caller_off"] = g_caller_off[eg]
    # call stacks: the entry's 3 interposer frames, then its group's tail
    tl = np.array([t.shape[0] for t in g_tail], dtype=np.int64)
    toff = np.zeros(G + 1, dtype=np.int64)
    toff[1:] = np.cumsum(tl)
    tails = np.concatenate(g_tail) if G else np.zeros(0, dtype=np.uint64)
    has = ~gnull[eg]
    clen = np.where(has, 3 + tl[eg], 0)
    coff = np.zeros(nent + 1, dtype=np.int64)
    coff[1:] = np.cumsum(clen)
    ent["has_callstack"] = has.astype(np.uint32)
    ent["callstack_size"] = clen.astype(np.int32)
    ent["callstack_off"] = np.where(has, coff[:-1], 0).astype(np.uint32)
    pe = np.repeat(np.arange(nent), clen)             # pool position -> entry
    pj = np.arange(coff[-1]) - coff[pe]               # position within the entry's stack
    pool_arr = np.where(pj < 3, head_frames[pe, np.minimum(pj, 2)],
                        tails[np.clip(toff[eg[pe]] + pj - 3, 0, max(0, tails.shape[0] - 1))] if tails.shape[0]
                        else np.uint64(0)).astype(np.uint64)
    e = nent
    keys_l = [keys]
    ent_l = [ent]
    off_l = [entry_off[:-1].astype(np.int64)]
    base = e
    # globals (insert_memory_info, mem_analyzer.c:680-731): alloc 0, free
    # stamped by warn_non_freed_buffers, no callstack, NULL caller_rip (Q6)
    if cfg.nb_globals:
        gk = GLOBAL_BASE + np.arange(cfg.nb_globals, dtype=np.uint64) * np.uint64(cfg.global_size * 2)
        ge = np.zeros(cfg.nb_globals, dtype=ENTRY_DTYPE)
        for i in range(cfg.nb_globals):
            ge[i]["buffer_addr"] = gk[i]
            ge[i]["buffer_size"] = cfg.global_size
            ge[i]["initial_buffer_size"] = cfg.global_size
            ge[i]["alloc_date"] = 0
            ge[i]["free_date"] = T0 + HORIZON + 1
            ge[i]["mem_type"] = MEM_GLOBAL
            ge[i]["caller_off"] = len(strings)
            strings += f"global_var_{i}".encode() + b"\0"
        keys_l.insert(0, gk)
        ent_l.insert(0, ge)
        off_l.insert(0, None)
    # [stack] (ma_register_stack after warn_non_freed_buffers: alloc = free = 0, Q4)
    if cfg.with_stack:
        se = np.zeros(1, dtype=ENTRY_DTYPE)
        se[0]["buffer_addr"] = STACK_BASE
        se[0]["buffer_size"] = STACK_END - STACK_BASE
        se[0]["initial_buffer_size"] = STACK_END - STACK_BASE
        se[0]["mem_type"] = MEM_STACK
        se[0]["caller_off"] = len(strings)
        strings += b"[stack]\0"
        keys_l.append(np.array([STACK_BASE], dtype=np.uint64))
        ent_l.append(se)
        off_l.append(None)
    keys_all = np.concatenate(keys_l)
    ent_all = np.concatenate(ent_l)
    # entry offsets: globals (1 each), heap (as built), stack (1)
    counts = []
    if cfg.nb_globals:
        counts.append(np.ones(cfg.nb_globals, dtype=np.int64))
    counts.append(np.diff(entry_off.astype(np.int64)))
    if cfg.with_stack:
        counts.append(np.ones(1, dtype=np.int64))
    cnt = np.concatenate(counts)
    eo = np.zeros(keys_all.shape[0] + 1, dtype=np.uint32)
    eo[1:] = np.cumsum(cnt)
    order = np.argsort(keys_all, kind="stable")
    assert np.all(order == np.arange(order.shape[0])), "regions are laid out in ascending order"
    ent_all["id"] = np.arange(1, ent_all.shape[0] + 1)
    return ObjectTable(keys_all, eo, ent_all, pool_arr.astype(np.uint64), bytes(strings))


def _records(n: int, rng: np.random.Generator, cfg: SynthConfig, table: ObjectTable,
             heap_keys: np.ndarray, heap_first: int, zipf_cdf: np.ndarray, access: int,
             t_lo: int, t_hi: int) -> np.ndarray:
    rec = np.zeros(n, dtype=RECORD_DTYPE)
    rec["type"] = PERF_RECORD_SAMPLE
    rec["misc"] = 2  # PERF_RECORD_MISC_USER
    rec["size"] = RECORD_BYTES
    ts = np.sort(rng.integers(t_lo, t_hi, n, dtype=np.uint64))
    rec["timestamp"] = ts
    u = rng.random(n)
    addr = np.zeros(n, dtype=np.uint64)
    ent = table.entries
    K = heap_keys.shape[0]
    # objects: Zipf over a random permutation of the heap keys
    cat_stack = u < cfg.frac_stack
    cat_gap = (u >= cfg.frac_stack) & (u < cfg.frac_stack + cfg.frac_gap)
    cat_glob = (u >= cfg.frac_stack + cfg.frac_gap) & (u < cfg.frac_stack + cfg.frac_gap + cfg.frac_global)
    cat_obj = ~(cat_stack | cat_gap | cat_glob)
    no = int(cat_obj.sum())
    if no:
        rank = np.searchsorted(zipf_cdf, rng.random(no))
        perm = _perm_cache(K, cfg.seed)
        k = perm[np.minimum(rank, K - 1)]
        e0 = table.entry_off[heap_first + k].astype(np.int64)
        e1 = table.entry_off[heap_first + k + 1].astype(np.int64)
        tso = ts[cat_obj]
        # newest entry whose lifetime has started (entries are newest-first,
        # allocations descending along the chain)
        e = e0.copy()
        ne = e1 - e0
        for i in range(1, int(ne.max()) if ne.shape[0] else 1):
            past = (ne > i) & (tso < ent["alloc_date"][np.minimum(e0 + i - 1, ent.shape[0] - 1)])
            e += past.astype(np.int64)
        base = ent["buffer_addr"][e]
        sz = ent["buffer_size"][e]
        addr[cat_obj] = base + (rng.random(no) * sz).astype(np.uint64)
    ng = int(cat_glob.sum())
    if ng and cfg.nb_globals:
        gi = rng.integers(0, cfg.nb_globals, ng)
        addr[cat_glob] = ent["buffer_addr"][gi] + (rng.random(ng) * cfg.global_size).astype(np.uint64)
    elif ng:
        cat_gap |= cat_glob
    ngap = int(cat_gap.sum())
    if ngap:
        k = rng.integers(0, K, ngap)
        e0 = table.entry_off[heap_first + k].astype(np.int64)
        start = heap_keys[k] + ent["initial_buffer_size"][e0]
        nxt = np.where(k + 1 < K, heap_keys[np.minimum(k + 1, K - 1)], start + np.uint64(4096))
        width = np.maximum(nxt - start, np.uint64(1))
        addr[cat_gap] = start + (rng.random(ngap) * width).astype(np.uint64)
    ns = int(cat_stack.sum())
    if ns:
        addr[cat_stack] = rng.integers(0x7FFC00000000, 0x7FFF00000000, ns, dtype=np.uint64)
    rec["addr"] = addr
    if access == 0:
        w = np.clip(np.round(np.exp(rng.normal(2.5, 1.2, n))), 1, 2000).astype(np.uint64)
    else:
        w = np.zeros(n, dtype=np.uint64)
    rec["weight"] = w
    probs = np.array([p for _, p in _LVL_MIX])
    lv = np.array([l for l, _ in _LVL_MIX], dtype=np.uint64)
    li = np.searchsorted(np.cumsum(probs) / probs.sum(), rng.random(n))
    op = MEM_OP_LOAD if access == 0 else MEM_OP_STORE
    # upper data_src fields (snoop / lock / tlb) are noise for the analyser
    noise = rng.integers(0, 1 << 16, n, dtype=np.uint64) << np.uint64(19)
    rec["data_src"] = (lv[np.minimum(li, lv.shape[0] - 1)] << np.uint64(5)) | np.uint64(op) | noise
    return rec


_PERM = {}


def _perm_cache(K: int, seed: int) -> np.ndarray:
    key = (K, seed)
    if key not in _PERM:
        _PERM.clear()
        _PERM[key] = np.random.default_rng(seed ^ 0x5EED).permutation(K)
    return _PERM[key]


def generate(cfg: SynthConfig) -> Replay:
    """Deterministic synthetic replay (seeded)."""
    rng = np.random.default_rng(cfg.seed)
    table = make_table(cfg, rng)
    if cfg.sample_seed is not None:  # same table, independent sample stream (shards)
        rng = np.random.default_rng(cfg.sample_seed)
    heap_first = cfg.nb_globals
    K = cfg.nb_intervals
    heap_keys = table.keys[heap_first : heap_first + K]
    ranks = np.arange(1, K + 1, dtype=np.float64)
    pmf = ranks ** (-cfg.zipf_s)
    cdf = np.cumsum(pmf) / pmf.sum()
    T = cfg.nb_threads
    per = []
    n_read = int(cfg.nb_samples * cfg.read_frac)
    n_write = cfg.nb_samples - n_read
    captures = []  # (start time, thread, access, records)
    for access, total in ((0, n_read), (1, n_write)):
        for t in range(T):
            n = total // T + (1 if t < total % T else 0)
            if n == 0:
                continue
            rec = _records(n, rng, cfg, table, heap_keys, heap_first, cdf, access, T0, T0 + HORIZON)
            for s in range(0, n, cfg.buffer_records):
                chunk = rec[s : s + cfg.buffer_records]
                captures.append((int(chunk["timestamp"][0]), t, access, chunk))
    captures.sort(key=lambda c: (c[0], c[1], c[2]))
    buffers: List[Buffer] = []
    for ts0, t, access, chunk in captures:
        raw = np.frombuffer(chunk.tobytes(), dtype=np.uint8)
        if cfg.lost_frac > 0:
            raw = _inject_lost(raw, chunk.shape[0], cfg.lost_frac, rng)
        buffers.append(Buffer(t, access, raw.copy(), 0, raw.shape[0]))
    if cfg.wrap_one and buffers:
        buffers[len(buffers) // 2] = _wrap(buffers[len(buffers) // 2], rng)
    buffers.reverse()  # `samples` is LIFO: analysis order = newest capture first
    meta = dataclasses.asdict(cfg)
    return Replay(T, table, buffers, meta)


def _inject_lost(raw: np.ndarray, nrec: int, frac: float, rng) -> np.ndarray:
    """Insert PERF_RECORD_LOST records (24 B: header, id, lost) between samples."""
    k = rng.binomial(nrec, frac)
    if k == 0:
        return raw
    pos = np.sort(rng.choice(nrec + 1, size=k, replace=False))
    parts = []
    prev = 0
    for p in pos:
        parts.append(raw[prev * RECORD_BYTES : p * RECORD_BYTES])
        lost = struct.pack("<IHHQQ", PERF_RECORD_LOST, 0, 24, int(rng.integers(1, 1 << 20)), int(rng.integers(1, 100)))
        parts.append(np.frombuffer(lost, dtype=np.uint8))
        prev = p
    parts.append(raw[prev * RECORD_BYTES :])
    return np.concatenate(parts)


def _wrap(b: Buffer, rng) -> Buffer:
    """Store a buffer as a wrapped ring segment (data_head < data_tail)."""
    lin = b.linear()
    n = lin.shape[0]
    cut = 8 * int(rng.integers(1, max(2, n // 8)))
    first, second = lin[:cut], lin[cut:]
    slack = np.full(64, 0xAB, dtype=np.uint8)  # stale ring bytes, never read
    ring = np.concatenate([second, slack, first])
    return Buffer(b.thread_rank, b.access_type, ring, second.shape[0] + 64, second.shape[0])


# ---------------------------------------------------------------------------
# --online-analysis: the object table at an alarm (mem_sampling.c:953-954)


def table_at(table: ObjectTable, t: int):
    """The flattened table as __process_samples sees it at an alarm at time t:
    an entry exists once it is allocated (alloc_date <= t; globals have 0), it
    carries its free_date only once freed (free_date <= t), 0 before (quirk Q3:
    a live object never matches), and a key exists while one of its entries
    does; entries keep their newest-first order.  Returns (keys, entry_off,
    entry_ids, ent4) for nmg_update_objects / the oracle's alarms, entry_ids
    indexing `table` (the final one)."""
    ent = table.entries
    present = ent["alloc_date"] <= np.uint64(t)
    eo = table.entry_off.astype(np.int64)
    key_of = np.repeat(np.arange(table.nb_keys), np.diff(eo))
    ids = np.flatnonzero(present).astype(np.uint32)
    kp = key_of[ids]
    keys_present = np.unique(kp)
    keys = table.keys[keys_present].astype(np.uint64)
    off = np.zeros(keys_present.shape[0] + 1, dtype=np.uint32)
    off[1:] = np.cumsum(np.bincount(np.searchsorted(keys_present, kp), minlength=keys_present.shape[0]))
    ent4 = np.zeros((ids.shape[0], 4), dtype=np.uint64)
    ent4[:, 0] = ent["buffer_addr"][ids]
    ent4[:, 1] = ent["buffer_size"][ids]
    ent4[:, 2] = ent["alloc_date"][ids]
    fr = ent["free_date"][ids]
    ent4[:, 3] = np.where(fr <= np.uint64(t), fr, np.uint64(0))
    return keys, off, ids, ent4


def online_alarms(replay: Replay, nb_alarms: int):
    """Split a replay whose buffers are in capture order (oldest first) and
    hold whole 40 B SAMPLE records into nb_alarms consecutive alarms of about
    equal buffer counts; each alarm fires just after the last sample it
    collects.  Returns [(buf_end, alarm_time)]."""
    nb = len(replay.buffers)
    lin = [b.linear() for b in replay.buffers]
    last_ts = np.array([int(x.view(RECORD_DTYPE)["timestamp"].max()) if x.shape[0] else 0 for x in lin],
                       dtype=np.uint64)
    cuts = [int(round(nb * (i + 1) / nb_alarms)) for i in range(nb_alarms)]
    out, b0, t = [], 0, 0
    for c in cuts:
        if c <= b0:
            continue
        t = max(t, int(last_ts[b0:c].max()) + 1)  # (alarms fire in time order)
        out.append((c, t))
        b0 = c
    return out
