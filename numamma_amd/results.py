"""Canonical raw-results dump ("NMGRES01") and the host-only report.

Both the engine (nmg_run_replay(..., raw_path)) and the test oracle write
this format, so parity checks compare every counter bit for bit:

    "NMGRES01", u32 nb_entries, u32 nb_buffers, u32 nb_threads, u32 0
    u64 global[2][75]          struct mem_counters x {read, write}
    u64 nb_samples_total, u64 nb_found_total
    u32 buf_samples[B], u32 buf_found[B]
    u64 entry[E][79]           first-match ordinal, then per access:
                               count, weight, na_miss_count, 18 x (count, sum)
    u64 n, u32 cells[n][4]     (entry, thread, page, read+write count),
                               (entry, thread, page) order, non-zero only
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class RawResults:
    nb_entries: int
    nb_buffers: int
    nb_threads: int
    global_counters: np.ndarray  # u64[2][75]
    nb_samples: int
    nb_found: int
    buf_samples: np.ndarray
    buf_found: np.ndarray
    entries: np.ndarray  # u64[E][79]
    cells: np.ndarray  # u32[n][4]

    @staticmethod
    def read(path: str) -> "RawResults":
        raw = open(path, "rb").read()
        if raw[:8] != b"NMGRES01":
            raise ValueError("not a raw-results dump")
        E, B, T, _ = np.frombuffer(raw, "<u4", 4, 8)
        off = 24
        g = np.frombuffer(raw, "<u8", 150, off).reshape(2, 75).copy()
        off += 1200
        ns, nf = np.frombuffer(raw, "<u8", 2, off)
        off += 16
        bs = np.frombuffer(raw, "<u4", B, off).copy()
        off += 4 * B
        bf = np.frombuffer(raw, "<u4", B, off).copy()
        off += 4 * B
        ent = np.frombuffer(raw, "<u8", E * 79, off).reshape(E, 79).copy()
        off += 8 * 79 * E
        (n,) = np.frombuffer(raw, "<u8", 1, off)
        off += 8
        cells = np.frombuffer(raw, "<u4", 4 * int(n), off).reshape(int(n), 4).copy()
        return RawResults(int(E), int(B), int(T), g, int(ns), int(nf), bs, bf, ent, cells)

    @property
    def first_ordinal(self) -> np.ndarray:
        return self.entries[:, 0]

    @property
    def count_weight(self) -> np.ndarray:
        cw = np.zeros((self.nb_entries, 2, 2), dtype=np.uint64)
        cw[:, 0, 0] = self.entries[:, 1]
        cw[:, 0, 1] = self.entries[:, 2]
        cw[:, 1, 0] = self.entries[:, 1 + 39]
        cw[:, 1, 1] = self.entries[:, 2 + 39]
        return cw


def report_host(res: RawResults, table, buf_bytes: np.ndarray, output_dir: str,
                stdout_path: Optional[str], match_samples: bool = True, dump_single_items: int = 1,
                dump_flags: int = 0, modules=None, online: bool = False) -> None:
    """nmg_report_host(): the report from host arrays (no GPU involved).
    dump_flags: NMG_DUMP_ALL writes all_memory_objects.dat (the sample dumps
    need the engine's per-sample matches: nmg_report)."""
    from . import _lib
    from .engine import build_meta, table_objects

    hr = _lib.nmg_host_results()
    gbytes = np.ascontiguousarray(res.global_counters, dtype="<u8").tobytes()
    C.memmove(C.addressof(hr.global_), gbytes, len(gbytes))
    keep = []

    def p(a, dt, ct):
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a.ctypes.data_as(C.POINTER(ct))

    hr.nb_buffers = res.nb_buffers
    hr.nb_entries = res.nb_entries
    hr.buf_samples = p(res.buf_samples, np.uint32, C.c_uint32)
    hr.buf_found = p(res.buf_found, np.uint32, C.c_uint32)
    hr.buf_bytes = p(buf_bytes, np.uint64, C.c_uint64)
    hr.buffer_size = p(table.entries["buffer_size"], np.uint64, C.c_uint64)
    hr.first_ordinal = p(res.first_ordinal, np.uint64, C.c_uint64)
    hr.count_weight = p(res.count_weight, np.uint64, C.c_uint64)
    hr.cells = p(res.cells, np.uint32, C.c_uint32)
    hr.nb_cells = res.cells.shape[0]
    hr.nb_threads = res.nb_threads
    hr.match_samples = int(match_samples)
    objs = table_objects(table)
    keep.append(objs)
    hr.objects = objs.ctypes.data_as(C.POINTER(_lib.nmg_object))
    meta, kmeta = build_meta(table)
    marr, nmods = _lib.module_array(modules)
    ro = _lib.nmg_report_options(output_dir.encode(), dump_single_items, dump_flags, None, None, marr, nmods,
                                 int(online))
    _lib.check(_lib.lib.nmg_report_host(C.byref(hr), meta, C.byref(ro),
                                        stdout_path.encode() if stdout_path else None))
    del keep, kmeta
