"""Python handle on the MI355X engine (thin wrapper over the C-ABI).

Mirrors the reference's analysis interface: ``set_objects`` takes the object
table snapshot, ``submit_ring`` is ``__copy_buffer`` (src/mem_sampling.c:675),
``analyze`` is the ``while(samples)`` loop of ``mem_sampling_finalize``
(:311-346) and ``report`` is the report half of ``ma_finalize``
(src/mem_analyzer.c:1802-1884).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from ._lib import check, lib
from .replay import ObjectTable, Replay


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def counters_to_numpy(c: "_lib.nmg_mem_counters") -> np.ndarray:
    """struct mem_counters -> u64[75] (total_count, total_weight, na, 18 x (count, min, max, sum))."""
    return np.frombuffer(bytes(c), dtype="<u8").copy()


def page_aligned_empty(nbytes: int) -> np.ndarray:
    """A u8 array of nbytes starting on a 4 KiB page, its last page its own
    (what nmg_register_host pins: whole pages)."""
    n = max(4096, (nbytes + 4095) // 4096 * 4096)
    buf = np.empty(n + 4096, dtype=np.uint8)
    off = (-buf.ctypes.data) % 4096
    return buf[off:off + n][:nbytes]


class Engine:
    def __init__(self, device: int = 0, flags: int = _lib.NMG_F_DEFAULT, nb_threads: int = 1,
                 hist_budget_bytes: int = 0, sparse_capacity: int = 0, copy_threads: int = 1,
                 devices=None):
        """devices: a list of GPU ordinals -> one engine sharding its host
        buffers over those GPUs (nmg_options.nb_gpus / devices)."""
        if devices is not None and len(devices) == 1:  # one GPU: nmg_options.device (nb_gpus <= 1 ignores devices)
            device, devices = int(devices[0]), None
        devs = (C.c_int32 * max(1, len(devices or [])))(*(devices or [device]))
        self._devs = devs
        opt = _lib.nmg_options(device, flags, nb_threads, copy_threads, hist_budget_bytes, sparse_capacity,
                               len(devices) if devices else 0, _lib.NMG_OPTIONS_ABI, devs if devices else None)
        h = _lib.H()
        check(lib.nmg_create(C.byref(h), C.byref(opt)))
        self.h = h
        self.flags = flags
        self.nb_threads = nb_threads
        self._keep = []
        self.table: Optional[ObjectTable] = None
        self.nb_entries = 0
        self.buffer_bytes: list = []  # lengths of the analysed (non-empty) buffers

    def close(self):
        if self.h:
            lib.nmg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, rc):
        return check(rc, self.h)

    # ------------------------------------------------------------------
    def set_objects(self, table: ObjectTable):
        objs = table_objects(table)
        keys = np.ascontiguousarray(table.keys, dtype=np.uint64)
        off = np.ascontiguousarray(table.entry_off, dtype=np.uint32)
        self._c(lib.nmg_set_objects(self.h, _ptr(keys, C.c_uint64), _ptr(off, C.c_uint32), keys.shape[0],
                                    objs.ctypes.data_as(C.POINTER(_lib.nmg_object)), table.nb_entries))
        self.table = table
        self.nb_entries = table.nb_entries  # (the engine's entry count: update_objects may add ids)

    def update_objects(self, keys: np.ndarray, entry_off: np.ndarray, entry_ids: np.ndarray, objs: np.ndarray):
        """nmg_update_objects: the table at an alarm (--online-analysis); objs in
        table_objects() layout, entry_ids = their ids in the set_objects table."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        off = np.ascontiguousarray(entry_off, dtype=np.uint32)
        ids = np.ascontiguousarray(entry_ids, dtype=np.uint32)
        objs = np.ascontiguousarray(objs)
        self._c(lib.nmg_update_objects(self.h, _ptr(keys, C.c_uint64), _ptr(off, C.c_uint32), keys.shape[0],
                                       _ptr(ids, C.c_uint32), objs.ctypes.data_as(C.POINTER(_lib.nmg_object))))
        if ids.shape[0]:
            self.nb_entries = max(self.nb_entries, int(ids.max()) + 1)

    def submit_ring(self, ring: np.ndarray, tail: int, head: int, thread_rank: int, access: int):
        ring = np.ascontiguousarray(ring, dtype=np.uint8)
        self._c(lib.nmg_submit_ring(self.h, ring.ctypes.data, ring.shape[0], tail, head, thread_rank, access))
        n = (head - tail) if head >= tail else ring.shape[0] - tail + head
        if n:
            self.buffer_bytes.append(n)

    def submit_buffer(self, data: np.ndarray, thread_rank: int, access: int):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        self._c(lib.nmg_submit_buffer(self.h, data.ctypes.data, data.shape[0], thread_rank, access))
        if data.shape[0]:
            self.buffer_bytes.append(data.shape[0])

    def submit_buffers(self, bufs):
        """nmg_submit_buffers: [(thread_rank, access, u8 array), ...] in analysis
        order, copied into pinned staging by the engine's copy threads."""
        n = len(bufs)
        arrs = [np.ascontiguousarray(b[2], dtype=np.uint8) for b in bufs]
        ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
        lens = np.array([a.shape[0] for a in arrs], dtype=np.uint64)
        ranks = np.array([b[0] for b in bufs], dtype=np.uint32)
        acc = np.array([b[1] for b in bufs], dtype=np.uint32)
        self._c(lib.nmg_submit_buffers(self.h, n, ptrs, _ptr(lens, C.c_uint64), _ptr(ranks, C.c_uint32),
                                       _ptr(acc, C.c_uint32)))
        self.buffer_bytes.extend(int(x) for x in lens if x)

    def submit_arena(self, arena: np.ndarray, offs, lens, ranks, acc):
        """nmg_submit_buffers over buffers laid out in one u8 host array:
        buffer i = arena[offs[i] : offs[i] + lens[i]] (analysis order), its
        pointers computed in numpy (no per-buffer Python objects; the arena
        registered with register_host is read in place)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        # bounds in signed 64-bit before the conversion: a negative offset
        # must not wrap to 2^64 - k and pass an unsigned check
        o64 = np.asarray(offs, dtype=np.int64)
        l64 = np.asarray(lens, dtype=np.int64)
        if o64.shape != l64.shape:
            raise ValueError("submit_arena: offs, lens, ranks and acc differ in length")
        if o64.size and (int(o64.min()) < 0 or int(l64.min()) < 0 or bool(np.any(o64 > arena.nbytes))
                         or bool(np.any(l64 > arena.nbytes - o64))):
            raise ValueError("submit_arena: a buffer lies outside the arena")
        offs = np.ascontiguousarray(o64, dtype=np.uint64)
        lens = np.ascontiguousarray(l64, dtype=np.uint64)
        ranks = np.ascontiguousarray(ranks, dtype=np.uint32)
        acc = np.ascontiguousarray(acc, dtype=np.uint32)
        n = offs.shape[0]
        if not (lens.shape[0] == ranks.shape[0] == acc.shape[0] == n):
            raise ValueError("submit_arena: offs, lens, ranks and acc differ in length")
        ptrs = offs + np.uint64(arena.ctypes.data)
        self._c(lib.nmg_submit_buffers(self.h, n, ptrs.ctypes.data_as(C.POINTER(C.c_void_p)),
                                       _ptr(lens, C.c_uint64), _ptr(ranks, C.c_uint32), _ptr(acc, C.c_uint32)))
        self.buffer_bytes.extend(lens[lens > 0].tolist())

    def register_host(self, arr: np.ndarray):
        """nmg_register_host over a host array the caller keeps alive (page
        aligned, its pages its own: page_aligned_empty): buffers submitted from
        inside it are read in place by the kernels (no copy)."""
        self._c(lib.nmg_register_host(self.h, C.c_void_p(arr.ctypes.data), arr.nbytes))

    def unregister_host(self, arr: np.ndarray):
        self._c(lib.nmg_unregister_host(self.h, C.c_void_p(arr.ctypes.data)))

    def stream_begin(self, chunk_bytes: int = 64 << 20, copy_threads: int = 1):
        """Streaming mode (configs[4]): chunks are uploaded and analysed while
        buffers keep arriving; analyze() flushes the last one."""
        self._c(lib.nmg_stream_begin(self.h, chunk_bytes, copy_threads))

    def stream_end(self):
        self._c(lib.nmg_stream_end(self.h))

    def submit_replay(self, replay: Replay):
        for b in replay.buffers:
            self.submit_ring(b.ring, b.data_tail, b.data_head, b.thread_rank, b.access_type)

    def set_device_buffers(self, d_ptr: int, offsets, lengths, ranks, access, seq_base: int = 0):
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        ranks = np.ascontiguousarray(ranks, dtype=np.uint32)
        access = np.ascontiguousarray(access, dtype=np.uint32)
        self._keep = [offsets, lengths, ranks, access]
        self._c(lib.nmg_set_device_buffers(self.h, C.c_void_p(d_ptr), _ptr(offsets, C.c_uint64),
                                           _ptr(lengths, C.c_uint64), _ptr(ranks, C.c_uint32),
                                           _ptr(access, C.c_uint32), offsets.shape[0], seq_base))
        self.buffer_bytes = [int(x) for x in lengths if x]

    def clear_buffers(self):
        self._c(lib.nmg_clear_buffers(self.h))
        self.buffer_bytes = []

    def analyze(self):
        self._c(lib.nmg_analyze(self.h))

    def synchronize(self):
        self._c(lib.nmg_synchronize(self.h))

    def reset(self):
        self._c(lib.nmg_reset_counters(self.h))

    def launch_times(self, n: int = 64):
        buf = (C.c_float * n)()
        cnt = self._c(lib.nmg_get_launch_times(self.h, buf, n))
        return [buf[i] for i in range(cnt)]

    def kernel_times(self, n: int = 64):
        """(attribution kernel ms, whole launch ms) of up to n recent launches."""
        a, t = (C.c_float * n)(), (C.c_float * n)()
        cnt = self._c(lib.nmg_get_kernel_times(self.h, a, t, n))
        return [a[i] for i in range(cnt)], [t[i] for i in range(cnt)]

    def phase_times(self, n: int = 64):
        """(first kernel ms, rest of the attribution ms) of up to n recent launches:
        route_kernel and the local pass (partition-first path), or
        attribute_kernel and nothing (single-pass path)."""
        a, t = (C.c_float * n)(), (C.c_float * n)()
        cnt = self._c(lib.nmg_debug_phase_times(self.h, a, t, n))
        return [a[i] for i in range(cnt)], [t[i] for i in range(cnt)]

    def route_count(self) -> int:
        """Analyses (streamed chunks) that took the partition-first path so far
        (internal; tests)."""
        n = C.c_uint64()
        self._c(lib.nmg_debug_route_count(self.h, C.byref(n)))
        return n.value

    def last_analyze_ms(self) -> float:
        ms = C.c_float()
        self._c(lib.nmg_last_analyze_ms(self.h, C.byref(ms)))
        return ms.value

    def merge_stats(self):
        """(merge ms, counter bytes per GPU) of a multi-GPU handle's last
        analysis (nmg_get_merge_stats); (0, 0) for a single-GPU engine."""
        ms, nb = C.c_float(), C.c_uint64()
        self._c(lib.nmg_get_merge_stats(self.h, C.byref(ms), C.byref(nb)))
        return ms.value, nb.value

    # ------------------------------------------------------------------
    def global_counters(self):
        out = (_lib.nmg_mem_counters * 2)()
        ns, nf = C.c_uint64(), C.c_uint64()
        self._c(lib.nmg_get_global_counters(self.h, out, C.byref(ns), C.byref(nf)))
        return np.stack([counters_to_numpy(out[0]), counters_to_numpy(out[1])]), ns.value, nf.value

    def buffer_counts(self):
        n = lib.nmg_get_nb_buffers(self.h)
        s = np.zeros(n, dtype=np.uint32)
        f = np.zeros(n, dtype=np.uint32)
        self._c(lib.nmg_get_buffer_counts(self.h, _ptr(s, C.c_uint32), _ptr(f, C.c_uint32)))
        return s, f

    def object_counters(self):
        E = max(self.table.nb_entries, self.nb_entries)
        first = np.zeros(E, dtype=np.uint64)
        cw = np.zeros((E, 2, 2), dtype=np.uint64)
        self._c(lib.nmg_get_object_counters(self.h, _ptr(first, C.c_uint64), _ptr(cw, C.c_uint64)))
        return first, cw

    def object_levels(self):
        E = max(self.table.nb_entries, self.nb_entries)
        lv = np.zeros((E, 2, 37), dtype=np.uint64)
        self._c(lib.nmg_get_object_levels(self.h, _ptr(lv, C.c_uint64)))
        return lv

    def page_cells(self) -> np.ndarray:
        n = lib.nmg_count_page_cells(self.h)
        self._c(n)
        rows = np.empty((n, 4), dtype=np.uint32)  # (every row written by the engine)
        self._c(lib.nmg_get_page_cells(self.h, _ptr(rows, C.c_uint32), n))
        return rows

    def results_begin(self):
        """nmg_results_begin: the results so far snapshotted on the device and
        copied to pinned host memory on a stream of their own; the engine may
        be reset and analyse again at once."""
        self._c(lib.nmg_results_begin(self.h))

    def results_end(self):
        """nmg_results_end: wait for the snapshot's copy; (global counters,
        nb_samples, nb_found, buffer samples, buffer found, first ordinals,
        count_weight [E, 2, 2], page-cell rows [n, 4]).  The arrays are views
        of the engine's pinned memory, valid until the next results_begin."""
        v = _lib.nmg_results_view()
        self._c(lib.nmg_results_end(self.h, C.byref(v)))

        def arr(ptr, n, shape=None):
            if not n:
                return np.zeros(shape or (0,), dtype=np.dtype(ptr._type_))
            a = np.ctypeslib.as_array(ptr, shape=(n,))
            return a.reshape(shape) if shape else a

        g = np.stack([counters_to_numpy(v.global_[0]), counters_to_numpy(v.global_[1])])
        nb, E, nc = v.nb_buffers, v.nb_entries, v.nb_cells
        return (g, int(v.nb_samples), int(v.nb_found), arr(v.buffer_samples, nb), arr(v.buffer_found, nb),
                arr(v.first_ordinal, E), arr(v.count_weight, 4 * E, (E, 2, 2)), arr(v.cells, 4 * nc, (nc, 4)))

    # ------------------------------------------------------------------
    def report(self, output_dir: str, stdout_path: Optional[str] = None, dump_single_items: int = 1,
               dump_flags: int = 0, maps_path: Optional[str] = None, maps_text: Optional[str] = None,
               modules=None, online: bool = False):
        """nmg_report; dump_flags = NMG_DUMP_* (engine created with
        NMG_F_SAMPLE_MATCHES | NMG_F_OBJECT_LEVELS); modules = [(lo, hi, fbase,
        fname)], dladdr()'s view of the traced process (all_memory_objects.dat)."""
        meta, keep = build_meta(self.table)
        marr, nmods = _lib.module_array(modules)
        ro = _lib.nmg_report_options(output_dir.encode(), dump_single_items, dump_flags,
                                     maps_path.encode() if maps_path else None,
                                     maps_text.encode() if maps_text else None, marr, nmods, int(online))
        self._c(lib.nmg_report(self.h, meta, C.byref(ro), stdout_path.encode() if stdout_path else None))
        del keep

    # ---- multi-GPU merge helpers
    def array_size(self, which: int) -> int:
        return int(lib.nmg_array_size(self.h, which))

    def export_array(self, which: int, d_dst: int):
        self._c(lib.nmg_export_array(self.h, which, C.c_void_p(d_dst)))

    def import_array(self, which: int, d_src: int):
        self._c(lib.nmg_import_array(self.h, which, C.c_void_p(d_src)))

    def hist_pack(self, threshold: int, d_u8: int, d_ovf: int, ovf_cap: int) -> int:
        """nmg_hist_pack: returns the number of overflow entries (> ovf_cap:
        the list is incomplete)."""
        n = C.c_uint64(0)
        self._c(lib.nmg_hist_pack(self.h, threshold, C.c_void_p(d_u8), C.c_void_p(d_ovf), ovf_cap, C.byref(n)))
        return n.value

    def hist_unpack(self, d_u8: int, d_ovf: int, n_ovf: int):
        self._c(lib.nmg_hist_unpack(self.h, C.c_void_p(d_u8), C.c_void_p(d_ovf), n_ovf))

    def objcw_pack(self, d_sum64: int, threshold: int, d_u32: int, d_ovf: int, ovf_cap: int) -> int:
        """nmg_objcw_pack over a sum64 image: returns the number of (row word,
        value) pairs (> ovf_cap: the list is incomplete)."""
        n = C.c_uint64(0)
        self._c(lib.nmg_objcw_pack(self.h, C.c_void_p(d_sum64), threshold, C.c_void_p(d_u32), C.c_void_p(d_ovf),
                                   ovf_cap, C.byref(n)))
        return n.value

    def objcw_unpack(self, d_sum64: int, d_u32: int, d_ovf: int, n_ovf: int):
        self._c(lib.nmg_objcw_unpack(self.h, C.c_void_p(d_sum64), C.c_void_p(d_u32), C.c_void_p(d_ovf), n_ovf))

    def sparse_export(self):
        n = lib.nmg_sparse_count(self.h)
        self._c(n)
        k = np.zeros(n, dtype=np.uint64)
        v = np.zeros(n, dtype=np.uint32)
        self._c(lib.nmg_sparse_export(self.h, _ptr(k, C.c_uint64), _ptr(v, C.c_uint32), n))
        return k, v

    def sparse_import(self, keys: np.ndarray, counts: np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        counts = np.ascontiguousarray(counts, dtype=np.uint32)
        self._c(lib.nmg_sparse_import(self.h, _ptr(keys, C.c_uint64), _ptr(counts, C.c_uint32), keys.shape[0]))

    def set_buffer_counts(self, samples: np.ndarray, found: np.ndarray, nbytes: np.ndarray):
        samples = np.ascontiguousarray(samples, dtype=np.uint32)
        found = np.ascontiguousarray(found, dtype=np.uint32)
        nbytes = np.ascontiguousarray(nbytes, dtype=np.uint64)
        self._c(lib.nmg_set_buffer_counts(self.h, samples.shape[0], _ptr(samples, C.c_uint32),
                                          _ptr(found, C.c_uint32), _ptr(nbytes, C.c_uint64)))


def table_objects(table: ObjectTable) -> np.ndarray:
    """struct nmg_object[] (buffer_addr, buffer_size, alloc_date, free_date) of a table."""
    ent = table.entries
    objs = np.zeros(table.nb_entries, dtype=[("a", "<u8"), ("s", "<u8"), ("al", "<u8"), ("fr", "<u8")])
    objs["a"] = ent["buffer_addr"]
    objs["s"] = ent["buffer_size"]
    objs["al"] = ent["alloc_date"]
    objs["fr"] = ent["free_date"]
    return objs


def write_replay_c(path: str, replay: Replay) -> None:
    """Record a replay through the C-ABI capture bridge (nmg_replay_open /
    add_ring / close): what the LD_PRELOAD host calls at finalize."""
    t = replay.table
    objs = table_objects(t)
    meta, keep = build_meta(t)
    keys = np.ascontiguousarray(t.keys, dtype=np.uint64)
    off = np.ascontiguousarray(t.entry_off, dtype=np.uint32)
    w = C.c_void_p()
    check(lib.nmg_replay_open(C.byref(w), path.encode(), replay.nb_threads, _ptr(keys, C.c_uint64),
                              _ptr(off, C.c_uint32), keys.shape[0], objs.ctypes.data_as(C.POINTER(_lib.nmg_object)),
                              meta, t.nb_entries))
    try:
        for b in replay.buffers:
            ring = np.ascontiguousarray(b.ring, dtype=np.uint8)
            check(lib.nmg_replay_add_ring(w, ring.ctypes.data, ring.shape[0], b.data_tail, b.data_head,
                                          b.thread_rank, b.access_type))
        if replay.modules or replay.maps_path or replay.maps_text:
            marr, nmods = _lib.module_array(replay.modules)
            check(lib.nmg_replay_set_context(w, C.cast(marr, C.c_void_p), nmods,
                                             replay.maps_path.encode() if replay.maps_path else None,
                                             replay.maps_text.encode() if replay.maps_text else None))
    finally:
        check(lib.nmg_replay_close(w))


def build_meta(table: ObjectTable):
    """nmg_object_meta[] for the call-site registry (+ objects to keep alive),
    filled with numpy in the struct's layout (include/numamma_gpu.h)."""
    E = table.nb_entries
    dt = np.dtype([("initial_buffer_size", "<u8"), ("caller_rip", "<u8"), ("callstack", "<u8"),
                   ("callstack_size", "<i4"), ("mem_type", "<u4"), ("caller", "<u8"), ("id", "<u4"),
                   ("reserved", "<u4")])
    assert dt.itemsize == C.sizeof(_lib.nmg_object_meta)
    arr = np.zeros(max(E, 1), dtype=dt)
    ent = table.entries
    pool = np.ascontiguousarray(table.callstack_pool, dtype=np.uint64)
    strings = C.create_string_buffer(table.string_pool + b"\0", len(table.string_pool) + 1)
    if E:
        arr["initial_buffer_size"][:E] = ent["initial_buffer_size"]
        arr["caller_rip"][:E] = ent["caller_rip"]
        arr["callstack_size"][:E] = ent["callstack_size"]
        arr["mem_type"][:E] = ent["mem_type"]
        arr["id"][:E] = ent["id"]
        has_cs = ent["has_callstack"] != 0
        arr["callstack"][:E] = np.where(has_cs, np.uint64(pool.ctypes.data) + np.uint64(8) *
                                        ent["callstack_off"].astype(np.uint64), np.uint64(0))
        has_caller = ent["caller_off"].astype(np.uint64) != 0xFFFFFFFF
        arr["caller"][:E] = np.where(has_caller, np.uint64(C.addressof(strings)) +
                                     ent["caller_off"].astype(np.uint64), np.uint64(0))
    meta = (_lib.nmg_object_meta * E).from_buffer(arr)
    return meta, (pool, strings, arr)


def run_replay(path: str, output_dir: str, stdout_path: Optional[str] = None, raw_path: Optional[str] = None,
               device: int = 0, flags: int = _lib.NMG_F_DEFAULT) -> None:
    """The nmg_replay CLI in-process (C++ driver)."""
    check(lib.nmg_run_replay(path.encode(), output_dir.encode(), stdout_path.encode() if stdout_path else None,
                             raw_path.encode() if raw_path else None, device, flags))
