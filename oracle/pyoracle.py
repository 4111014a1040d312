"""TEST INFRASTRUCTURE ONLY -- ctypes access to the CPU oracle (liboracle.so)
and to the reference's own AVL index (oracle/_ref/libref_hash.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# (NMG_ORACLE_DIR: the sanitizer build of the oracle libraries, tools/sanitize.sh)
SO_DIR = os.environ.get("NMG_ORACLE_DIR") or HERE
ORACLE_SO = os.path.join(SO_DIR, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_hash.so")
REF_HASH_TEST = os.path.join(HERE, "_ref", "hash_test")


def build(quiet: bool = True) -> None:
    """make -C oracle (the reference pieces only build where /root/reference exists)."""
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL if quiet else None)


class _Module(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("hi", C.c_uint64), ("fbase", C.c_uint64), ("fname", C.c_char_p)]


class _Alarm(C.Structure):
    _fields_ = [("buf_end", C.c_uint32), ("nb_keys", C.c_uint32), ("keys", C.c_void_p), ("entry_off", C.c_void_p),
                ("entry_ids", C.c_void_p), ("ent4", C.c_void_p)]


class _Settings(C.Structure):
    _fields_ = [("match_samples", C.c_int), ("dump_single_items", C.c_int), ("dump", C.c_int),
                ("dump_all", C.c_int), ("dump_unmatched", C.c_int), ("reserved", C.c_int),
                ("maps_path", C.c_char_p), ("maps_text", C.c_char_p),
                ("modules", C.POINTER(_Module)), ("nb_modules", C.c_uint32), ("reserved2", C.c_uint32),
                ("alarms", C.POINTER(_Alarm)), ("nb_alarms", C.c_uint32), ("reserved3", C.c_uint32)]


class _Timing(C.Structure):
    _fields_ = [("analysis_s", C.c_double), ("total_s", C.c_double), ("nb_samples", C.c_uint64)]


_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build()
        lib = C.CDLL(ORACLE_SO)
        lib.nmo_run.restype = C.c_int
        lib.nmo_run.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(_Settings), C.POINTER(_Timing)]
        lib.nmo_strerror.restype = C.c_char_p
        lib.nmo_strerror.argtypes = [C.c_int]
        lib.nmo_lookup.restype = C.c_int64
        lib.nmo_lookup.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64]
        _oracle = lib
    return _oracle


def run(replay_path: str, outdir: str, stdout_path: str, raw_path: str | None = None,
        match_samples: bool = True, dump_single_items: bool = True, dump: bool = False,
        dump_all: bool = False, dump_unmatched: bool = False, maps_path: str | None = None,
        maps_text: str | None = None, modules=None, alarms=None) -> dict:
    """Dump modes (-d / -D / -u) write callsite_dump_<id>.dat, callsite_summary_<id>.dat,
    all_memory_accesses.dat, all_memory_objects.dat and unmatched_samples.log into
    outdir like the reference.  modules = [(lo, hi, fbase, fname)]: dladdr()'s view
    of the traced process, for all_memory_objects.dat.  alarms = [(buf_end, keys,
    entry_off, entry_ids, ent4)]: --online-analysis, each alarm's buffers against
    the table at that alarm (replay.table_at)."""
    import numpy as np

    lib = oracle()
    mods = list(modules or [])
    marr = (_Module * max(1, len(mods)))(*[_Module(lo, hi, fb, fn.encode()) for lo, hi, fb, fn in mods])
    keep = []
    al = list(alarms or [])
    aarr = (_Alarm * max(1, len(al)))()
    for i, (buf_end, keys, off, ids, ent4) in enumerate(al):
        arrs = [np.ascontiguousarray(keys, dtype=np.uint64), np.ascontiguousarray(off, dtype=np.uint32),
                np.ascontiguousarray(ids, dtype=np.uint32), np.ascontiguousarray(ent4, dtype=np.uint64)]
        keep += arrs
        aarr[i] = _Alarm(buf_end, arrs[0].shape[0], *[a.ctypes.data for a in arrs])
    s = _Settings(int(match_samples), int(dump_single_items), int(dump), int(dump_all), int(dump_unmatched), 0,
                  maps_path.encode() if maps_path else None, maps_text.encode() if maps_text else None,
                  marr, len(mods), 0, aarr, len(al), 0)
    t = _Timing()
    rc = lib.nmo_run(replay_path.encode(), outdir.encode(), stdout_path.encode(),
                     raw_path.encode() if raw_path else None, C.byref(s), C.byref(t))
    if rc:
        raise RuntimeError(f"oracle failed: {lib.nmo_strerror(rc).decode()} ({rc})")
    return {"analysis_s": t.analysis_s, "total_s": t.total_s, "nb_samples": t.nb_samples}


def lookup(keys, entry_off, ent4, addr: int, ts: int) -> int:
    import numpy as np

    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    entry_off = np.ascontiguousarray(entry_off, dtype=np.uint32)
    ent4 = np.ascontiguousarray(ent4, dtype=np.uint64)
    return oracle().nmo_lookup(keys.ctypes.data, entry_off.ctypes.data, keys.shape[0], ent4.ctypes.data, addr, ts)


_ref = None


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref():
    """The reference's tools/hash.c (unchanged) behind oracle/ref_hash_shim.c."""
    global _ref
    if _ref is None:
        lib = C.CDLL(REF_SO)
        lib.ref_reset.restype = None
        lib.ref_insert.argtypes = [C.c_uint64, C.c_uint64]
        lib.ref_insert.restype = None
        lib.ref_lower_key.argtypes = [C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int]
        lib.ref_lower_key.restype = C.c_int
        lib.ref_foreach.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int64]
        lib.ref_foreach.restype = C.c_int64
        lib.ref_size.restype = C.c_int
        _ref = lib
    return _ref


# ---- the multi-threaded restatement (oracle/nmg_cpu_mt.cpp)
class _MtTiming(C.Structure):
    _fields_ = [("load_s", C.c_double), ("analysis_s", C.c_double), ("merge_s", C.c_double),
                ("nb_samples", C.c_uint64), ("threads", C.c_int)]


_mt = None


def run_mt(replay_path: str, raw_path: str | None = None, threads: int = 16, levels: bool = True) -> dict:
    """Analyse a replay with `threads` host threads (bit-exact with run());
    returns the timings: load, parallel analysis, merge."""
    global _mt
    if _mt is None:
        so = os.path.join(SO_DIR, "liboracle_mt.so")
        if not os.path.exists(so):
            build()
        _mt = C.CDLL(so)
        _mt.nmo_mt_run.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(_MtTiming)]
        _mt.nmo_mt_run.restype = C.c_int
    t = _MtTiming()
    rc = _mt.nmo_mt_run(replay_path.encode(), raw_path.encode() if raw_path else None, threads, int(levels),
                        C.byref(t))
    if rc:
        raise RuntimeError(f"multi-threaded restatement failed ({rc})")
    return {"load_s": t.load_s, "analysis_s": t.analysis_s, "merge_s": t.merge_s, "nb_samples": t.nb_samples,
            "threads": t.threads}
