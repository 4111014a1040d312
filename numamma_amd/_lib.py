"""ctypes binding of the C-ABI in include/numamma_gpu.h.

The shared library is built in-tree (numamma_amd/libnumamma_gpu.so, see
numamma_amd/Makefile and __graft_entry__.build()).  There is no fallback: if
the library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# (NMG_LIB_PATH: another in-tree build of the same library, for A/B timing
# of two kernel versions on one box; tools/ab_lib.sh.  Every export must still
# be there unless NMG_LIB_AB=1 says the build is an older A/B side.)
LIB_PATH = os.environ.get("NMG_LIB_PATH") or os.path.join(_HERE, "libnumamma_gpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "numamma_gpu.h")

# One HIP runtime per process: torch ships its own libamdhip64.so (same
# soname as /opt/rocm's).  Loaded first, it is the one the engine's
# libamdhip64.so.7 dependency resolves to; loaded after the engine, torch
# would bring a second runtime instance into the process, and on some boxes
# the second one to initialise finds no GPU.
try:
    import torch  # noqa: F401
except ImportError:  # (a process without torch uses /opt/rocm's runtime)
    pass

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `make -C numamma_amd` or "
        "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)"
    )
lib = C.CDLL(LIB_PATH)

NMG_OK = 0
NMG_F_MATCH_SAMPLES = 0x1
NMG_F_PAGE_HIST = 0x2
NMG_F_OBJECT_LEVELS = 0x4
NMG_F_SAMPLE_MATCHES = 0x8
NMG_F_SINGLE_PASS = 0x10  # large tables: single-pass attribute_kernel instead of the partition-first passes
NMG_F_DEFAULT = NMG_F_MATCH_SAMPLES | NMG_F_PAGE_HIST
NMG_F_ALL = NMG_F_MATCH_SAMPLES | NMG_F_PAGE_HIST | NMG_F_OBJECT_LEVELS | NMG_F_SAMPLE_MATCHES | NMG_F_SINGLE_PASS
NMG_OPTIONS_V1_SIZE = 32
NMG_DUMP_CALLSITES, NMG_DUMP_ALL, NMG_DUMP_UNMATCHED = 0x1, 0x2, 0x4
NMG_ARR_SUM64, NMG_ARR_MIN64, NMG_ARR_MAX64, NMG_ARR_HIST32 = range(4)
ERRORS = {
    -1: "NMG_ERR_INVALID",
    -2: "NMG_ERR_HIP",
    -3: "NMG_ERR_NOMEM",
    -4: "NMG_ERR_ZERO_SIZE",
    -5: "NMG_ERR_TRUNCATED",
    -6: "NMG_ERR_STATE",
    -7: "NMG_ERR_RANGE",
    -8: "NMG_ERR_CAPACITY",
    -9: "NMG_ERR_UNALIGNED",
    -10: "NMG_ERR_IO",
}


class nmg_count(C.Structure):
    _fields_ = [("count", C.c_uint64), ("min_weight", C.c_uint64), ("max_weight", C.c_uint64), ("sum_weight", C.c_uint64)]


class nmg_mem_counters(C.Structure):
    _fields_ = [
        ("total_count", C.c_uint64),
        ("total_weight", C.c_uint64),
        ("na_miss_count", C.c_uint64),
        ("b", nmg_count * 18),
    ]


class nmg_object(C.Structure):
    _fields_ = [("buffer_addr", C.c_uint64), ("buffer_size", C.c_uint64), ("alloc_date", C.c_uint64), ("free_date", C.c_uint64)]


class nmg_object_meta(C.Structure):
    _fields_ = [
        ("initial_buffer_size", C.c_uint64),
        ("caller_rip", C.c_uint64),
        ("callstack", C.POINTER(C.c_uint64)),
        ("callstack_size", C.c_int32),
        ("mem_type", C.c_uint32),
        ("caller", C.c_char_p),
        ("id", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


NMG_OPTIONS_ABI = 0x4E4D4702


class nmg_options(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("flags", C.c_uint32),
        ("nb_threads", C.c_uint32),
        ("copy_threads", C.c_uint32),
        ("hist_budget_bytes", C.c_uint64),
        ("sparse_capacity", C.c_uint64),
        ("nb_gpus", C.c_uint32),
        ("abi_version", C.c_uint32),  # NMG_OPTIONS_ABI: nb_gpus / devices are read
        ("devices", C.POINTER(C.c_int32)),
    ]


class nmg_module(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("hi", C.c_uint64), ("fbase", C.c_uint64), ("fname", C.c_char_p)]


class nmg_report_options(C.Structure):
    _fields_ = [("output_dir", C.c_char_p), ("dump_single_items", C.c_int32), ("dump_flags", C.c_int32),
                ("maps_path", C.c_char_p), ("maps_text", C.c_char_p),
                ("modules", C.POINTER(nmg_module)), ("nb_modules", C.c_uint32), ("online", C.c_uint32)]


def module_array(modules):
    """[(lo, hi, fbase, fname)] -> (nmg_module array, count) for nmg_report_options."""
    mods = list(modules or [])
    arr = (nmg_module * max(1, len(mods)))(*[nmg_module(lo, hi, fb, fn.encode()) for lo, hi, fb, fn in mods])
    return arr, len(mods)


class nmg_host_results(C.Structure):
    _fields_ = [
        ("global_", nmg_mem_counters * 2),
        ("nb_buffers", C.c_uint32),
        ("nb_entries", C.c_uint32),
        ("buf_samples", C.POINTER(C.c_uint32)),
        ("buf_found", C.POINTER(C.c_uint32)),
        ("buf_bytes", C.POINTER(C.c_uint64)),
        ("buffer_size", C.POINTER(C.c_uint64)),
        ("first_ordinal", C.POINTER(C.c_uint64)),
        ("count_weight", C.POINTER(C.c_uint64)),
        ("cells", C.POINTER(C.c_uint32)),
        ("nb_cells", C.c_int64),
        ("nb_threads", C.c_uint32),
        ("match_samples", C.c_uint32),
        ("objects", C.POINTER(nmg_object)),
    ]


class nmg_results_view(C.Structure):
    _fields_ = [
        ("global_", nmg_mem_counters * 2),
        ("nb_samples", C.c_uint64),
        ("nb_found", C.c_uint64),
        ("nb_buffers", C.c_uint32),
        ("nb_entries", C.c_uint32),
        ("buffer_samples", C.POINTER(C.c_uint32)),
        ("buffer_found", C.POINTER(C.c_uint32)),
        ("first_ordinal", C.POINTER(C.c_uint64)),
        ("count_weight", C.POINTER(C.c_uint64)),
        ("nb_cells", C.c_int64),
        ("cells", C.POINTER(C.c_uint32)),
    ]


assert C.sizeof(nmg_mem_counters) == 600
assert C.sizeof(nmg_object) == 32

P = C.c_void_p
u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
H = C.c_void_p  # nmg_engine*

_SIGS = {
    "nmg_strerror": (C.c_char_p, [C.c_int]),
    "nmg_get_last_error_detail": (C.c_int, [H, C.c_char_p, C.c_size_t]),
    "nmg_create": (C.c_int, [C.POINTER(H), C.POINTER(nmg_options)]),
    "nmg_create_ex": (C.c_int, [C.POINTER(H), C.c_void_p, C.c_size_t]),
    "nmg_destroy": (None, [H]),
    "nmg_set_objects": (C.c_int, [H, u64p, u32p, C.c_uint32, C.POINTER(nmg_object), C.c_uint32]),
    "nmg_update_objects": (C.c_int, [H, u64p, u32p, C.c_uint32, u32p, C.POINTER(nmg_object)]),
    "nmg_submit_ring": (C.c_int, [H, P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32]),
    "nmg_submit_buffer": (C.c_int, [H, P, C.c_uint64, C.c_uint32, C.c_uint32]),
    "nmg_submit_buffers": (C.c_int, [H, C.c_uint32, C.POINTER(C.c_void_p), u64p, u32p, u32p]),
    "nmg_register_host": (C.c_int, [H, C.c_void_p, C.c_uint64]),
    "nmg_unregister_host": (C.c_int, [H, C.c_void_p]),
    "nmg_stream_begin": (C.c_int, [H, C.c_uint64, C.c_uint32]),
    "nmg_stream_end": (C.c_int, [H]),
    "nmg_replay_open": (C.c_int, [C.POINTER(C.c_void_p), C.c_char_p, C.c_uint32, u64p, u32p, C.c_uint32,
                                  C.POINTER(nmg_object), C.POINTER(nmg_object_meta), C.c_uint32]),
    "nmg_replay_add_ring": (C.c_int, [C.c_void_p, P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32]),
    "nmg_replay_close": (C.c_int, [C.c_void_p]),
    "nmg_replay_set_context": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_char_p, C.c_char_p]),
    "nmg_set_device_buffers": (C.c_int, [H, P, u64p, u64p, u32p, u32p, C.c_uint32, C.c_uint64]),
    "nmg_analyze": (C.c_int, [H]),
    "nmg_synchronize": (C.c_int, [H]),
    "nmg_reset_counters": (C.c_int, [H]),
    "nmg_clear_buffers": (C.c_int, [H]),
    "nmg_get_global_counters": (C.c_int, [H, C.POINTER(nmg_mem_counters), u64p, u64p]),
    "nmg_get_nb_buffers": (C.c_uint32, [H]),
    "nmg_get_buffer_counts": (C.c_int, [H, u32p, u32p]),
    "nmg_get_object_counters": (C.c_int, [H, u64p, u64p]),
    "nmg_get_object_levels": (C.c_int, [H, u64p]),
    "nmg_count_page_cells": (C.c_int64, [H]),
    "nmg_get_page_cells": (C.c_int, [H, u32p, C.c_int64]),
    "nmg_results_begin": (C.c_int, [H]),
    "nmg_results_end": (C.c_int, [H, C.POINTER(nmg_results_view)]),
    "nmg_array_size": (C.c_uint64, [H, C.c_int]),
    "nmg_export_array": (C.c_int, [H, C.c_int, P]),
    "nmg_import_array": (C.c_int, [H, C.c_int, P]),
    "nmg_hist_pack": (C.c_int, [H, C.c_uint32, P, P, C.c_uint64, u64p]),
    "nmg_hist_unpack": (C.c_int, [H, P, P, C.c_uint64]),
    "nmg_objcw_pack": (C.c_int, [H, P, C.c_uint64, P, P, C.c_uint64, u64p]),
    "nmg_objcw_unpack": (C.c_int, [H, P, P, P, C.c_uint64]),
    "nmg_sparse_count": (C.c_int64, [H]),
    "nmg_sparse_export": (C.c_int, [H, u64p, u32p, C.c_int64]),
    "nmg_sparse_import": (C.c_int, [H, u64p, u32p, C.c_int64]),
    "nmg_set_buffer_counts": (C.c_int, [H, C.c_uint32, u32p, u32p, u64p]),
    "nmg_last_analyze_ms": (C.c_int, [H, C.POINTER(C.c_float)]),
    "nmg_get_merge_stats": (C.c_int, [H, C.POINTER(C.c_float), C.POINTER(C.c_uint64)]),
    "nmg_get_launch_times": (C.c_int, [H, C.POINTER(C.c_float), C.c_int]),
    "nmg_get_kernel_times": (C.c_int, [H, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int]),
    "nmg_debug_phase_times": (C.c_int, [H, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int]),
    "nmg_debug_route_count": (C.c_int, [H, u64p]),
    "nmg_report": (C.c_int, [H, C.POINTER(nmg_object_meta), C.POINTER(nmg_report_options), C.c_char_p]),
    "nmg_report_host": (C.c_int, [C.POINTER(nmg_host_results), C.POINTER(nmg_object_meta), C.POINTER(nmg_report_options), C.c_char_p]),
    "nmg_run_replay": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_uint32]),
}

_SKIPPED = []
for _name, (_res, _args) in _SIGS.items():
    if os.environ.get("NMG_LIB_AB") == "1" and not hasattr(lib, _name):
        _SKIPPED.append(_name)  # (A/B timing of an older build: functions it predates stay unbound)
        continue
    _fn = getattr(lib, _name)  # AttributeError == missing export: fail loudly
    _fn.restype = _res
    _fn.argtypes = _args
if _SKIPPED:
    import sys as _sys

    print(f"numamma_amd: NMG_LIB_AB=1, {LIB_PATH} lacks {', '.join(_SKIPPED)}", file=_sys.stderr)


def declared_symbols():
    """Names of every function declared in include/numamma_gpu.h."""
    import re

    src = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(nmg_[a-z_0-9]+)\s*\(", src)))


class NmgError(RuntimeError):
    def __init__(self, code: int, detail: str = ""):
        self.code = code
        name = ERRORS.get(code, str(code))
        msg = lib.nmg_strerror(code).decode()
        super().__init__(f"{name}: {msg}" + (f" ({detail})" if detail else ""))


def check(rc: int, h=None) -> int:
    if rc < 0:
        buf = C.create_string_buffer(512)
        lib.nmg_get_last_error_detail(h, buf, 512)  # (h None: the last failed nmg_create)
        detail = buf.value.decode(errors="replace")
        raise NmgError(rc, detail)
    return rc
