"""The C-ABI library loads, exports every symbol include/numamma_gpu.h
declares, and fails loudly (no CPU fallback) when no GPU is present."""
import ctypes as C
import os
import subprocess
import sys

import pytest
import torch

from numamma_amd import _lib


def test_all_declared_symbols_exported():
    declared = _lib.declared_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(_lib.lib, s)]
    assert missing == []


def test_strerror_names_every_code():
    for code in range(-10, 1):
        msg = _lib.lib.nmg_strerror(code).decode()
        assert msg and msg != "unknown error"


def test_struct_layouts_match_reference():
    # struct mem_counters is 600 bytes in the reference (mem_analyzer.h:17-41)
    assert C.sizeof(_lib.nmg_mem_counters) == 600
    assert C.sizeof(_lib.nmg_count) == 32


@pytest.mark.skipif(torch.cuda.device_count() > 0, reason="GPU present")
def test_create_fails_loudly_without_gpu():
    from numamma_amd.engine import Engine

    with pytest.raises(_lib.NmgError) as ei:
        Engine(device=0)
    assert ei.value.code == -2  # NMG_ERR_HIP


def test_null_arguments_rejected():
    assert _lib.lib.nmg_create(None, None) == -1
    assert _lib.lib.nmg_analyze(None) == -1
    assert _lib.lib.nmg_report_host(None, None, None, None) == -1


def test_header_compiles_as_c99(tmp_path):
    """include/numamma_gpu.h from a plain C99 translation unit: the test host
    of INTEGRATION.md section 1 (tests/c/nmg_c99_host.c) compiles with
    -std=c99 -Wall -Wextra -Werror -pedantic and links against the library."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(str(tmp_path), "host")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                    "-I" + os.path.join(root, "include"), os.path.join(root, "tests", "c", "nmg_c99_host.c"),
                    "-o", exe, "-L" + os.path.join(root, "numamma_amd"), "-lnumamma_gpu"], check=True)
    assert os.path.exists(exe)


def test_options_abi_version_matches_header():
    """nmg_options.abi_version gates nb_gpus / devices (older, shorter structs
    get a one-GPU engine): the binding's layout and magic follow the header."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "numamma_gpu.h")).read()
    assert "#define NMG_OPTIONS_ABI 0x4e4d4702u" in hdr
    assert _lib.NMG_OPTIONS_ABI == 0x4E4D4702
    assert C.sizeof(_lib.nmg_options) == 48
    assert _lib.nmg_options.abi_version.offset == 36 and _lib.nmg_options.devices.offset == 40


def _opts(**kw):
    o = _lib.nmg_options()
    o.device = 0
    o.flags = _lib.NMG_F_DEFAULT
    o.nb_threads = 8
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _create(o, size=None):
    h = C.c_void_p()
    if size is None:
        rc = _lib.lib.nmg_create(C.byref(h), C.byref(o))
    else:
        rc = _lib.lib.nmg_create_ex(C.byref(h), C.byref(o), size)
    if rc == 0:
        _lib.lib.nmg_destroy(h)
    return rc


def test_internal_flag_bits_rejected(monkeypatch):
    """Bits outside NMG_F_ALL (the internal ablation switches, e.g. 0x200 no
    global counters, 0x1000000 no object counters) are refused with
    NMG_ERR_INVALID before any GPU call, unless NMG_INTERNAL_FLAGS is set."""
    monkeypatch.delenv("NMG_INTERNAL_FLAGS", raising=False)
    for bad in (0x200, 0x1000000, 0x8000000, 0x20, 0x80000000):
        assert _create(_opts(flags=_lib.NMG_F_DEFAULT | bad)) == -1, hex(bad)
    detail = C.create_string_buffer(512)
    _lib.lib.nmg_get_last_error_detail(None, detail, 512)
    assert b"NMG_F_ALL" in detail.value
    # public flags pass validation (then: an engine, or NMG_ERR_HIP without a GPU)
    assert _create(_opts(flags=_lib.NMG_F_ALL)) in (0, -2)
    monkeypatch.setenv("NMG_INTERNAL_FLAGS", "1")
    assert _create(_opts(flags=_lib.NMG_F_DEFAULT | 0x20000)) in (0, -2)


def test_multi_gpu_without_abi_version_rejected(monkeypatch):
    """nb_gpus > 1 is used only with abi_version = NMG_OPTIONS_ABI.  A caller
    that declares the v2 fields (nmg_create_ex with the full struct size)
    fails without it instead of building a silent one-GPU engine; nmg_create,
    which a first-version binary may call with 32 bytes of struct, ignores
    nb_gpus / devices without the ABI word (stray bytes past that struct)."""
    devs = (C.c_int32 * 2)(0, 1)
    full = C.sizeof(_lib.nmg_options)
    assert _create(_opts(nb_gpus=2, devices=devs), full) == -1
    assert _create(_opts(nb_gpus=2, abi_version=0x4E4D4701, devices=devs), full) == -1
    assert _create(_opts(nb_gpus=2, devices=devs)) in (0, -2)  # nmg_create: one GPU, as in version 1
    assert _create(_opts(nb_gpus=0x7fffffff, abi_version=0x12345678)) in (0, -2)
    assert _create(_opts(nb_gpus=1), full) in (0, -2)  # one GPU: nothing to gate


def test_create_ex_reads_only_the_first_struct_version(tmp_path):
    """A first-version caller's 32-byte nmg_options placed right before an
    unreadable page: nmg_create_ex(opt, NMG_OPTIONS_V1_SIZE) reads only those
    bytes (an over-read would fault the child process)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r"""
import ctypes as C, mmap, sys
sys.path.insert(0, %r)
from numamma_amd import _lib
libc = C.CDLL(None)
m = mmap.mmap(-1, 2 * mmap.PAGESIZE)
base = C.addressof(C.c_char.from_buffer(m))
assert libc.mprotect(C.c_void_p(base + mmap.PAGESIZE), C.c_size_t(mmap.PAGESIZE), 0) == 0
o = _lib.nmg_options(); o.device = 0; o.flags = _lib.NMG_F_DEFAULT; o.nb_threads = 4
p = base + mmap.PAGESIZE - _lib.NMG_OPTIONS_V1_SIZE
C.memmove(p, C.addressof(o), _lib.NMG_OPTIONS_V1_SIZE)
h = C.c_void_p()
rc = _lib.lib.nmg_create_ex(C.byref(h), C.c_void_p(p), _lib.NMG_OPTIONS_V1_SIZE)
if rc == 0: _lib.lib.nmg_destroy(h)
bad = _lib.nmg_options(); bad.flags = 0x200
C.memmove(p, C.addressof(bad), _lib.NMG_OPTIONS_V1_SIZE)
rc2 = _lib.lib.nmg_create_ex(C.byref(h), C.c_void_p(p), _lib.NMG_OPTIONS_V1_SIZE)
rc3 = _lib.lib.nmg_create_ex(C.byref(h), C.c_void_p(p), 16)
print(rc, rc2, rc3)
""" % root
    env = dict(os.environ)
    env.pop("NMG_INTERNAL_FLAGS", None)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    rc, rc2, rc3 = map(int, out.stdout.split()[-3:])
    assert rc in (0, -2) and rc2 == -1 and rc3 == -1
