"""The C-ABI library loads, exports every symbol include/numamma_gpu.h
declares, and fails loudly (no CPU fallback) when no GPU is present."""
import ctypes as C
import os
import subprocess

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
