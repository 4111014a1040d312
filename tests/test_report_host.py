"""Host report writer (nmg_report_host, product C++) against the oracle (C),
and both against the reference README's example output -- all on CPU.

The oracle's raw-results dump feeds the product's report writer, so these
tests check the call-site registry, the sort and every printf format of the
product independently of the GPU kernels."""
import os

import numpy as np
import pytest

import pyoracle
import readme_fixture
from numamma_amd.replay import Replay, SynthConfig, generate
from numamma_amd.results import RawResults, report_host


def _run_oracle(rp: Replay, d, match=True):
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    os.makedirs(odir, exist_ok=True)
    pyoracle.run(path, odir, os.path.join(d, "oracle_stdout.txt"), os.path.join(d, "oracle_raw.bin"),
                 match_samples=match)
    return RawResults.read(os.path.join(d, "oracle_raw.bin")), odir


def _buf_bytes(rp: Replay):
    return np.array([x[2].shape[0] for x in rp.linear_buffers()], dtype=np.uint64)


def _compare_dirs(a, b):
    fa, fb = sorted(os.listdir(a)), sorted(os.listdir(b))
    assert fa == fb
    for f in fa:
        assert open(os.path.join(a, f), "rb").read() == open(os.path.join(b, f), "rb").read(), f


def test_readme_block_reproduced_by_oracle(tmp_path):
    rp = readme_fixture.build()
    _run_oracle(rp, str(tmp_path))
    got = readme_fixture.normalize(open(tmp_path / "oracle_stdout.txt", newline="").read())
    assert got == readme_fixture.expected_lines()


def test_readme_block_reproduced_by_product_report(tmp_path):
    rp = readme_fixture.build()
    raw, _ = _run_oracle(rp, str(tmp_path))
    out = str(tmp_path / "product")
    report_host(raw, rp.table, _buf_bytes(rp), out, str(tmp_path / "product_stdout.txt"))
    got = readme_fixture.normalize(open(tmp_path / "product_stdout.txt", newline="").read())
    assert got == readme_fixture.expected_lines()


@pytest.mark.parametrize("cfg", [
    SynthConfig(nb_samples=60_000, nb_intervals=400, seed=1),
    SynthConfig(nb_samples=40_000, nb_intervals=2_000, nb_threads=3, lost_frac=2e-3, wrap_one=True, seed=2),
    SynthConfig(nb_samples=30_000, nb_intervals=50, nb_threads=16, site_ratio=0.5, null_callstack_frac=0.5, seed=3),
    SynthConfig(nb_samples=20_000, nb_intervals=300, nb_globals=0, with_stack=False, reuse_frac=0.3,
                realloc_frac=0.2, seed=4),
])
def test_product_report_matches_oracle(tmp_path, cfg):
    rp = generate(cfg)
    raw, odir = _run_oracle(rp, str(tmp_path))
    pdir = str(tmp_path / "product")
    report_host(raw, rp.table, _buf_bytes(rp), pdir, str(tmp_path / "product_stdout.txt"))
    assert open(tmp_path / "oracle_stdout.txt", "rb").read() == open(tmp_path / "product_stdout.txt", "rb").read()
    _compare_dirs(odir, pdir)


def test_no_match_mode(tmp_path):
    rp = generate(SynthConfig(nb_samples=10_000, nb_intervals=100, seed=9))
    raw, odir = _run_oracle(rp, str(tmp_path), match=False)
    assert raw.nb_found == 0
    pdir = str(tmp_path / "product")
    report_host(raw, rp.table, _buf_bytes(rp), pdir, str(tmp_path / "p.txt"), match_samples=False)
    assert open(tmp_path / "oracle_stdout.txt", "rb").read() == open(tmp_path / "p.txt", "rb").read()


def test_sort_with_int_truncated_weights(tmp_path):
    """__sort_sites compares against an int-truncated running minimum (Q9):
    site read weights >= 2^31 exercise the exact selection simulation."""
    rp = generate(SynthConfig(nb_samples=30_000, nb_intervals=200, site_ratio=0.3, seed=12))
    raw, odir = _run_oracle(rp, str(tmp_path))
    rng = np.random.default_rng(0)
    matched = np.nonzero(raw.first_ordinal != np.uint64(2**64 - 1))[0]
    # inflate read weights of many objects past 2^31 (and some past 2^32)
    for e in matched:
        raw.entries[e, 2] = np.uint64(int(rng.integers(0, 3)) * (1 << 31) + int(rng.integers(0, 1 << 31)))
    pdir = str(tmp_path / "product")
    report_host(raw, rp.table, _buf_bytes(rp), pdir, str(tmp_path / "p.txt"))
    # restated O(S^2) selection on the same numbers (mem_analyzer.c:1531-1557)
    lines = [l for l in open(pdir + "/call_sites.log").read().splitlines()]
    ids = [int(l.split("\t")[0]) for l in lines]
    weights = {}
    for l in lines:
        sid = int(l.split("\t")[0])
        weights[sid] = int(l.split("total weight: ")[1].split(",")[0])
    # the printed list includes only sites with accesses; the selection runs on all sites,
    # but sites without accesses have weight 0 and never change the relative order of others
    lst = sorted(weights, reverse=True)  # LIFO list: newest (highest id) first
    head = []
    while lst:
        mw = weights[lst[0]] & 0xFFFFFFFF
        mw = mw - (1 << 32) if mw >= 1 << 31 else mw
        pick = lst[0]
        for s in lst:
            if weights[s] < (mw & 0xFFFFFFFFFFFFFFFF):
                mw = weights[s] & 0xFFFFFFFF
                mw = mw - (1 << 32) if mw >= 1 << 31 else mw
                pick = s
        lst.remove(pick)
        head.insert(0, pick)
    assert ids == head


# ---- all_memory_objects.dat (-D): print_object_summary, mem_analyzer.c:1642-1748
# dladdr()'s view of the traced process: the synthetic callstack tails live in
# [0x400000, 0x500000); frames in [0x4f0000, 0x500000) belong to no module.
MODULES = [(0x400000, 0x480000, 0x400000, "/usr/bin/app"), (0x480000, 0x4F0000, 0x470000, "/usr/lib/libfoo.so.1")]


def _expected_object_rows(table):
    """The row format restated a third time, from _print_object_summary's
    fprintf (:1699-1703) and its dladdr loop (:1660-1690)."""
    ent, pool, strings = table.entries, table.callstack_pool, table.string_pool
    rows = []
    for r in ent:
        if r["has_callstack"]:
            cs = [int(x) for x in pool[int(r["callstack_off"]):int(r["callstack_off"]) + int(r["callstack_size"])]]
            rips, offs = [], []
            for rip in cs[3:]:
                mod = next((m for m in MODULES if m[0] <= rip < m[1]), None)
                rips.append(f"0x{rip:x}")
                offs.append(f"{mod[3]}:{rip - mod[2]}" if mod else f"(null):{rip}")
            rips, offs = ",".join(rips), ",".join(offs)
        else:
            rips = offs = "NULL"
        if int(r["caller_off"]) != 0xFFFFFFFF:
            o = int(r["caller_off"])
            caller = strings[o:strings.index(b"\0", o)].decode()
        else:
            caller = "???" if int(r["caller_rip"]) == 0 else f"[0x{int(r['caller_rip']):x}]"
        rows.append(f"{int(r['id'])}\t0x{int(r['buffer_addr']):x}\t{int(r['buffer_size'])}\t{int(r['alloc_date'])}\t"
                    f"{int(r['free_date'])}\t{rips}\t{offs}\t0x{int(r['caller_rip']):x}\t{caller}\n")
    head = ("#object_id\taddress\tsize\tallocation_date\tdeallocation_date\tcallstack_rip\tcallstack_offsets"
            "\tcallsite_rip\tcallsite\n")
    return head + "".join(rows) * 2  # USE_HASHTABLE: mem_list printed twice (Q20)


@pytest.mark.parametrize("cfg", [
    SynthConfig(nb_samples=20_000, nb_intervals=300, lost_frac=2e-3, seed=21),
    SynthConfig(nb_samples=10_000, nb_intervals=120, null_callstack_frac=0.5, reuse_frac=0.3, realloc_frac=0.2,
                site_ratio=0.5, seed=22),
])
def test_all_memory_objects(tmp_path, cfg):
    """all_memory_objects.dat from the product's host report writer, the
    oracle, and the test's own restatement: byte-identical."""
    from numamma_amd import _lib

    d = str(tmp_path)
    rp = generate(cfg)
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    odir = os.path.join(d, "oracle")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), os.path.join(d, "raw.bin"), dump_all=True, modules=MODULES)
    raw = RawResults.read(os.path.join(d, "raw.bin"))
    pdir = os.path.join(d, "product")
    report_host(raw, rp.table, _buf_bytes(rp), pdir, os.path.join(d, "p.txt"), dump_flags=_lib.NMG_DUMP_ALL,
                modules=MODULES)
    want = _expected_object_rows(rp.table)
    got_o = open(os.path.join(odir, "all_memory_objects.dat"), newline="").read()
    got_p = open(os.path.join(pdir, "all_memory_objects.dat"), newline="").read()
    assert got_o == want
    assert got_p == want
    assert "(null):" in want and "/usr/lib/libfoo.so.1:" in want and "\tNULL\tNULL\t" in want
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "p.txt"), "rb").read()
    for f in ("call_sites.log",):
        assert open(os.path.join(odir, f), "rb").read() == open(os.path.join(pdir, f), "rb").read()


def test_report_files_independent_of_writer_threads(tmp_path, monkeypatch):
    """The per-site page files are written by a thread pool (NMG_REPORT_THREADS):
    one writer and many give the same bytes, and both match the oracle."""
    rp = generate(SynthConfig(nb_samples=50_000, nb_intervals=3_000, site_ratio=0.5, seed=5))
    raw, odir = _run_oracle(rp, str(tmp_path))
    outs = []
    for n in ("1", "7"):
        monkeypatch.setenv("NMG_REPORT_THREADS", n)
        pdir = str(tmp_path / f"product_{n}")
        report_host(raw, rp.table, _buf_bytes(rp), pdir, str(tmp_path / f"stdout_{n}.txt"))
        outs.append(pdir)
        _compare_dirs(odir, pdir)
    assert len(os.listdir(outs[0])) > 100  # many call sites: the pool has work to split
    assert open(tmp_path / "stdout_1.txt", "rb").read() == open(tmp_path / "stdout_7.txt", "rb").read()
