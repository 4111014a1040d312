"""Golden vectors from the reference README (README.md:115-131, 141-148,
159-175), on the CPU: the oracle reproduces call_sites.log,
callsite_counters_3.dat and the dump-mode callsite_dump_<id>.dat and
callsite_summary_<id>.dat blocks exactly (tests/golden/
readme_sites_fixture.py builds the replays), and the product's report writer
(numamma_amd.results.report_host, the C++ report of the C-ABI) prints the same
call_sites.log and callsite_counters files from the oracle's raw counters."""
import os

import numpy as np

import pyoracle
import readme_sites_fixture as F
from numamma_amd.results import RawResults, report_host


def test_readme_call_sites_and_counters(tmp_path):
    d = str(tmp_path)
    rp = F.build_call_sites()
    path = os.path.join(d, "r.bin")
    rp.write(path)
    bytes_per_buf = np.array([x[2].shape[0] for x in rp.linear_buffers()], dtype=np.uint64)
    table = rp.table
    del rp
    odir = os.path.join(d, "o")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"))
    os.remove(path)
    assert F.produced(os.path.join(odir, "call_sites.log")) == F.expected(F.CALL_SITES)
    assert F.produced(os.path.join(odir, "callsite_counters_3.dat")) == F.expected(F.COUNTERS_3)
    pdir = os.path.join(d, "p")
    report_host(RawResults.read(os.path.join(d, "o_raw.bin")), table, bytes_per_buf, pdir, os.path.join(d, "p.txt"))
    for f in sorted(os.listdir(odir)):
        assert open(os.path.join(odir, f), "rb").read() == open(os.path.join(pdir, f), "rb").read(), f
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "p.txt"), "rb").read()


def test_readme_callsite_summary(tmp_path):
    d = str(tmp_path)
    path = os.path.join(d, "r.bin")
    F.build_summary().write(path)
    odir = os.path.join(d, "o")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), dump=True)
    assert F.produced(os.path.join(odir, "callsite_summary_1.dat")) == F.expected(F.SUMMARY)


def test_readme_callsite_dump(tmp_path):
    d = str(tmp_path)
    path = os.path.join(d, "r.bin")
    F.build_dump().write(path)
    odir = os.path.join(d, "o")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), dump=True)
    assert F.dump_rows(os.path.join(odir, "callsite_dump_1.dat")) == F.dump_rows(F.DUMP)
