"""README golden vectors on the GPU (README.md:115-131, 141-148, 159-175; replays from
tests/golden/readme_sites_fixture.py): the engine's call_sites.log,
callsite_counters_3.dat and dump-mode callsite_dump_1.dat / callsite_summary_1.dat
equal the README blocks, and every output file equals the oracle's byte for byte."""
import os

import pytest

import pyoracle
import readme_sites_fixture as F
from numamma_amd import _lib

pytestmark = pytest.mark.gpu


def _same_dirs(a, b):
    fa, fb = sorted(os.listdir(a)), sorted(os.listdir(b))
    assert fa == fb
    for f in fa:
        assert open(os.path.join(a, f), "rb").read() == open(os.path.join(b, f), "rb").read(), f


def test_readme_call_sites_on_gpu(tmp_path):
    """58.9M records through the replay driver (nmg_run_replay: staged
    buffers, attribution, report)."""
    from numamma_amd.engine import run_replay

    d = str(tmp_path)
    path = os.path.join(d, "r.bin")
    F.build_call_sites().write(path)
    odir, edir = os.path.join(d, "o"), os.path.join(d, "e")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"))
    run_replay(path, edir, os.path.join(d, "e.txt"))
    os.remove(path)
    assert F.produced(os.path.join(edir, "call_sites.log")) == F.expected(F.CALL_SITES)
    assert F.produced(os.path.join(edir, "callsite_counters_3.dat")) == F.expected(F.COUNTERS_3)
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)


def test_readme_callsite_summary_on_gpu(tmp_path):
    """Dump mode (-d): per-object level buckets and every sample's match kept
    on the device, callsite_summary_1.dat written by the report."""
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = F.build_summary()
    path = os.path.join(d, "r.bin")
    rp.write(path)
    odir, edir = os.path.join(d, "o"), os.path.join(d, "e")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), dump=True)
    eng = Engine(flags=_lib.NMG_F_DEFAULT | _lib.NMG_F_SAMPLE_MATCHES | _lib.NMG_F_OBJECT_LEVELS,
                 nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    eng.report(edir, os.path.join(d, "e.txt"), dump_flags=_lib.NMG_DUMP_CALLSITES)
    eng.close()
    assert F.produced(os.path.join(edir, "callsite_summary_1.dat")) == F.expected(F.SUMMARY)
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)


def test_readme_callsite_dump_on_gpu(tmp_path):
    """Dump mode (-d): the six README rows of callsite_dump_1.dat from the
    engine's per-record matches (first five columns; the README has no
    access_type column)."""
    from numamma_amd.engine import Engine

    d = str(tmp_path)
    rp = F.build_dump()
    path = os.path.join(d, "r.bin")
    rp.write(path)
    odir, edir = os.path.join(d, "o"), os.path.join(d, "e")
    pyoracle.run(path, odir, os.path.join(d, "o.txt"), dump=True)
    eng = Engine(flags=_lib.NMG_F_DEFAULT | _lib.NMG_F_SAMPLE_MATCHES | _lib.NMG_F_OBJECT_LEVELS,
                 nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    eng.submit_replay(rp)
    eng.analyze()
    eng.synchronize()
    eng.report(edir, os.path.join(d, "e.txt"), dump_flags=_lib.NMG_DUMP_CALLSITES)
    eng.close()
    assert F.dump_rows(os.path.join(edir, "callsite_dump_1.dat")) == F.dump_rows(F.DUMP)
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "e.txt"), "rb").read()
    _same_dirs(odir, edir)
