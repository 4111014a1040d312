"""The PMC staleness guard (numamma_amd/srchash.py): any change to a source
under numamma_amd/csrc/ -- partition building and chunk-pool sizing included
(nmg_table.hip, nmg_route_host.hip), not only the kernel files -- or to the
Makefile's HIP flags changes the hash, and bench.py then drops the stamped
traffic of profiles/pmc_<workload>.json."""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from numamma_amd import srchash  # noqa: E402


def _copy_tree(tmp_path, monkeypatch):
    pkg = tmp_path / "numamma_amd"
    shutil.copytree(srchash.CSRC, pkg / "csrc")
    shutil.copy(srchash.MAKEFILE, pkg / "Makefile")
    monkeypatch.setattr(srchash, "CSRC", str(pkg / "csrc"))
    monkeypatch.setattr(srchash, "MAKEFILE", str(pkg / "Makefile"))
    return pkg


def test_hash_covers_every_csrc_file():
    names = srchash.kernel_sources()
    for must in ("nmg_table.hip", "nmg_route_host.hip", "nmg_submit.hip", "nmg_route.hip", "nmg_kernels.hip",
                 "nmg_engine_impl.h"):
        assert must in names
    assert "--offload-arch" in srchash.hip_flags()


def test_edit_to_partition_builder_changes_hash(tmp_path, monkeypatch):
    pkg = _copy_tree(tmp_path, monkeypatch)
    h0 = srchash.kernel_source_hash()
    assert h0 == srchash.kernel_source_hash()
    with open(pkg / "csrc" / "nmg_table.hip", "a") as f:
        f.write("\n// a change to build_partitions\n")
    h1 = srchash.kernel_source_hash()
    assert h1 != h0
    mk = (pkg / "Makefile").read_text()
    (pkg / "Makefile").write_text(mk.replace("HIPFLAGS := -O3", "HIPFLAGS := -O2"))
    assert srchash.kernel_source_hash() != h1


def test_bench_drops_stale_traffic(tmp_path, monkeypatch):
    import bench

    pkg = _copy_tree(tmp_path, monkeypatch)
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_c4.json").write_text(json.dumps({"source_hash": srchash.kernel_source_hash(),
                                                  "hbm_bytes_per_launch": 123, "kernels": {}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    traffic, pmc, _ = bench.load_traffic("c4")
    assert traffic == 123 and pmc is not None
    with open(pkg / "csrc" / "nmg_route_host.hip", "a") as f:
        f.write("\n// chunk-pool sizing changed\n")
    traffic, pmc, why = bench.load_traffic("c4")
    assert traffic is None and pmc is None and "not reported" in why
