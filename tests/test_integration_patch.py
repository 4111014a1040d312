"""INTEGRATION.md section 1's reference-side patch, compiled and run as written.

tests/c/extract_patch.py cuts the patched mem_sampling.c and mem_analyzer.c
blocks out of INTEGRATION.md; each is compiled as its own translation unit
over tests/c/ref_stubs.h (the reference declarations restated) and linked with
tests/c/nmg_patch_host.c, which fills `mem_list` and `samples` from a replay
and calls the patched ma_finalize() (src/mem_analyzer.c:1802-1884).

* CPU: the blocks compile and link as written, and the binary the GPU test
  runs was built from the document as it stands.
* GPU: the process's whole stdout and every report file equal the oracle's,
  and the MEM ANALYZER banner appears once, after `bytes processed`
  (mem_sampling.c:343-344, then mem_analyzer.c:1809-1811)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "tests", "c")
PKG = os.path.join(ROOT, "numamma_amd")
sys.path.insert(0, CDIR)
import extract_patch  # noqa: E402

BANNER = b"---------------------------------\n         MEM ANALYZER\n---------------------------------\n"


def _blocks():
    return extract_patch.extract(open(os.path.join(ROOT, "INTEGRATION.md")).read())


def test_patch_blocks_compile_and_link(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("gcc")
    d = str(tmp_path)
    subprocess.run([sys.executable, os.path.join(CDIR, "extract_patch.py"), os.path.join(ROOT, "INTEGRATION.md"), d],
                   check=True)
    objs = []
    for name in ("patch_mem_sampling.c", "patch_mem_analyzer.c", "nmg_patch_host.c"):
        src = os.path.join(d if name.startswith("patch_") else CDIR, name)
        obj = os.path.join(d, name + ".o")
        subprocess.run(["gcc", "-std=gnu99", "-O2", "-Wall", "-Werror", "-c", "-I", os.path.join(ROOT, "include"),
                        "-I", CDIR, src, "-o", obj], check=True)
        objs.append(obj)
    lib = os.path.join(PKG, "libnumamma_gpu.so")
    if not os.path.exists(lib):
        pytest.skip("libnumamma_gpu.so not built")
    subprocess.run(["gcc", "-o", os.path.join(d, "host"), *objs, "-L", PKG, "-lnumamma_gpu"], check=True)


def test_patch_prints_no_banner_of_its_own():
    # nmg_report prints the banner (numamma_amd/csrc/nmg_report.cpp); the patched
    # ma_finalize must not print it a second time
    analyzer = _blocks()["patch_mem_analyzer.c"]
    assert "MEM ANALYZER" not in analyzer.replace("MEM ANALYZER banner", "")
    assert "nmg_report(gpu" in analyzer


def test_built_patch_matches_document():
    built = os.path.join(PKG, "build", "patch")
    if not os.path.isdir(built):
        pytest.skip("numamma_amd not built")
    for name, body in _blocks().items():
        text = open(os.path.join(built, name)).read()
        assert text.endswith(body), f"{name} is stale: rebuild numamma_amd (make)"


@pytest.mark.gpu
@pytest.mark.parametrize("nb_intervals", [600, 25_000])
def test_patch_whole_stdout_bit_exact(tmp_path, nb_intervals):
    import pyoracle
    from numamma_amd.replay import SynthConfig, generate

    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=120_000, nb_intervals=nb_intervals, lost_frac=1e-3, wrap_one=True,
                              seed=91 + nb_intervals))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"))
    edir = os.path.join(d, "e")
    os.makedirs(edir)
    env = dict(os.environ)
    pre = [x for x in env.get("LD_PRELOAD", "").split(":") if x and "libnumamma" not in os.path.basename(x)]
    if pre:
        env["LD_PRELOAD"] = ":".join(pre)
    else:
        env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(PKG, "bin", "nmg_patch_host"), path, edir], env=env, capture_output=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")
    out = r.stdout
    assert out.count(BANNER) == 1
    assert out.index(BANNER) > out.index(b" bytes processed\n")
    assert out == open(os.path.join(d, "o.txt"), "rb").read()
    fa, fb = sorted(os.listdir(os.path.join(d, "o"))), sorted(os.listdir(edir))
    assert fa == fb and fa
    for f in fa:
        assert open(os.path.join(d, "o", f), "rb").read() == open(os.path.join(edir, f), "rb").read(), f
