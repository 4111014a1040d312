"""The boundary from outside Python, on the GPU.

* tests/c/nmg_c99_host.c (built as numamma_amd/bin/nmg_c99_host): a C99
  program that includes include/numamma_gpu.h and runs INTEGRATION.md
  section 1's sequence -- nmg_create, nmg_set_objects, nmg_submit_ring for
  every buffer (a wrapped ring and LOST records included), nmg_analyze,
  nmg_synchronize, nmg_report, nmg_destroy;
* numamma_amd/bin/nmg_replay as a child process, the out-of-process helper
  of INTEGRATION.md section 2 (system("nmg_replay ...") after
  unset_ld_preload, src/mem_intercept.c:472-502).  The child's environment
  drops NumaMMa's interposer from LD_PRELOAD like unset_ld_preload does;
  other preloaded libraries of the test environment stay in place.

Both outputs are compared byte for byte with the oracle's."""
import os
import subprocess

import pytest

import pyoracle
from numamma_amd.replay import SynthConfig, generate

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "numamma_amd", "bin")


def _child_env():
    env = dict(os.environ)
    pre = [x for x in env.get("LD_PRELOAD", "").split(":") if x and "libnumamma" not in os.path.basename(x)]
    if pre:
        env["LD_PRELOAD"] = ":".join(pre)
    else:
        env.pop("LD_PRELOAD", None)
    return env


def _compare(d, odir, ostdout, edir, estdout):
    assert open(ostdout, "rb").read() == open(estdout, "rb").read()
    fa, fb = sorted(os.listdir(odir)), sorted(os.listdir(edir))
    assert fa == fb and fa
    for f in fa:
        assert open(os.path.join(odir, f), "rb").read() == open(os.path.join(edir, f), "rb").read(), f


@pytest.mark.parametrize("nb_intervals", [700, 30_000])
def test_c99_host_bit_exact(tmp_path, nb_intervals):
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=150_000, nb_intervals=nb_intervals, lost_frac=1e-3, wrap_one=True,
                              seed=71 + nb_intervals))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"))
    r = subprocess.run([os.path.join(BIN, "nmg_c99_host"), path, os.path.join(d, "e"), os.path.join(d, "e.txt")],
                       env=_child_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    _compare(d, os.path.join(d, "o"), os.path.join(d, "o.txt"), os.path.join(d, "e"), os.path.join(d, "e.txt"))


def test_replay_helper_child_process(tmp_path):
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=120_000, nb_intervals=2_000, lost_frac=1e-3, wrap_one=True, seed=73))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"))
    edir = os.path.join(d, "e")
    r = subprocess.run([os.path.join(BIN, "nmg_replay"), path, edir], env=_child_env(), capture_output=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")
    with open(os.path.join(d, "e.txt"), "wb") as f:
        f.write(r.stdout)
    _compare(d, os.path.join(d, "o"), os.path.join(d, "o.txt"), edir, os.path.join(d, "e.txt"))
