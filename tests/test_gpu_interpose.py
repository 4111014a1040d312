"""The engine inside an LD_PRELOAD'ed process, on
the GPU: bin/nmg_c99_host runs INTEGRATION.md section 1's sequence with
tests/c/nmg_interpose.c preloaded -- every malloc/new of the HIP runtime, the
engine, its copy pool and the report's writer threads goes through a 64-byte
header + canary block, safe allocations are recorded (mutex + backtrace) and
every pthread_create is trampolined through a per-thread init, as under
NumaMMa's libnumamma.so (src/mem_intercept.c:75-130, 246-299, 325-387).

* protected: the host raises the interposer's thread-local recursion
  counter around every engine call (is_recurse_unsafe, numamma.h.in:60-74):
  the calling thread's allocations are not recorded, the runtime's own
  threads' are;
* unprotected: everything recorded;
* bridge: the out-of-process fallback (capture bridge under the interposer,
  helper nmg_replay without it, mem_intercept.c:472-502).

Each is byte-identical to the oracle's report with the interposer's canary
check on (NumaMMa's --canary-check).  NumaMMa's default is canary_check = 0
(numamma.h.in:41): CANARY_OK is then always true (mem_intercept.h:68) and
free() reads a header in front of every pointer (mem_intercept.c:266-298).
The HIP runtime frees hundreds of thousands of blocks it got from memalign &
co, which the interposer does not wrap, so the engine cannot run inside the
traced process under that default: test_in_process_needs_canary_check
records that, and test_bridge_without_canary_check runs the helper path --
the wiring INTEGRATION.md section 2 makes the default -- under it."""
import os
import subprocess

import pytest

import pyoracle
from numamma_amd.replay import SynthConfig, generate
from test_interpose_host import BIN, interposed_env, interposer_stats

pytestmark = pytest.mark.gpu


def _compare(d, a, b):
    assert open(os.path.join(d, a + ".txt"), "rb").read() == open(os.path.join(d, b + ".txt"), "rb").read()
    fa, fb = sorted(os.listdir(os.path.join(d, a))), sorted(os.listdir(os.path.join(d, b)))
    assert fa == fb and fa
    for f in fa:
        assert open(os.path.join(d, a, f), "rb").read() == open(os.path.join(d, b, f), "rb").read(), f


@pytest.mark.parametrize("mode", ["protected", "unprotected", "bridge"])
def test_engine_under_interposer(tmp_path, mode):
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=150_000, nb_intervals=3_000, lost_frac=1e-3, wrap_one=True, seed=83))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"))
    args = [os.path.join(BIN, "nmg_c99_host")] + (["--bridge"] if mode == "bridge" else [])
    extra = {"protected": {"NMG_HOST_PROTECT": "1"}, "unprotected": {},
             "bridge": {"NMG_BRIDGE_HELPER": os.path.join(BIN, "nmg_replay")}}[mode]
    r = subprocess.run(args + [path, os.path.join(d, "e"), os.path.join(d, "e.txt")],
                       env=interposed_env(**extra), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    st = interposer_stats(r.stderr)
    print(mode, st)
    assert st["recorded"] > 0
    if mode != "bridge":
        assert st["threads"] > 0  # HIP runtime / copy pool / report writer threads went through the hook
    if mode == "protected":
        assert st["unsafe_skips"] > 0
    _compare(d, "o", "e")


def _run(d, args, **extra):
    return subprocess.run(args, env=interposed_env(**extra), capture_output=True, text=True, timeout=180)


def _replay(d, seed):
    rp = generate(SynthConfig(nb_samples=150_000, nb_intervals=3_000, lost_frac=1e-3, wrap_one=True, seed=seed))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"))
    return path


def test_bridge_without_canary_check(tmp_path):
    """NumaMMa's default canary_check = 0: the capture bridge (no HIP in the
    traced process) frees nothing foreign, and the helper's report is the
    oracle's."""
    d = str(tmp_path)
    path = _replay(d, 84)
    r = _run(d, [os.path.join(BIN, "nmg_c99_host"), "--bridge", path, os.path.join(d, "e"), os.path.join(d, "e.txt")],
             NMG_BRIDGE_HELPER=os.path.join(BIN, "nmg_replay"), NMG_INTERPOSE_CANARY_CHECK="0")
    assert r.returncode == 0, r.stderr[-3000:]
    st = interposer_stats(r.stderr)
    assert st["recorded"] > 0 and st["foreign_frees"] == 0
    _compare(d, "o", "e")


FOREIGN_EXIT = 86  # NMG_INTERPOSE_FOREIGN_EXIT (tests/c/nmg_interpose.c)


def test_in_process_needs_canary_check(tmp_path):
    """The engine in-process under canary_check = 0: the HIP runtime frees a
    block the interposer did not allocate, whose header NumaMMa would trust
    (the outcome INTEGRATION.md section 2 states: in-process only with
    --canary-check).  The test interposer stops at that free, before libc
    sees the bogus pointer, with its own exit code and counters: any other
    failure (a missing binary, a HIP init error) fails this test."""
    d = str(tmp_path)
    path = _replay(d, 85)
    r = _run(d, [os.path.join(BIN, "nmg_c99_host"), path, os.path.join(d, "e"), os.path.join(d, "e.txt")],
             NMG_HOST_PROTECT="1", NMG_INTERPOSE_CANARY_CHECK="0")
    print("returncode", r.returncode, r.stderr[-500:])
    assert r.returncode == FOREIGN_EXIT, r.stderr[-3000:]
    assert "foreign block" in r.stderr
    st = interposer_stats(r.stderr)
    assert st["foreign_frees"] >= 1
