"""The LD_PRELOAD hazards of INTEGRATION.md section 2, on the CPU:
tests/c/nmg_interpose.c (header-wrapped malloc/free/new, dlsym bootstrap
arena, recorded allocations with backtraces, pthread_create trampoline --
the shape of src/mem_intercept.c:75-130, 246-299, 325-387) preloaded into
bin/nmg_c99_host running the capture bridge (--bridge).  The helper here is
`cp` (the GPU helper runs in tests/test_gpu_interpose.py): the replay the
bridge wrote under the interposer must give the oracle's report byte for
byte, and the child must have run without the interposer."""
import json
import os
import subprocess

import pytest

import pyoracle
from numamma_amd.replay import SynthConfig, generate

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "numamma_amd", "bin")
# (NMG_INTERPOSER: the UBSan build of the interposer, tools/sanitize.sh)
INTERPOSER = os.environ.get("NMG_INTERPOSER") or os.path.join(BIN, "libnmg_interpose.so")


def interposed_env(**extra):
    env = dict(os.environ)
    pre = env.get("LD_PRELOAD", "")
    env["LD_PRELOAD"] = INTERPOSER + (":" + pre if pre else "")
    env["NMG_BRIDGE_PRELOAD"] = pre  # the value without the interposer (unset_ld_preload)
    env.update(extra)
    return env


def interposer_stats(stderr: str):
    lines = [x for x in stderr.splitlines() if x.startswith("nmg_interpose: ")]
    assert lines, stderr[-2000:]
    return json.loads(lines[-1][len("nmg_interpose: "):])


@pytest.mark.parametrize("canary_check", ["1", "0"])
def test_capture_bridge_under_interposer(tmp_path, canary_check):
    """canary_check "0" is NumaMMa's default (numamma.h.in:41): free() trusts
    every pointer's header (mem_intercept.h:68), so the process must free
    nothing it did not allocate through the wrapped malloc -- the capture
    bridge frees none."""
    d = str(tmp_path)
    rp = generate(SynthConfig(nb_samples=60_000, nb_intervals=800, lost_frac=1e-3, wrap_one=True, seed=81))
    path = os.path.join(d, "replay.bin")
    rp.write(path)
    copy = os.path.join(d, "copied.bin")
    # helper = cp: `cp <bridge replay> <copy>`; it must not see the interposer
    helper = os.path.join(d, "helper.sh")
    with open(helper, "w") as f:
        f.write("#!/bin/sh\ncase \"$LD_PRELOAD\" in *libnmg_interpose*) exit 3;; esac\ncp \"$1\" \"$2\"\n")
    os.chmod(helper, 0o755)
    r = subprocess.run([os.path.join(BIN, "nmg_c99_host"), "--bridge", path, copy, os.path.join(d, "h.txt")],
                       env=interposed_env(NMG_BRIDGE_HELPER=helper, NMG_INTERPOSE_CANARY_CHECK=canary_check),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    st = interposer_stats(r.stderr)
    assert st["recorded"] > 0 and st["hand_made"] >= 0
    assert st["foreign_frees"] == 0
    pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"))
    pyoracle.run(copy, os.path.join(d, "c"), os.path.join(d, "c.txt"))
    assert open(os.path.join(d, "o.txt"), "rb").read() == open(os.path.join(d, "c.txt"), "rb").read()
    for f in sorted(os.listdir(os.path.join(d, "o"))):
        assert open(os.path.join(d, "o", f), "rb").read() == open(os.path.join(d, "c", f), "rb").read(), f


def test_interposer_survives_threads_and_python():
    """The interposer itself: a threaded numpy program runs under it (header
    blocks through malloc/realloc/free, trampolined threads)."""
    code = ("import threading, numpy as np\n"
            "def f():\n  a = [np.arange(i + 1000).tobytes() for i in range(200)]\n"
            "ts = [threading.Thread(target=f) for _ in range(6)]\n"
            "[t.start() for t in ts]; [t.join() for t in ts]; print('ok')\n")
    r = subprocess.run(["python3", "-c", code], env=interposed_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]
    st = interposer_stats(r.stderr)
    assert st["threads"] >= 6 and st["recorded"] > 1000 and st["freed"] > 0
