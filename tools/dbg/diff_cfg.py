"""Debug helper: run one synthetic config through the oracle and the engine
and print which raw-result fields differ."""
import os, sys, tempfile
import numpy as np
import torch
torch.zeros(1).cuda()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import pyoracle
from numamma_amd.engine import run_replay
from numamma_amd.replay import SynthConfig, generate
from numamma_amd.results import RawResults

cfg = SynthConfig(nb_samples=30_000, nb_intervals=1, nb_globals=0, with_stack=False, buffer_records=10_000, seed=5)
d = tempfile.mkdtemp()
rp = generate(cfg)
path = os.path.join(d, "r.bin"); rp.write(path)
pyoracle.run(path, os.path.join(d, "o"), os.path.join(d, "o.txt"), os.path.join(d, "o_raw.bin"))
run_replay(path, os.path.join(d, "e"), os.path.join(d, "e.txt"), os.path.join(d, "e_raw.bin"))
a, b = RawResults.read(os.path.join(d, "o_raw.bin")), RawResults.read(os.path.join(d, "e_raw.bin"))
g1, g2 = a.global_counters, b.global_counters
for acc in range(2):
    for i in np.nonzero(g1[acc] != g2[acc])[0]:
        print("global", acc, i, int(g1[acc, i]), int(g2[acc, i]))
print("samples", a.nb_samples, b.nb_samples, "found", a.nb_found, b.nb_found)
print("entries equal", np.array_equal(a.entries, b.entries), "cells equal", np.array_equal(a.cells, b.cells))
print("bufs", a.buf_samples.tolist(), b.buf_samples.tolist())

# windows per workgroup (timing variant, flag 0x1000)
import ctypes as C
import torch
from numamma_amd._lib import lib
from numamma_amd.engine import Engine
lib.nmg_debug_timing.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_size_t)]
arena, offs, lens, ranks, acc = rp.packed()
dd = torch.from_numpy(arena).cuda()
for fl in (0x3 | 0x1000,):
    e = Engine(flags=fl, nb_threads=rp.nb_threads)
    e.set_objects(rp.table)
    e.set_device_buffers(dd.data_ptr(), offs, lens, ranks, acc)
    e.reset(); e.analyze(); e.synchronize()
    n = C.c_size_t(0)
    lib.nmg_debug_timing(e.h, None, 0, C.byref(n))
    buf = np.zeros(n.value, dtype=np.uint64)
    lib.nmg_debug_timing(e.h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), n.value, C.byref(n))
    t = buf.reshape(-1, 16, 24)
    for w in (11, 12, 13):
        for k in range(4):
            a, b = int(t[w, 0, 8 + 2 * k]), int(t[w, 0, 9 + 2 * k])
            print("WG", w, "win", k, "idx", a >> 40, "cur", a & 0xFFFFFFFFFF, "n0", b & 0x7FF, "n1", (b >> 11) & 0x7FF,
                  "f", (b >> 22) & 3, "nidx", (b >> 24) & 0xFF, "ncur", b >> 32)
    print("windows per WG", t[:, 0, 5].tolist())
    s, f = e.buffer_counts()
    print("timing-variant bufs", s.tolist())
