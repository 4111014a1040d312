#!/usr/bin/env python3
"""A/B timing of alternative builds of the engine (numamma_amd/build/variants,
`make -C numamma_amd variants VARIANTS="a:-DX,b:-DY"`): each variant runs in its
own process (the C-ABI library is loaded once per process), rounds interleaved.

    python tools/ab.py --variants base,a,b --workloads c2,k1m --rounds 2
Prints one JSON line per (workload, variant, round): median kernel ms."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys, time
import numpy as np
sys.path.insert(0, sys.argv[1])
import torch
from numamma_amd.engine import Engine
from numamma_amd.replay import SynthConfig, generate
W = {"c2": dict(nb_samples=10_000_000, nb_intervals=1_000),
     "k100k": dict(nb_samples=10_000_000, nb_intervals=100_000),
     "k1m": dict(nb_samples=10_000_000, nb_intervals=1_000_000, size_max=64 * 1024),
     "c3": dict(nb_samples=100_000_000, nb_intervals=100_000),
     "c4": dict(nb_samples=125_000_000, nb_intervals=1_000_000, size_max=64 * 1024)}
for w in sys.argv[3].split(","):
    rp = generate(SynthConfig(seed=1, **W[w]))
    arena, offs, lens, ranks, acc = rp.packed()
    d = torch.from_numpy(arena).cuda()
    e = Engine(nb_threads=rp.nb_threads)
    e.set_objects(rp.table)
    e.set_device_buffers(d.data_ptr(), offs, lens, ranks, acc)
    ts = []
    for r in range(int(sys.argv[4]) + 3):
        e.reset(); e.analyze(); e.synchronize()
        if r >= 3: ts.append(e.last_analyze_ms())
    print(json.dumps({"workload": w, "variant": sys.argv[2], "median_ms": float(np.median(ts)),
                      "min_ms": float(np.min(ts))}), flush=True)
    e.close()
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--workloads", default="c2")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    for rnd in range(a.rounds):
        for v in a.variants.split(","):
            env = dict(os.environ)
            env.pop("NMG_LIB_VARIANT", None)
            if v != "base":
                env["NMG_LIB_VARIANT"] = v
            out = subprocess.run([sys.executable, "-c", CHILD, ROOT, v, a.workloads, str(a.reps)],
                                 env=env, capture_output=True, text=True, timeout=600)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(out.returncode)
            for line in out.stdout.splitlines():
                rec = json.loads(line)
                rec["round"] = rnd
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
