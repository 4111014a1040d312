#!/usr/bin/env python3
"""End-to-end rate of the drop-in path with host-resident buffers, as the
reference's C host would drive it: buffers start in pageable
host memory (the malloc'd __copy_buffer copies, mem_sampling.c:696),
nmg_submit_buffer stages them into pinned memory, nmg_analyze uploads with
hipMemcpyAsync and runs the kernel, and the results come back D2H
(nmg_get_global_counters + object counters + page cells).  Prints one JSON
line per phase split, next to the device-resident kernel time."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from numamma_amd.engine import Engine
    from numamma_amd.replay import CONFIGS, generate

    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    rp = generate(CONFIGS[wl])
    lins = rp.linear_buffers()
    nbytes = sum(x[2].shape[0] for x in lins)
    nsamples = nbytes // 40
    eng = Engine(nb_threads=rp.nb_threads)
    eng.set_objects(rp.table)
    reps = []
    for r in range(4):
        eng.clear_buffers()
        eng.reset()
        eng.synchronize()
        t0 = time.perf_counter()
        for rank, acc, data in lins:  # host copy into pinned staging
            eng.submit_buffer(data, rank, acc)
        t1 = time.perf_counter()
        eng.analyze()  # H2D + kernel
        eng.synchronize()
        t2 = time.perf_counter()
        eng.global_counters()
        eng.object_counters()
        eng.page_cells()  # D2H of everything the report reads
        t3 = time.perf_counter()
        reps.append((t1 - t0, t2 - t1, t3 - t2, eng.last_analyze_ms() / 1e3))
    st, up, dn, kern = np.median(np.array(reps[1:]), axis=0)
    total = st + up + dn
    print(json.dumps({
        "workload": wl, "records": int(nsamples), "bytes": int(nbytes),
        "stage_host_s": st, "h2d_plus_kernel_s": up, "d2h_results_s": dn, "kernel_s": kern,
        "e2e_samples_per_s": nsamples / total,
        "e2e_excl_staging_samples_per_s": nsamples / (up + dn),
        "h2d_GBps_est": nbytes / max(up - kern, 1e-9) / 1e9,
        "device_resident_samples_per_s": nsamples / kern,
    }), flush=True)


if __name__ == "__main__":
    main()
