#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per dispatch of one kernel.

    python tools/pmc_summary.py gpurun_out/pmc_TAG_1 gpurun_out/pmc_TAG_2 ... [--kernel attribute_kernel]
        [--stream-bytes BYTES]

Prints one JSON object: counter -> mean value per dispatch (summed over the
dispatch's dimensions), plus derived figures when the inputs are present:
FETCH_SIZE / WRITE_SIZE are in KiB and gfx950 under-reports FETCH_SIZE by 2x
(MI355X_MICROARCH.md, HBM/rocprofv3 section), so hbm_read_bytes = 2 * 1024 *
FETCH_SIZE."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    kernel = "attribute_kernel"
    if "--kernel" in sys.argv:
        kernel = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != kernel]
    stream = None
    if "--stream-bytes" in sys.argv:
        sb = sys.argv[sys.argv.index("--stream-bytes") + 1]
        stream = float(sb)
        args = [a for a in args if a != sb]
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f, newline="") as fh:
                for row in csv.DictReader(fh):
                    if kernel not in row["Kernel_Name"]:
                        continue
                    key = (f, row["Dispatch_Id"])
                    vals[row["Counter_Name"]][key] += float(row["Counter_Value"])
    out = {}
    for c, per in sorted(vals.items()):
        out[c] = sum(per.values()) / len(per)
        out[c + "_dispatches"] = len(per)
    if "FETCH_SIZE" in out:
        # gfx950 tallies a wide coalesced streaming read at half its bytes
        # (MI355X_MICROARCH.md, HBM): with --stream-bytes S (the record stream
        # of one launch) only that part is corrected, the random table probes
        # are taken as counted; without it every byte is doubled (upper bound)
        if stream is not None:
            out["hbm_read_bytes"] = out["FETCH_SIZE"] * 1024 + stream / 2
            out["stream_bytes"] = stream
        else:
            out["hbm_read_bytes"] = out["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in out:
        out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    if "hbm_read_bytes" in out and "hbm_write_bytes" in out:  # bench.py roofline.traffic
        out["hbm_bytes_per_launch"] = out["hbm_read_bytes"] + out["hbm_write_bytes"]
    if "SQ_WAVES" in out and "SQ_INSTS_VALU" in out:
        out["valu_per_wave"] = out["SQ_INSTS_VALU"] / out["SQ_WAVES"]
        out["salu_per_wave"] = out["SQ_INSTS_SALU"] / out["SQ_WAVES"]
        out["lds_per_wave"] = out["SQ_INSTS_LDS"] / out["SQ_WAVES"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
