#!/usr/bin/env python3
"""Per-kernel statistics of the c4 (main workload) dispatches of a
`rocprofv3 --kernel-trace` run of bench.py: the dispatches before the first
attribute_kernel of the c2 secondary line.

    tools/prof_c4_only.py gpurun_out/prof_<tag>/run_kernel_trace.csv > profiles/rN/kernel_stats_c4_only_<tag>.txt
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    stats = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if "attribute_kernel" in name:
            break
        short = name.split("(")[0].replace("void ", "")
        stats[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"# rocprofv3 --kernel-trace of `bench.py --steps 10 --warmup 2 --no-cpu-baseline` ({path}):")
    print("# the c4 dispatches only (before the first attribute_kernel of the c2 secondary line)")
    for k in sorted(stats):
        v = stats[k]
        print(f"{k:45s} n={len(v):3d} avg_us={sum(v) / len(v):9.1f} min={min(v):9.1f} max={max(v):9.1f}")


if __name__ == "__main__":
    main()
