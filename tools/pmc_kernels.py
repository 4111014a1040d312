#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 counter-collection CSVs (one directory per
--pmc pass): prints one JSON line per (kernel, counter) group, values per
dispatch, for the attribution and reduce kernels."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                agg[r["Kernel_Name"].split("(")[0][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        if not any(s in k for s in ("attribute", "reduce", "route_kernel", "route2_kernel", "local_kernel", "found_kernel")):
            continue
        print(json.dumps({"kernel": k, **{c: sum(x) / len(x) for c, x in sorted(v.items())},
                          "dispatches": max(len(x) for x in v.values())}))


if __name__ == "__main__":
    main()
