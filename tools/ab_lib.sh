#!/bin/bash
# A/B of two builds of libnumamma_gpu.so on one box (NMG_LIB_PATH):
#   gpurun -- bash tools/ab_lib.sh build_ab/lib_a.so build_ab/lib_b.so [workload]
# Alternates the two libraries twice over bench.py's c4 line and prints the
# analysis time split (route / rest) of each run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
A=$1; B=$2; WL=${3:-c4}
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$A" "$B"; do
    tag=$(basename "$lib" .so)_$rep
    NMG_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --workload "$WL" --secondary "" --no-cpu-baseline \
      > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/ab_$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$tag.json')); k=d['roofline']['kernels']; print('$tag', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', {n: round(v['avg_ms'],3) for n,v in k.items()})"
  done
done
