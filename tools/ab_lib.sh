#!/bin/bash
# A/B of two builds of libnumamma_gpu.so on one box (NMG_LIB_PATH):
#   gpurun -- bash tools/ab_lib.sh build_ab/lib_a.so build_ab/lib_b.so[:FLAGS] [more.so ...]
# (:FLAGS: NMG_BENCH_DEBUG_FLAGS for that run, e.g. lib.so:0x20000000 for route_kernel)
# Alternates the libraries twice over bench.py's line (AB_WL, default c4) and
# prints the analysis time split (route / rest) of each run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
WL=${AB_WL:-c4}
mkdir -p gpurun_out
for rep in 1 2; do
  for arg in "$@"; do
    lib=${arg%%:*}; fl=${arg#*:}; [ "$fl" = "$arg" ] && fl=${NMG_BENCH_DEBUG_FLAGS:-0}
    tag=$(basename "$lib" .so); [ "$fl" != "0" ] && tag=${tag}_$fl; tag=${tag}_$rep
    NMG_BENCH_DEBUG_FLAGS=$fl NMG_LIB_AB=1 NMG_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --workload "$WL" --secondary "" --no-cpu-baseline \
      > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/ab_$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$tag.json')); k=d['roofline']['kernels']; print('$tag', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', {n: round(v['avg_ms'],3) for n,v in k.items()})"
  done
done
