#!/bin/bash
# Counter passes over engine variants (tools/pmc_variants.py); one rocprofv3
# run per counter set, each under its own time limit.
#   gpurun -- bash tools/pmc_variants.sh TAG WORKLOAD VARIANTS "SET1;SET2;..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=$1; WL=$2; VARS=$3; SETS=$4; REPS=${REPS:-2}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; ROOT=$PWD
IFS=';' read -ra SS <<< "$SETS"
i=0; dirs=""
for s in "${SS[@]}"; do
  i=$((i+1)); d=$OUT/pmcv_${TAG}_$i; rm -rf $d
  timeout -s KILL 300 rocprofv3 --pmc $s --kernel-trace -d $ROOT/$d -o run --output-format csv \
    -- python3 $ROOT/tools/pmc_variants.py run --workload $WL --variants $VARS --reps $REPS > $d.log 2>&1 \
    || { echo "pass $i failed"; tail -20 $d.log; exit 1; }
  dirs="$dirs $d"
done
for K in ${KERNELS:-attribute_kernel}; do
  python3 tools/pmc_variants.py parse $dirs --variants $VARS --reps $REPS --kernel $K | sed "s/^{/{\"k\": \"$K\", /"
done | tee $OUT/pmcv_$TAG.jsonl
