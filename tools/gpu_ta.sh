# TA / TD / TCP busy counters of the bench's kernels (one pass each):
#   gpurun -- bash tools/gpu_ta.sh TAG [lib.so]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; LIB=${2:-}
[ -n "$LIB" ] && export NMG_LIB_PATH=$PWD/$LIB NMG_LIB_AB=1
i=0
for set in "TA_TA_BUSY_sum TA_BUFFER_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE" "TA_BUFFER_TOTAL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf gpurun_out/ta_${TAG}_$i
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace -d $PWD/gpurun_out/ta_${TAG}_$i -o run --output-format csv -- python3 $PWD/bench.py --workload c4 --secondary "" --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ta_${TAG}_$i.log 2>&1 || { tail -20 gpurun_out/ta_${TAG}_$i.log; exit 1; }
  python3 tools/pmc_kernels.py gpurun_out/ta_${TAG}_$i | grep -v "dispatches\": 0" | grep "route2\|local_kernel"
done
