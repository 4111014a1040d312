# one A/B session: route/parity tests on the in-tree lib, then bench A/B of the
# given libs and an SQ instruction-count pass of each
#   gpurun -- bash tools/gpu_ab.sh TAG [TESTS] -- build_ab/lib_a.so build_ab/lib_b.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
TESTS=""
while [ "$1" != "--" ] && [ -n "$1" ]; do TESTS="$TESTS $1"; shift; done
shift
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
bash tools/ab_lib.sh "$@" || exit 1
for lib in "$@"; do
  n=$(basename $lib .so)
  rm -rf gpurun_out/pmc_${TAG}_$n
  NMG_LIB_AB=1 NMG_LIB_PATH=$PWD/$lib timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $PWD/gpurun_out/pmc_${TAG}_$n -o run --output-format csv -- python3 $PWD/bench.py --workload c4 --secondary "" --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${TAG}_$n.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG}_$n.log; exit 1; }
  echo $n; python3 tools/pmc_kernels.py gpurun_out/pmc_${TAG}_$n | grep -v "dispatches\": 0"
done
