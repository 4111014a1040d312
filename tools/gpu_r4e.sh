set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r4}
timeout -k 10 600 bash tools/ab_lib.sh build_ab/lib_base.so build_ab/lib_pipe.so || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_route.py \
  > gpurun_out/pytest_route_$T.log 2>&1 || { tail -40 gpurun_out/pytest_route_$T.log; exit 1; }
tail -2 gpurun_out/pytest_route_$T.log
