set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_route.py > gpurun_out/pytest_r5f.log 2>&1 || { tail -40 gpurun_out/pytest_r5f.log; exit 1; }
tail -2 gpurun_out/pytest_r5f.log
NMG_LIB_PATH=$PWD/build_ab/lib_w8.so timeout -k 10 300 python tools/route_timing.py --workloads c4 --reps 2 > gpurun_out/route_timing_r5f.json 2> gpurun_out/route_timing_r5f.err || { tail -20 gpurun_out/route_timing_r5f.err; exit 1; }
cat gpurun_out/route_timing_r5f.json
bash tools/ab_lib.sh build_ab/lib_u3.so build_ab/lib_w8.so
