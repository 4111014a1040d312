set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_route.py -k "route-case or lapnowait-case or accumulates" > gpurun_out/pytest_r5c.log 2>&1 || { tail -40 gpurun_out/pytest_r5c.log; exit 1; }
tail -2 gpurun_out/pytest_r5c.log
for n in 8 16; do
NMG_LIB_PATH=$PWD/build_ab/lib_r$n.so timeout -k 10 300 python tools/route_timing.py --workloads c4 > gpurun_out/route_timing_r5c_$n.json 2> gpurun_out/route_timing_r5c_$n.err || { tail -20 gpurun_out/route_timing_r5c_$n.err; exit 1; }
cat gpurun_out/route_timing_r5c_$n.json
done
bash tools/ab_lib.sh build_ab/lib_r3.so build_ab/lib_r8.so build_ab/lib_r16.so
