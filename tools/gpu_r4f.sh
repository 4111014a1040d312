set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r4}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_route.py \
  > gpurun_out/pytest_route_$T.log 2>&1 || { tail -40 gpurun_out/pytest_route_$T.log; exit 1; }
tail -2 gpurun_out/pytest_route_$T.log
timeout -k 10 300 python -u tools/route_timing.py --workloads c4 --flags 0x3 > gpurun_out/route_timing_$T.json 2> gpurun_out/route_timing_$T.err || { tail -20 gpurun_out/route_timing_$T.err; exit 1; }
cat gpurun_out/route_timing_$T.json
timeout -k 10 400 python -u tools/ablate.py --workloads c4 --reps 8 --variants route,route_v1 > gpurun_out/ablate_$T.json 2> gpurun_out/ablate_$T.err || { tail -20 gpurun_out/ablate_$T.err; exit 1; }
cat gpurun_out/ablate_$T.json
