set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r4}
# 1. partition-first parity (route v1 and v2, tiny pools, escapes) + the merge tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_route.py tests/test_gpu_distributed.py > gpurun_out/pytest_route_$T.log 2>&1 || { tail -40 gpurun_out/pytest_route_$T.log; exit 1; }
tail -2 gpurun_out/pytest_route_$T.log
# 2. route variants at the c4 shard, and v2's phase cycles
timeout -k 10 400 python -u tools/ablate.py --workloads c4 --reps 8 --variants ${VARIANTS:-route,route_v1,route_atomics} > gpurun_out/ablate_$T.json 2> gpurun_out/ablate_$T.err || { tail -20 gpurun_out/ablate_$T.err; exit 1; }
cat gpurun_out/ablate_$T.json
timeout -k 10 300 python -u tools/route_timing.py --workloads c4 --flags ${TFLAGS:-0x3} > gpurun_out/route_timing_v2_$T.json 2> gpurun_out/route_timing_v2_$T.err || { tail -20 gpurun_out/route_timing_v2_$T.err; exit 1; }
cat gpurun_out/route_timing_v2_$T.json
# 3. the rest of the GPU suite (FULL=1)
if [ "${FULL:-0}" = "1" ]; then
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider tests -m gpu --ignore=tests/test_gpu_route.py --ignore=tests/test_gpu_distributed.py > gpurun_out/pytest_gpu_$T.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$T.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$T.log
fi
