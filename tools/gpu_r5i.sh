set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_route.py tests/test_gpu_parity.py > gpurun_out/r5i_tests.log 2>&1 || { tail -30 gpurun_out/r5i_tests.log; exit 1; }
tail -3 gpurun_out/r5i_tests.log
for n in w8 cur; do
if [ $n = cur ]; then unset NMG_LIB_PATH; else export NMG_LIB_PATH=$PWD/build_ab/lib_$n.so; fi
timeout -k 10 300 python tools/local_timing.py --workloads c4 > gpurun_out/local_timing_r5i_$n.json 2> gpurun_out/local_timing_r5i_$n.err || { tail -20 gpurun_out/local_timing_r5i_$n.err; exit 1; }
echo $n; cat gpurun_out/local_timing_r5i_$n.json
done
unset NMG_LIB_PATH
timeout -k 10 300 python bench.py --workload c4 --secondary "" --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err || { tail -20 gpurun_out/r5i_bench.err; exit 1; }
cat gpurun_out/r5i_bench.json
