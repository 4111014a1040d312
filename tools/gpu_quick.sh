set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_route.py tests/test_gpu_parity.py -k "route or short_sample or lookup or large_weights or two_shard" > gpurun_out/pytest_r3v.log 2>&1 || { tail -40 gpurun_out/pytest_r3v.log; exit 1; }
tail -3 gpurun_out/pytest_r3v.log
timeout -k 10 300 python bench.py --secondary "" --no-cpu-baseline > gpurun_out/bench_r3v.json 2> gpurun_out/bench_r3v.err || { tail -20 gpurun_out/bench_r3v.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r3v.json')); print(d['value']/1e9, d['ms_per_step'], d['roofline']['kernels'])"
timeout -k 10 300 python tools/route_timing.py > gpurun_out/route_timing_r3v.json 2> gpurun_out/route_timing_r3v.err || { tail -20 gpurun_out/route_timing_r3v.err; exit 1; }
cat gpurun_out/route_timing_r3v.json
