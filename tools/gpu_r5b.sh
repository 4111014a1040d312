set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/route_timing.py --workloads c4 > gpurun_out/route_timing_r5b.json 2> gpurun_out/route_timing_r5b.err || { tail -20 gpurun_out/route_timing_r5b.err; exit 1; }
cat gpurun_out/route_timing_r5b.json
bash tools/ab_lib.sh build_ab/lib_s1.so build_ab/lib_s3.so build_ab/lib_s8.so
