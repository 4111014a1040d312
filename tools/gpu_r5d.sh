set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in r1 r3 p2; do
NMG_LIB_PATH=$PWD/build_ab/lib_$n.so timeout -k 10 300 python tools/route_timing.py --workloads c4 --reps 2 > gpurun_out/route_timing_r5d_$n.json 2> gpurun_out/route_timing_r5d_$n.err || { tail -20 gpurun_out/route_timing_r5d_$n.err; exit 1; }
echo $n; cat gpurun_out/route_timing_r5d_$n.json
done
bash tools/ab_lib.sh build_ab/lib_r1.so build_ab/lib_r2.so build_ab/lib_r3.so build_ab/lib_p1.so build_ab/lib_p2.so
