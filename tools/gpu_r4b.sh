set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r4}
export NMG_BENCH_DEBUG_FLAGS=${ABFLAGS:-0x20000000}
timeout -k 10 900 bash tools/ab_lib.sh build_ab/lib_base.so build_ab/lib_dir2k.so || exit 1
unset NMG_BENCH_DEBUG_FLAGS
timeout -k 10 300 python -u tools/local_timing.py --workloads c4 --flags 0x20000003 > gpurun_out/local_timing_$T.json 2> gpurun_out/local_timing_$T.err || { tail -20 gpurun_out/local_timing_$T.err; exit 1; }
cat gpurun_out/local_timing_$T.json
timeout -k 10 400 python -u tools/ablate.py --workloads c4 --reps 6 --variants route,route_noloc,local_noobj,local_nopage,local_nosearch > gpurun_out/ablate_local_$T.json 2> gpurun_out/ablate_local_$T.err || { tail -20 gpurun_out/ablate_local_$T.err; exit 1; }
cat gpurun_out/ablate_local_$T.json
