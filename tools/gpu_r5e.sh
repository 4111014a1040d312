set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/route_timing.py --workloads c4 --reps 2 > gpurun_out/route_timing_r5e.json 2> gpurun_out/route_timing_r5e.err || { tail -20 gpurun_out/route_timing_r5e.err; exit 1; }
cat gpurun_out/route_timing_r5e.json
bash tools/ab_lib.sh build_ab/lib_r3.so build_ab/lib_u3.so || exit 1
rm -rf gpurun_out/pmcsq_r5e
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT --kernel-trace -d $PWD/gpurun_out/pmcsq_r5e -o run --output-format csv -- python3 $PWD/bench.py --workload c4 --secondary "" --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcsq_r5e.log 2>&1 || { tail -20 gpurun_out/pmcsq_r5e.log; exit 1; }
python3 tools/pmc_kernels.py gpurun_out/pmcsq_r5e
