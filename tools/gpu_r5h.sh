set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in w8 d6t; do
NMG_LIB_PATH=$PWD/build_ab/lib_$n.so timeout -k 10 300 python tools/local_timing.py --workloads c4 > gpurun_out/local_timing_r5h_$n.json 2> gpurun_out/local_timing_r5h_$n.err || { tail -20 gpurun_out/local_timing_r5h_$n.err; exit 1; }
echo $n; cat gpurun_out/local_timing_r5h_$n.json
done
for n in w8 d6t; do
rm -rf gpurun_out/pmcsq_r5h_$n
NMG_LIB_PATH=$PWD/build_ab/lib_$n.so timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT --kernel-trace -d $PWD/gpurun_out/pmcsq_r5h_$n -o run --output-format csv -- python3 $PWD/bench.py --workload c4 --secondary "" --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcsq_r5h_$n.log 2>&1 || { tail -20 gpurun_out/pmcsq_r5h_$n.log; exit 1; }
echo $n; python3 tools/pmc_kernels.py gpurun_out/pmcsq_r5h_$n
done
