set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" gpurun_out/rocprof_counters.txt | sort -u > gpurun_out/sq_counters.txt || true
wc -l gpurun_out/sq_counters.txt
rm -rf gpurun_out/pmcsq_r5l
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace -d $PWD/gpurun_out/pmcsq_r5l -o run --output-format csv -- python3 $PWD/bench.py --workload c4 --secondary "" --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcsq_r5l.log 2>&1 || { tail -20 gpurun_out/pmcsq_r5l.log; exit 1; }
python3 tools/pmc_kernels.py gpurun_out/pmcsq_r5l
