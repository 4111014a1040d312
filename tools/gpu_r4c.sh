set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r4}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_route.py \
  tests/test_gpu_online.py -k "route_bit_exact or failed_growth or partial_update" > gpurun_out/pytest_c_$T.log 2>&1 || { tail -40 gpurun_out/pytest_c_$T.log; exit 1; }
tail -2 gpurun_out/pytest_c_$T.log
timeout -k 10 400 python -u tools/ablate.py --workloads c4 --reps 8 --variants ${VARIANTS:-route,route_v2} > gpurun_out/ablate_$T.json 2> gpurun_out/ablate_$T.err || { tail -20 gpurun_out/ablate_$T.err; exit 1; }
cat gpurun_out/ablate_$T.json
timeout -k 10 300 python -u tools/route_timing.py --workloads c4 --flags 0x20000003 > gpurun_out/route_timing_v2_$T.json 2> gpurun_out/route_timing_v2_$T.err || { tail -20 gpurun_out/route_timing_v2_$T.err; exit 1; }
cat gpurun_out/route_timing_v2_$T.json
if [ "${SQ:-1}" = "1" ]; then
KERNELS="route_kernel route2_kernel local_kernel" REPS=2 timeout -k 10 700 bash tools/pmc_variants.sh sq_$T c4 route,route_v2 \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
fi
