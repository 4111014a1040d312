#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; the first failure ends the call.
#   gpurun -- bash tools/gpu_round.sh [tag] [stages...]
#   stages: test bench prof smoke (default: test bench prof)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${1:-r1}
shift || true
STAGES=${*:-test bench prof}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$PWD

for s in $STAGES; do
  case $s in
    smoke)
      echo "== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 \
        || { echo "smoke failed"; tail -40 $OUT/smoke_$TAG.log; exit 1; }
      tail -3 $OUT/smoke_$TAG.log ;;
    test)
      echo "== pytest -m gpu"
      timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu_$TAG.log 2>&1 \
        || { echo "pytest failed"; tail -60 $OUT/pytest_gpu_$TAG.log; exit 1; }
      tail -5 $OUT/pytest_gpu_$TAG.log ;;
    bench)
      echo "== bench"
      timeout -k 10 900 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err \
        || { echo "bench failed"; tail -40 $OUT/bench_$TAG.err; exit 1; }
      cat $OUT/bench_$TAG.json ;;
    bench3)
      echo "== bench c3"
      timeout -k 10 900 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c3_$TAG.json 2> $OUT/bench_c3_$TAG.err \
        || { echo "bench c3 failed"; tail -40 $OUT/bench_c3_$TAG.err; exit 1; }
      cat $OUT/bench_c3_$TAG.json ;;
    prof)
      echo "== rocprofv3 kernel trace"
      rm -rf $OUT/prof_$TAG
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_$TAG -o run --output-format csv \
        -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 \
        || { echo "rocprof failed"; tail -40 $OUT/prof_$TAG.log; exit 1; }
      find $OUT/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \; | head -20 ;;
    ablate)
      echo "== ablation"
      timeout -k 10 900 python tools/ablate.py --workloads ${ABLATE_WL:-c2,k100k,k1m} ${ABLATE_VARIANTS:+--variants $ABLATE_VARIANTS} > $OUT/ablate_$TAG.json 2> $OUT/ablate_$TAG.err \
        || { echo "ablate failed"; tail -40 $OUT/ablate_$TAG.err; exit 1; }
      cat $OUT/ablate_$TAG.json ;;
    e2e)
      echo "== end-to-end (host buffers, PCIe)"
      timeout -k 10 600 python tools/e2e.py ${E2E_WL:-c2} --modes ${E2E_MODES:-per_buffer,batch,stream} --threads ${E2E_THREADS:-16} --chunk-mb ${E2E_CHUNK:-64} > $OUT/e2e_$TAG.json 2> $OUT/e2e_$TAG.err \
        || { echo "e2e failed"; tail -30 $OUT/e2e_$TAG.err; exit 1; }
      cat $OUT/e2e_$TAG.json ;;
    phases)
      echo "== phase timing"
      timeout -k 10 600 python tools/phase_timing.py --workloads ${PHASE_WL:-c2,k100k} > $OUT/phases_$TAG.json 2> $OUT/phases_$TAG.err \
        || { echo "phase timing failed"; tail -30 $OUT/phases_$TAG.err; exit 1; }
      cat $OUT/phases_$TAG.json ;;
    bench2g)
      echo "== bench, 2 ranks sharing GPU 0 over gloo (multi-rank code path)"
      timeout -k 10 600 env NMG_BENCH_BACKEND=gloo NMG_BENCH_SAME_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $OUT/bench2g_$TAG.json 2> $OUT/bench2g_$TAG.err \
        || { echo "bench2g failed"; tail -40 $OUT/bench2g_$TAG.err; exit 1; }
      cat $OUT/bench2g_$TAG.json ;;
    handle)
      # the one-process multi-GPU path on this box: one engine handle over 1 GPU, and 2
      # workers sharing GPU 0 (device merges): each line carries its merge split
      echo "== bench --handle (1 GPU; 2 workers on GPU 0)"
      timeout -k 10 600 python bench.py --handle --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_handle1_$TAG.json 2> $OUT/bench_handle1_$TAG.err \
        || { echo "bench handle1 failed"; tail -30 $OUT/bench_handle1_$TAG.err; exit 1; }
      cat $OUT/bench_handle1_$TAG.json
      timeout -k 10 600 env NMG_BENCH_SAME_GPU=1 python bench.py --handle --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_handle2_$TAG.json 2> $OUT/bench_handle2_$TAG.err \
        || { echo "bench handle2 failed"; tail -30 $OUT/bench_handle2_$TAG.err; exit 1; }
      cat $OUT/bench_handle2_$TAG.json ;;
    pmcsq)
      echo "== rocprofv3 -L + SQ counter passes"
      timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
      i=0
      for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
                 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
                 "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"; do
        i=$((i+1))
        rm -rf $OUT/pmc_${TAG}_$i
        timeout -k 10 400 rocprofv3 --pmc $set --kernel-trace -d $ROOT/$OUT/pmc_${TAG}_$i -o run --output-format csv \
          -- python3 $ROOT/bench.py --workload ${PMC_WL:-c2} --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_${TAG}_$i.log 2>&1 \
          || { echo "pmc pass $i failed"; tail -20 $OUT/pmc_${TAG}_$i.log; exit 1; }
      done
      echo "pmc passes done" ;;
    traffic)
      # HBM bytes per launch for bench.py's roofline.traffic: FETCH_SIZE and
      # WRITE_SIZE in passes of their own (MI355X_MICROARCH.md, HBM/rocprofv3)
      echo "== rocprofv3 traffic passes (${TRAFFIC_WL:-c2})"
      for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf $OUT/traffic_${TAG}_$c
        timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $ROOT/$OUT/traffic_${TAG}_$c -o run --output-format csv \
          -- python3 $ROOT/bench.py --workload ${TRAFFIC_WL:-c2} --secondary "" --steps 3 --warmup 1 --no-cpu-baseline \
          > $OUT/traffic_${TAG}_$c.log 2>&1 || { echo "traffic pass $c failed"; tail -20 $OUT/traffic_${TAG}_$c.log; exit 1; }
      done
      # per kernel of the attribution launch, stamped with the kernel-source hash
      python3 tools/pmc_pipeline.py --workload ${TRAFFIC_WL:-c2} --fetch $OUT/traffic_${TAG}_FETCH_SIZE \
        --write $OUT/traffic_${TAG}_WRITE_SIZE --out $OUT/pmc_${TRAFFIC_WL:-c2}_$TAG.json ;;
    marker)
      # roctx ranges (stage, attribute, merge, report) beside the kernel trace
      echo "== rocprofv3 marker + kernel trace"
      rm -rf $OUT/marker_$TAG
      timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --stats -d $ROOT/$OUT/marker_$TAG -o run --output-format csv \
        -- python3 $ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --secondary "" > $OUT/marker_$TAG.log 2>&1 \
        || { echo "marker trace failed"; tail -30 $OUT/marker_$TAG.log; exit 1; }
      find $OUT/marker_$TAG -name "*marker*" | head ;;
    merge)
      echo "== merge timing (${MERGE_WL:-c4})"
      timeout -k 10 900 python tools/merge_timing.py --workload ${MERGE_WL:-c4} > $OUT/merge_$TAG.json 2> $OUT/merge_$TAG.err \
        || { echo "merge timing failed"; tail -30 $OUT/merge_$TAG.err; exit 1; }
      cat $OUT/merge_$TAG.json ;;
    l2)
      # L2 hit rate and memory-side atomics of the attribution kernel
      echo "== rocprofv3 L2 passes (${L2_WL:-k1m})"
      i=0
      for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum" "TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_32B_sum"; do
        i=$((i+1))
        rm -rf $OUT/l2_${TAG}_$i
        timeout -k 10 400 rocprofv3 --pmc $set --kernel-trace -d $ROOT/$OUT/l2_${TAG}_$i -o run --output-format csv \
          -- python3 $ROOT/bench.py --workload ${L2_WL:-k1m} --steps 3 --warmup 1 --no-cpu-baseline > $OUT/l2_${TAG}_$i.log 2>&1 \
          || { echo "l2 pass $i failed"; tail -20 $OUT/l2_${TAG}_$i.log; exit 1; }
      done
      echo "l2 passes done" ;;
    pmcx)
      # arbitrary counter passes: PMCX_SETS="A B;C D" (one rocprofv3 run per set)
      echo "== rocprofv3 counter passes (${PMCX_WL:-c4})"
      i=0
      IFS=';' read -ra SETS <<< "${PMCX_SETS:-TCC_HIT_sum TCC_MISS_sum}"
      for set in "${SETS[@]}"; do
        i=$((i+1))
        rm -rf $OUT/pmcx_${TAG}_$i
        NMG_BENCH_DEBUG_FLAGS=${PMCX_FLAGS:-0} timeout -k 10 400 rocprofv3 --pmc $set --kernel-trace -d $ROOT/$OUT/pmcx_${TAG}_$i -o run --output-format csv \
          -- python3 $ROOT/bench.py --workload ${PMCX_WL:-c4} --secondary "" --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmcx_${TAG}_$i.log 2>&1 \
          || { echo "pmcx pass $i failed"; tail -20 $OUT/pmcx_${TAG}_$i.log; exit 1; }
      done
      python3 tools/pmc_kernels.py $OUT/pmcx_${TAG}_* ;;
    alloc)
      echo "== arena allocation experiment (${ALLOC_WL:-c4})"
      timeout -k 10 900 python tools/exp_alloc.py --workload ${ALLOC_WL:-c4} > $OUT/alloc_$TAG.json 2> $OUT/alloc_$TAG.err \
        || { echo "alloc failed"; tail -30 $OUT/alloc_$TAG.err; exit 1; }
      cat $OUT/alloc_$TAG.json ;;
    pmc)
      echo "== rocprofv3 pmc FETCH_SIZE"
      rm -rf $OUT/pmc_$TAG
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $ROOT/$OUT/pmc_$TAG -o run --output-format csv \
        -- python3 $ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/pmc_$TAG.log 2>&1 \
        || { echo "rocprof pmc failed"; tail -40 $OUT/pmc_$TAG.log; exit 1; }
      find $OUT/pmc_$TAG -name "*counter_collection.csv" -exec head -5 {} \; ;;
  esac
done
echo "== done"
