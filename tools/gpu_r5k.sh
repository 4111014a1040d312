set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out profiles/r5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_distributed.py > gpurun_out/r5k_dist.log 2>&1 || { tail -30 gpurun_out/r5k_dist.log; exit 1; }
tail -3 gpurun_out/r5k_dist.log
timeout -k 10 900 python -u tools/merge8.py > gpurun_out/merge8_c4.json 2> gpurun_out/merge8_c4.err || { tail -30 gpurun_out/merge8_c4.err; exit 1; }
tail -12 gpurun_out/merge8_c4.err
python -c "import json; d=json.loads(open('gpurun_out/merge8_c4.json').read().splitlines()[-1]); print({k: d[k] for k in ('bit_exact','checks','records_total','matched_total','payload_bytes_per_rank','merge_s_rank0','analyze_s_rank0','wall_s')})"
