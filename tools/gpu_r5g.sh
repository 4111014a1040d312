set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5g.log 2>&1 || { tail -60 gpurun_out/pytest_r5g.log; exit 1; }
tail -2 gpurun_out/pytest_r5g.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r5g.log 2>&1 || { tail -20 gpurun_out/smoke_r5g.log; exit 1; }
tail -2 gpurun_out/smoke_r5g.log
bash tools/ab_lib.sh build_ab/lib_w8.so build_ab/lib_d6.so build_ab/lib_rd.so
