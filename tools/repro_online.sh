# (diagnosis) the online GPU tests, three runs of the module on the tree as built
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 400 python -m pytest -q -p no:cacheprovider tests/test_gpu_online.py > gpurun_out/repro_online_malloc_$i.log 2>&1
  echo "run $i rc=$? $(tail -1 gpurun_out/repro_online_malloc_$i.log)"
done
