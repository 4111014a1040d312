# (diagnosis) the whole GPU suite over the mapped-pool library (build_ab/lib_mapped.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
NMG_LIB_AB=1 NMG_LIB_PATH=$PWD/build_ab/lib_mapped.so timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/repro_suite_mapped.log 2>&1
rc=$?
tail -25 gpurun_out/repro_suite_mapped.log
exit $rc
