#!/bin/bash
# Round-5 GPU session: route tests, then an A/B of library builds.
#   gpurun -- bash tools/gpu_r5.sh TAG "test-selection" lib_a.so[:FLAGS] ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=$1; shift
SEL=$1; shift
mkdir -p gpurun_out
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider $SEL \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_$TAG.log
fi
[ $# -gt 0 ] && bash tools/ab_lib.sh "$@"
