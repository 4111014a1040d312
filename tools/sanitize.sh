#!/bin/bash
# Sanitizer pass over the host-side C/C++ (CPU only; no GPU code runs here).
#
#   bash tools/sanitize.sh [LOG]       (default profiles/r6/sanitize_r6.log)
#
# 1. ASan + UBSan (-fno-sanitize-recover: the first report fails the run):
#    - build_san/libnmg_host_san.so: the report writer (nmg_report.cpp: up to
#      16 page-file writer threads) and the replay reader / writer
#      (nmg_replay.cpp), with the device half stubbed (tools/san/nmg_host_stubs.cpp);
#    - build_san/liboracle.so, liboracle_mt.so: the oracle and the
#      multi-threaded restatement (test infrastructure);
#    then the CPU test modules that drive them (pytest -m "not gpu"), with the
#    sanitizer runtimes preloaded into python and the libraries swapped in
#    through NMG_LIB_PATH / NMG_ORACLE_DIR.
# 2. UBSan on the LD_PRELOAD test interposer (tests/c/nmg_interpose.c; ASan
#    owns malloc, so not both) under tests/test_interpose_host.py.
# 3. TSan: the report writer with 1 vs 7 writer threads
#    (tools/san/report_threads.cpp) and the multi-threaded restatement with
#    1 vs 8 threads (tools/san/mt_driver.c), each output compared.
# The engine's HIP host code (nmg_submit.hip's copy pool) is built by hipcc and
# is not covered: the GPU runtime cannot run here.
set -eo pipefail
cd "$(dirname "$0")/.."
ROOT=$PWD
LOG=${1:-profiles/r6/sanitize_r6.log}
OUT=build_san
mkdir -p $OUT "$(dirname "$LOG")"
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
TSAN="-fsanitize=thread -fno-omit-frame-pointer"
INC="-Iinclude -Inumamma_amd/csrc"
exec > >(tee "$LOG") 2>&1
echo "== sanitize.sh $(date -u +%FT%TZ) head $(git rev-parse --short HEAD) ($(gcc --version | head -1))"

echo "== build (ASan + UBSan)"
g++ -O1 -g -std=c++17 -fPIC -shared -pthread $SAN $INC -o $OUT/libnmg_host_san.so \
  numamma_amd/csrc/nmg_report.cpp numamma_amd/csrc/nmg_replay.cpp tools/san/nmg_host_stubs.cpp
gcc -O1 -g -fPIC -shared $SAN -o $OUT/liboracle.so oracle/nmg_oracle.c
g++ -O1 -g -std=c++17 -fPIC -shared -pthread $SAN -o $OUT/liboracle_mt.so oracle/nmg_cpu_mt.cpp
echo "== build (UBSan interposer)"
mkdir -p $OUT/bin
gcc -O1 -g -shared -fPIC -fsanitize=undefined -fno-sanitize-recover=undefined -o $OUT/bin/libnmg_interpose.so \
  tests/c/nmg_interpose.c -ldl -lpthread
echo "== build (TSan drivers)"
g++ -O1 -g -std=c++17 -pthread $TSAN $INC -o $OUT/report_threads tools/san/report_threads.cpp \
  numamma_amd/csrc/nmg_report.cpp numamma_amd/csrc/nmg_replay.cpp tools/san/nmg_host_stubs.cpp
g++ -O1 -g -std=c++17 -fPIC -shared -pthread $TSAN -o $OUT/liboracle_mt_tsan.so oracle/nmg_cpu_mt.cpp
gcc -O1 -g $TSAN -o $OUT/mt_driver tools/san/mt_driver.c -L$OUT -loracle_mt_tsan -Wl,-rpath,$ROOT/$OUT

echo "== ASan + UBSan: CPU tests over the report writer, replay format, oracle, restatement"
PRE="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
LD_PRELOAD=$PRE ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:allocator_may_return_null=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  NMG_LIB_PATH=$ROOT/$OUT/libnmg_host_san.so NMG_LIB_AB=1 NMG_ORACLE_DIR=$ROOT/$OUT \
  timeout -k 10 1500 python -m pytest -p no:cacheprovider -q -m "not gpu" \
  tests/test_report_host.py tests/test_readme_golden.py tests/test_replay.py tests/test_oracle_ref.py \
  tests/test_cpu_mt.py tests/test_online_oracle.py

echo "== UBSan: the test interposer under LD_PRELOAD"
NMG_INTERPOSER=$ROOT/$OUT/bin/libnmg_interpose.so UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  timeout -k 10 600 python -m pytest -p no:cacheprovider -q -m "not gpu" tests/test_interpose_host.py

echo "== TSan: report writer threads, multi-threaded restatement"
rm -rf $OUT/tsan_out && mkdir -p $OUT/tsan_out
TSAN_OPTIONS=halt_on_error=1 timeout -k 10 600 $OUT/report_threads $OUT/tsan_out
python3 -c "
import sys; sys.path.insert(0, '.')
from numamma_amd.replay import SynthConfig, generate
generate(SynthConfig(nb_samples=300_000, nb_intervals=20_000, lost_frac=1e-3, wrap_one=True, seed=5)).write('$OUT/tsan_out/r.bin')"
TSAN_OPTIONS=halt_on_error=1 timeout -k 10 600 $OUT/mt_driver $OUT/tsan_out/r.bin $OUT/tsan_out/raw
echo "== sanitize.sh: clean"
