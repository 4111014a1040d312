#!/bin/bash
# Build a variant of libnumamma_gpu.so with extra -D flags into build_ab/:
#   tools/ab_build.sh NAME "-DFOO=1 -DBAR=2"
set -e
cd "$(dirname "$0")/../numamma_amd"
NAME=$1; DEFS=$2
mkdir -p ../build_ab/obj_$NAME
for f in nmg_kernels nmg_route nmg_engine nmg_table nmg_submit nmg_route_host nmg_results nmg_multi; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -Wall -Wno-unused-result $DEFS \
    -x hip -c csrc/$f.hip -o ../build_ab/obj_$NAME/$f.o &
done
wait
for f in nmg_kernels nmg_route nmg_engine nmg_table nmg_submit nmg_route_host nmg_results nmg_multi; do [ -f ../build_ab/obj_$NAME/$f.o ] || { echo "compile of $f failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../build_ab/lib_$NAME.so ../build_ab/obj_$NAME/*.o build/nmg_report.o \
  build/nmg_replay.o -L/opt/rocm/lib -lrocprofiler-sdk-roctx
rm -rf ../build_ab/obj_$NAME
echo built build_ab/lib_$NAME.so
