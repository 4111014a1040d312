# route2 ablation builds (build_ab/lib_abl*.so): the route kernel's time per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r4}
for lib in ${LIBS:-build_ab/lib_abl0.so build_ab/lib_abl4.so build_ab/lib_abl8.so build_ab/lib_abl12.so}; do
  n=$(basename $lib .so)
  NMG_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u tools/ablate.py --workloads c4 --reps 6 --variants ${VARIANTS:-route_v2} > gpurun_out/abl_${n}_$T.json 2> gpurun_out/abl_${n}_$T.err || { tail -20 gpurun_out/abl_${n}_$T.err; exit 1; }
  sed "s/^/$n /" gpurun_out/abl_${n}_$T.json
done
