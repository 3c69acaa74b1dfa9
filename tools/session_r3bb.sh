# one-wave workgroups for the multi-frame block dispatch (grids, small row bands)
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
AB_K="not fullsize" bash tools/gpu_session.sh gpurun_out/r3bb_t ptest=RTAMD_LIB=$L/var_bb64.so || exit 1
for wl in grid grid_shipped; do
  AB_WL=$wl AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3bb_$wl ab= ab=RTAMD_LIB=$L/var_bb64.so ab= ab=RTAMD_LIB=$L/var_bb64.so || exit 1
done
set -o pipefail
mkdir -p gpurun_out/r3bb
for v in base bb64; do
  if [ $v = base ]; then E=""; else E="RTAMD_LIB=$L/var_bb64.so"; fi
  timeout -k 10 400 env $E AB_NS=4,8 python tools/ab.py split bunny > gpurun_out/r3bb/split_$v.log 2>&1 || exit 1
  echo "== split $v"; grep "max over\|N=1:" gpurun_out/r3bb/split_$v.log
done
