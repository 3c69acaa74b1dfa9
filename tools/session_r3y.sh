# persistent workgroup size A/B: 256 (shipping) vs 64 / 128 threads per block
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
set -o pipefail
bash tools/gpu_session.sh gpurun_out/r3y short= short=RTAMD_LIB=$L/var_pb64.so short=RTAMD_LIB=$L/var_pb128.so \
  short= short=RTAMD_LIB=$L/var_pb64.so || exit 1
for wl in mesh_large octree_shipped default_mode; do
  AB_WL=$wl AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3y_$wl ab= ab=RTAMD_LIB=$L/var_pb64.so || exit 1
done
mkdir -p gpurun_out/r3y
for v in stamps64 stamps; do
  timeout -k 10 240 env RTAMD_LIB=$L/var_$v.so python tools/overlap_probe.py bunny 20 2 > gpurun_out/r3y/overlap_$v.log 2>&1 || exit 1
  grep "launch \|span\|mean resident" gpurun_out/r3y/overlap_$v.log
done
bash tools/gpu_session.sh gpurun_out/r3y_t ptest=RTAMD_LIB=$L/var_pb64.so
