# scene-first queue order (RTAMD_SCENE_FIRST=0 restores frame after frame):
# GPU suite, same-box bench A/B, batch A/B on the other workloads, stamps
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3s tests fulltests \
  short= short=RTAMD_SCENE_FIRST=0 short= short=RTAMD_SCENE_FIRST=0 || exit 1
for wl in mesh_large octree_shipped octree; do
  AB_WL=$wl AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3s_$wl ab= ab=RTAMD_SCENE_FIRST=0 || exit 1
done
for v in 1 0; do
  timeout -k 10 240 env RTAMD_SCENE_FIRST=$v RTAMD_LIB=$L/var_stamps.so python tools/overlap_probe.py bunny 20 2 > gpurun_out/r3s/overlap_sf$v.log 2>&1 || exit 1
  grep "launch \|span\|mean resident" gpurun_out/r3s/overlap_sf$v.log
done
