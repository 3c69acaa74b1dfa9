# queue item size / dispatch re-measured with one-wave persistent workgroups
for wl in grid grid_shipped; do
  AB_WL=$wl AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3q2_$wl ab= ab=RTAMD_PERSIST_G=4 ab=RTAMD_PERSIST_G=2 || exit 1
done
for wl in octree_shipped bunny; do
  AB_WL=$wl AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3q2_$wl ab= ab=RTAMD_PERSIST_G=1 ab=RTAMD_PERSIST_G=4 || exit 1
done
