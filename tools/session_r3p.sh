# paired-frame queue order (RTAMD_PAIR=1) against frame after frame, same box
bash tools/gpu_session.sh gpurun_out/r3p ptest=RTAMD_PAIR=1 short= short=RTAMD_PAIR=1 short= short=RTAMD_PAIR=1 || exit 1
for wl in mesh_large octree_shipped; do
  AB_WL=$wl AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3p_$wl ab= ab=RTAMD_PAIR=1 || exit 1
done
