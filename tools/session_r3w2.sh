# occupancy floors re-measured with one-wave persistent workgroups: default shading
# (RT_GENERAL_WAVES 3 / 4 / 5) and the octree (RT_OCT_WAVES 5 / 6 / 7)
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
AB_WL=default_mode AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3w2_dm ab= ab=RTAMD_LIB=$L/var_gw3.so ab=RTAMD_LIB=$L/var_gw5.so ab= || exit 1
for wl in octree_shipped octree; do
  AB_WL=$wl AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3w2_$wl ab= ab=RTAMD_LIB=$L/var_ow5.so ab=RTAMD_LIB=$L/var_ow7.so || exit 1
done
