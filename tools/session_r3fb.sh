# one-wave workgroups for the one-frame kernel (frame latency, drop-in path), parity first
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
AB_K="not fullsize" bash tools/gpu_session.sh gpurun_out/r3fb_t ptest=RTAMD_LIB=$L/var_fb64.so || exit 1
for wl in bunny grid octree_shipped default_mode; do
  AB_WL=$wl AB_VARIANTS=1x1,1x2 bash tools/gpu_session.sh gpurun_out/r3fb_$wl ab= ab=RTAMD_LIB=$L/var_fb64.so ab= ab=RTAMD_LIB=$L/var_fb64.so || exit 1
done
