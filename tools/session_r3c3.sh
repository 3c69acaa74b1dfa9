# cooperative mesh tail threshold: 32 / 40 / 48 / 64 rays against 8 (shipping)
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3c3 short= short=RTAMD_LIB=$L/var_coop32.so short=RTAMD_LIB=$L/var_coop40.so \
  short=RTAMD_LIB=$L/var_coop48.so short=RTAMD_LIB=$L/var_coop64.so short=RTAMD_LIB=$L/var_coop32.so || exit 1
AB_WL=mesh_large AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3c3_ml ab=RTAMD_LIB=$L/var_coop32.so ab=RTAMD_LIB=$L/var_coop48.so ab=RTAMD_LIB=$L/var_coop64.so
