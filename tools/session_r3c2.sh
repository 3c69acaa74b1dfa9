# cooperative mesh tail threshold: 16 / 20 / 24 / 32 rays against 8 (shipping)
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3c2 short= short=RTAMD_LIB=$L/var_coop16.so short=RTAMD_LIB=$L/var_coop20.so \
  short=RTAMD_LIB=$L/var_coop24.so short=RTAMD_LIB=$L/var_coop32.so short=RTAMD_LIB=$L/var_coop16.so short= || exit 1
AB_WL=mesh_large AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3c2_ml ab=RTAMD_LIB=$L/var_coop16.so ab=RTAMD_LIB=$L/var_coop24.so ab=RTAMD_LIB=$L/var_coop32.so
