# cooperative mesh tail threshold 12 / 16 rays in rounds of 8 (fixed round size), parity first
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
AB_K="parity or fullsize_primary" bash tools/gpu_session.sh gpurun_out/r3c4_t ptest=RTAMD_LIB=$L/var_coop16.so || exit 1
bash tools/gpu_session.sh gpurun_out/r3c4 short= short=RTAMD_LIB=$L/var_coop12.so short=RTAMD_LIB=$L/var_coop16.so short= short=RTAMD_LIB=$L/var_coop16.so
