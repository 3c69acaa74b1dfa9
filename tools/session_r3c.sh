# cooperative mesh tail threshold: 8 (shipping) vs 12 / 16 rays (rounds of 8 groups)
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3c short= short=RTAMD_LIB=$L/var_coop12.so short=RTAMD_LIB=$L/var_coop16.so short= || exit 1
AB_WL=mesh_large AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3c_ml ab= ab=RTAMD_LIB=$L/var_coop12.so ab=RTAMD_LIB=$L/var_coop16.so
