# cooperative mesh tail off (RT_COOP_RAYS=0) against on (8), one-wave workgroups
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3c5 short= short=RTAMD_LIB=$L/var_coop0.so short= short=RTAMD_LIB=$L/var_coop0.so || exit 1
AB_WL=mesh_large AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3c5_ml ab= ab=RTAMD_LIB=$L/var_coop0.so
