# uniform-node scalar loads (RT_UNIFORM_NODE variant) against the shipping build
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3u2 short= short=RTAMD_LIB=$L/var_uni.so short= short=RTAMD_LIB=$L/var_uni.so || exit 1
AB_WL=mesh_large AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3u2_ml ab= ab=RTAMD_LIB=$L/var_uni.so || exit 1
AB_K="parity or rowsplit" bash tools/gpu_session.sh gpurun_out/r3u2_t ptest=RTAMD_LIB=$L/var_uni.so
