export AB_WL="bunny octree octree_shipped grid mesh_large" AB_VARIANTS="8x2,8x1"
export PMC_PLAN="octree:octree:3840:2160:primary,octree_shipped:sdf_6.octree:3840:2160:primary"
L=triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3b tests ab= ab=RTAMD_LIB=$L/var_r2.so ab=RTAMD_LIB=$L/var_st.so \
  pmc=PMC_COUNTERS=WRITE_SIZE pmc=PMC_COUNTERS=WRITE_SIZE,RTAMD_LIB=$L/var_r2.so pmc=PMC_COUNTERS=WRITE_SIZE,RTAMD_LIB=$L/var_st.so split_large
