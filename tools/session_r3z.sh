# persistent workgroup of one wave (new default): GPU suite, full-size tests,
# smoke, the driver's bench command, and a same-box A/B against 256 threads
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3z tests fulltests smoke bench \
  short= short=RTAMD_LIB=$L/var_pb256.so short= short=RTAMD_LIB=$L/var_pb256.so
