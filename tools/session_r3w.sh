# round-3 final-build session: GPU suite (incl. the grid pump), full-size tests,
# smoke, the driver's bench command, rocprof stats of it; then A/B legs:
# coop-tail wave priority (prio2/prio3 variants) and the grid on the pump
L=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib
bash tools/gpu_session.sh gpurun_out/r3w tests fulltests smoke bench prof_driver \
  short= short=RTAMD_LIB=$L/var_prio2.so short=RTAMD_LIB=$L/var_prio3.so && \
AB_WL=grid AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3w_g ab= ab=RTAMD_PUMP=1 ab=RTAMD_PUMP=1,RTAMD_REFILL=32 ab=RTAMD_PUMP=1,RTAMD_REFILL=48 && \
AB_WL=grid_shipped AB_VARIANTS=8x2,8x1 bash tools/gpu_session.sh gpurun_out/r3w_g65 ab= ab=RTAMD_PUMP=1 ab=RTAMD_PUMP=1,RTAMD_REFILL=32
