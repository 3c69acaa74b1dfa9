# round-3 checkpoint: BVH builder tests + timing, the whole GPU suite, smoke,
# the driver's bench command, its rocprof kernel stats, distributed legs
OUT=r3q bash tools/session_bvh.sh || exit 1
bash tools/gpu_session.sh gpurun_out/r3q tests fulltests smoke bench prof_driver dist_gloo dist_rccl1
