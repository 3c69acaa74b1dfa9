# round-3 session: BVH builder tests + timing, driver-command rocprof, distributed legs, bench
OUT=r3h bash tools/session_bvh.sh || exit 1
bash tools/gpu_session.sh gpurun_out/r3h prof_driver dist_gloo dist_rccl1 bench
