# drop-in rt_render: 4 row bands with overlapped copies vs the whole frame (RTAMD_DROP_BANDS=1)
bash tools/gpu_session.sh gpurun_out/r3v ptest=RTAMD_DROP_BANDS=4 short= short=RTAMD_DROP_BANDS=1 short=RTAMD_DROP_BANDS=2
