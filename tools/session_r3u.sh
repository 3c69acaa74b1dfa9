# builder at the 1024 short-sort bound (tests + timing); banded drop-in rt_render (tests + bench row)
OUT=r3u bash tools/session_bvh.sh || exit 1
bash tools/gpu_session.sh gpurun_out/r3u tests short=
