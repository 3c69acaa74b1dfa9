#!/bin/bash
# rocprofv3 kernel trace of one-frame renders (the frame_latency / drop-in
# kernels): tools/oneframe_prof.sh OUT [plan] [lib]
set -o pipefail
OUT=${1:-gpurun_out/of}; PLAN=${2:-bunny:stanford-bunny.obj:1920:1080:primary}; LIB=${3:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
[ -n "$LIB" ] && export RTAMD_LIB=$PWD/$LIB
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o p -- python3 tools/prof_frames.py --plan "$PLAN" --group 1 --launches 64 > "$OUT/log.txt" 2>&1
rc=$?; echo rc=$rc; [ $rc -ne 0 ] && tail -5 "$OUT/log.txt" && exit $rc
find "$OUT/prof" -name "*kernel_stats.csv" | xargs grep -h -E "Name|render_|order_kernel" | cut -c1-60,200-330
