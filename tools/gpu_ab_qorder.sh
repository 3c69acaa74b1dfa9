#!/bin/bash
# Work-queue item order A/B (dev): RTAMD_QORDER 0 (frame-major), 1 (cost-ordered),
# 2 (frames interleaved) on the persistent workloads and the driver's bench command.
set -o pipefail
OUT=gpurun_out/${1:-qorder}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in 0 2 1; do
  RTAMD_QORDER=$v AB_VARIANTS=8x1,8x2 timeout -k 10 300 python tools/ab.py batch bunny octree_shipped mesh_large > $OUT/ab_q$v.log 2>&1 || { tail -20 $OUT/ab_q$v.log; exit 1; }
  echo "== QORDER=$v"; grep -v amdgpu.ids $OUT/ab_q$v.log
  for st in 20 128; do
    RTAMD_QORDER=$v timeout -k 10 200 python bench.py --steps $st --warmup 5 --no-pmc --no-extra --no-cpu-baseline > $OUT/bench_q${v}_$st.log 2>&1 || { tail -20 $OUT/bench_q${v}_$st.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/bench_q${v}_$st.log').read().strip().splitlines()[-1]); print('bench steps $st', d['ms_per_step'], d['roofline']['kernel_ms'], d.get('roofline_one_stream',{}).get('ms_per_step'))"
  done
done
