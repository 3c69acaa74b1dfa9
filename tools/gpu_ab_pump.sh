#!/bin/bash
# Ray-pump A/B (dev): refill thresholds x occupancy variants on the octree, plus
# lane-utilisation counters for the pump and the tile-per-wave kernel.
set -o pipefail
OUT=gpurun_out/${1:-pump}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
LIBDIR=triangles-sdf-cpu-raytracing_amd/lib
ab() { local tag=$1; shift
  env "$@" AB_VARIANTS=8x1,8x2 timeout -k 10 200 python tools/ab.py batch octree_shipped > $OUT/ab_$tag.log 2>&1 || { tail -20 $OUT/ab_$tag.log; exit 1; }
  echo "== $tag"; grep -v amdgpu.ids $OUT/ab_$tag.log; }
ab nopump RTAMD_PUMP=0
for r in 32 48 64; do ab r$r RTAMD_REFILL=$r; done
for r in 16 32 48 64; do ab pw1_r$r RTAMD_LIB=$LIBDIR/var_pw1.so RTAMD_REFILL=$r; done
pmc() { local tag=$1; shift
  env "$@" timeout -s KILL 90 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $OUT/pmc_$tag -o p -- python3 tools/prof_frames.py --plan o:sdf_6.octree:3840:2160:primary > $OUT/pmc_$tag.log 2>&1 || { tail -5 $OUT/pmc_$tag.log; exit 1; }
  echo "== pmc $tag done"; }
pmc nopump RTAMD_PUMP=0
pmc r32 RTAMD_REFILL=32
pmc pw1_r48 RTAMD_LIB=$LIBDIR/var_pw1.so RTAMD_REFILL=48
