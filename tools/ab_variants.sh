#!/bin/bash
# Interleaved A/B of build variants (tools/build_variant.sh) on the GPU box:
#   tools/ab_variants.sh OUT ROUNDS "var1 var2 ..." [workload ...]
# each round runs tools/ab.py batch over the workloads once per variant
# (RTAMD_LIB=lib/var_<v>.so; "ship" = the shipping lib/librtamd.so), variants
# in order, AB_VARIANTS frames x streams (default 10x2,8x1,1x1). Every run has
# its own time limit; the first failure ends the session.
set -o pipefail
OUT=${1:-gpurun_out/ab}; ROUNDS=${2:-2}; VARS=${3:-"base"}; shift 3
WL=${*:-bunny}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export AB_VARIANTS=${AB_VARIANTS:-10x2,8x1,1x1}
L=triangles-sdf-cpu-raytracing_amd/lib
for r in $(seq 1 "$ROUNDS"); do
  for v in $VARS; do
    lib=$L/var_$v.so; [ "$v" = ship ] && lib=$L/librtamd.so
    echo "== round $r variant $v"
    timeout -k 10 300 env RTAMD_LIB=$PWD/$lib python tools/ab.py batch $WL > "$OUT/r${r}_$v.log" 2>&1
    rc=$?; grep -v amdgpu "$OUT/r${r}_$v.log" | sed "s/^/[$v r$r] /"
    [ $rc -ne 0 ] && { echo "variant $v failed rc=$rc"; exit 1; }
  done
done
echo "== ab done"
