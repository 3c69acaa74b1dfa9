# LLVM scheduling strategies for rt_device.hip (tools/build_variant.sh
# libraries) vs the shipping library, 8 x 2 over 128 frames, two interleaved
# rounds: tools/sched_ab.sh [outdir] [variants]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/sched_ab}; mkdir -p $O
V=${2:-"main ilp memclause bias0"}
L=triangles-sdf-cpu-raytracing_amd/lib
for r in 1 2; do
  for v in $V; do
    if [ $v = main ]; then lib=$L/librtamd.so; else lib=$L/var_$v.so; fi
    RTAMD_LIB=$lib AB_VARIANTS="8x2" timeout -k 10 150 python tools/ab.py batch octree octree_shipped bunny mesh_large > $O/${v}_$r.log 2>&1
    echo "$v round $r: $(grep frames $O/${v}_$r.log | sed 's/ frames x 2 streams//; s/ ms\/launch//' | tr '\n' ';')"
  done
done
