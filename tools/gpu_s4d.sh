set -o pipefail
# persistent queue A/B in one box: block dispatch vs queue (tiles per claim G, head stride S), twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4d
mkdir -p $O
for rep in 1 2; do
for cfg in "0 1 1088" "1 1 16" "1 1 1088" "1 2 1088" "1 4 1088"; do
set -- $cfg
echo "== rep $rep persist $1 G $2 stride $3" >> $O/ab.log
RTAMD_PERSIST=$1 RTAMD_PERSIST_G=$2 RTAMD_QSTRIDE=$3 AB_VARIANTS=8x2 timeout -k 10 120 python tools/ab_batch.py bunny grid example_grid.grid sdf_6.octree octree mesh_large >> $O/ab.log 2>&1 || { echo AFAIL; tail -20 $O/ab.log; exit 1; }
done
done
echo ALLOK
