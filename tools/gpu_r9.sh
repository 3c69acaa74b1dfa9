set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r9
mkdir -p $O
AB_VARIANTS=8x2,8x1,16x1,32x1,16x2,32x2,64x1 timeout -k 10 500 python tools/ab_batch.py bunny grid octree mesh_large > $O/ab.log 2>&1 || { echo AFAIL; tail -20 $O/ab.log; exit 1; }
echo ALLOK
