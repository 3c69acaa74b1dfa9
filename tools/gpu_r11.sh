set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r11
mkdir -p $O
for v in g7o5 g8o6 g8o8 g7o5; do
RTAMD_LIB=$R/triangles-sdf-cpu-raytracing_amd/lib/var_$v.so AB_VARIANTS=8x2,8x1 timeout -k 10 300 python tools/ab_batch.py grid example_grid.grid octree sdf_6.octree > $O/ab_$v.log 2>&1 || { echo AFAIL; tail -20 $O/ab_$v.log; exit 1; }
done
echo ALLOK
