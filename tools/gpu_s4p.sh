set -o pipefail
# occupancy floors under the current dispatch: octree 1 (compiler) / 5 / 6 (default) / 8, grid 1 (default) / 6
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4p
mkdir -p $O
L=$R/triangles-sdf-cpu-raytracing_amd/lib
for rep in 1 2; do
for v in librtamd var_ow1 var_ow5 var_ow8; do
echo "== $v" >> $O/ab.log; RTAMD_LIB=$L/$v.so AB_VARIANTS=8x2 timeout -k 10 200 python tools/ab_batch.py sdf_6.octree octree >> $O/ab.log 2>&1 || { echo F $v; exit 1; }
done
for v in librtamd var_gw6; do
echo "== $v" >> $O/ab.log; RTAMD_LIB=$L/$v.so AB_VARIANTS=8x2,8x1 timeout -k 10 200 python tools/ab_batch.py grid example_grid.grid >> $O/ab.log 2>&1 || { echo F $v; exit 1; }
done
done
echo ALLOK
