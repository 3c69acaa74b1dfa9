set -o pipefail
# persistent queue: tiles per claim (G) A/B, spread heads
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rowsplit.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
for g in 1 2 4; do
RTAMD_PERSIST_G=$g AB_VARIANTS=8x1,8x2 timeout -k 10 240 python tools/ab_batch.py bunny grid example_grid.grid sdf_6.octree octree mesh_large > $O/ab_g$g.log 2>&1 || { echo AFAIL; tail -20 $O/ab_g$g.log; exit 1; }
done
echo ALLOK
