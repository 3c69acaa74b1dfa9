set -o pipefail
# persistent work-queue batch kernel: parity, then A/B against the block dispatch
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rowsplit.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
AB_VARIANTS=8x1,8x2 timeout -k 10 240 python tools/ab_batch.py bunny grid example_grid.grid sdf_6.octree octree mesh_large > $O/ab_persist.log 2>&1 || { echo AFAIL; tail -20 $O/ab_persist.log; exit 1; }
RTAMD_PERSIST=0 AB_VARIANTS=8x1,8x2 timeout -k 10 240 python tools/ab_batch.py bunny grid example_grid.grid sdf_6.octree octree mesh_large > $O/ab_block.log 2>&1 || { echo AFAIL2; tail -20 $O/ab_block.log; exit 1; }
echo ALLOK
