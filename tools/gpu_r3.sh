mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_rowsplit.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r3/tests.log; exit 1; }
timeout -k 10 400 python -u tools/ab_batch.py bunny grid example_grid.grid octree sdf_6.octree mesh_large > gpurun_out/r3/ab.log 2>&1 || { echo ABFAIL; tail -30 gpurun_out/r3/ab.log; exit 1; }
echo ALLOK
