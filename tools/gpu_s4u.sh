set -o pipefail
# grid march: taps of the last cell reused
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4u
mkdir -p $O
L=$R/triangles-sdf-cpu-raytracing_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
for rep in 1 2; do
for v in librtamd var_tc0; do
echo "== $v" >> $O/ab.log; RTAMD_LIB=$L/$v.so AB_VARIANTS=8x2,8x1 timeout -k 10 200 python tools/ab_batch.py grid example_grid.grid >> $O/ab.log 2>&1 || { echo F $v; exit 1; }
done
done
echo ALLOK
