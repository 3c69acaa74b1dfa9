set -o pipefail
# octree child-word prefetch: parity, then A/B against the variant without it
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "octree or oct or sdf_6 or sdf_5 or standin or orbit or golden" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
for rep in 1 2; do
AB_VARIANTS=1x1,8x1,8x2 timeout -k 10 200 python tools/ab_batch.py sdf_6.octree octree >> $O/ab_pf.log 2>&1 || { echo AFAIL; exit 1; }
RTAMD_LIB=$R/triangles-sdf-cpu-raytracing_amd/lib/var_nopf.so AB_VARIANTS=1x1,8x1,8x2 timeout -k 10 200 python tools/ab_batch.py sdf_6.octree octree >> $O/ab_nopf.log 2>&1 || { echo AFAIL2; exit 1; }
done
echo ALLOK
