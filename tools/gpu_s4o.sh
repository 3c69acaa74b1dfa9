set -o pipefail
# mesh kernel registers: leaf batch 4/2 x waves floor compiler/4
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4o
mkdir -p $O
L=$R/triangles-sdf-cpu-raytracing_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
RTAMD_LIB=$L/var_lb2mw4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "not no_fallback" -x -q --timeout 120 --timeout-method thread >> $O/tests.log 2>&1 || { echo TFAIL2; tail -30 $O/tests.log; exit 1; }
for rep in 1 2; do
for v in librtamd var_mw4 var_lb2 var_lb2mw4; do
echo "== $v" >> $O/ab.log; RTAMD_LIB=$L/$v.so AB_VARIANTS=8x2 timeout -k 10 200 python tools/ab_batch.py bunny mesh_large >> $O/ab.log 2>&1 || { echo F $v; exit 1; }
done
done
echo ALLOK
