set -o pipefail
# one-probe queue drain: parity, then A/B vs block dispatch (N=1) and the row split legs
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
for rep in 1 2; do
echo "== persist1" >> $O/ab.log; AB_VARIANTS=8x1,8x2 timeout -k 10 200 python tools/ab_batch.py bunny grid sdf_6.octree mesh_large >> $O/ab.log 2>&1 || { echo F1; exit 1; }
echo "== persist0" >> $O/ab.log; RTAMD_PERSIST=0 AB_VARIANTS=8x1,8x2 timeout -k 10 200 python tools/ab_batch.py bunny grid sdf_6.octree mesh_large >> $O/ab.log 2>&1 || { echo F2; exit 1; }
done
AB_NS=1,2,4,8 timeout -k 10 150 python tools/ab_split.py bunny > $O/split.log 2>&1 || { echo F3; exit 1; }
echo ALLOK
