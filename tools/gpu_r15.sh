set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r15
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
AB_VARIANTS=8x2,8x1 timeout -k 10 300 python tools/ab_batch.py grid example_grid.grid > $O/ab_main.log 2>&1 || { echo AFAIL; tail -20 $O/ab_main.log; exit 1; }
echo ALLOK
