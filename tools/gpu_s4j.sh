set -o pipefail
# per-rank compute of the row split at N = 1, 2, 4, 8 on one GPU (no exchange)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4j
mkdir -p $O
timeout -k 10 200 python tools/ab_split.py bunny > $O/split_bunny.log 2>&1 || { echo SFAIL; tail -20 $O/split_bunny.log; exit 1; }
AB_STREAMS=3 timeout -k 10 200 python tools/ab_split.py bunny > $O/split_bunny_s3.log 2>&1 || { echo SFAIL3; tail -20 $O/split_bunny_s3.log; exit 1; }
timeout -k 10 200 python tools/ab_split.py grid > $O/split_grid.log 2>&1 || { echo SFAIL2; tail -20 $O/split_grid.log; exit 1; }
echo ALLOK
