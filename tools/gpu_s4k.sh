set -o pipefail
# N=8 per-rank compute: frames per launch 8 vs 16, block dispatch, items of 1 tile
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4k
mkdir -p $O
V=$R/triangles-sdf-cpu-raytracing_amd/lib/var_mb16.so
for rep in 1 2; do
echo "== base g8" >> $O/ab.log; AB_NS=1,8 timeout -k 10 120 python tools/ab_split.py bunny >> $O/ab.log 2>&1 || { echo F1; exit 1; }
echo "== mb16 g16" >> $O/ab.log; RTAMD_LIB=$V AB_GROUP=16 AB_NS=1,8 timeout -k 10 120 python tools/ab_split.py bunny >> $O/ab.log 2>&1 || { echo F2; exit 1; }
echo "== persist0 g8" >> $O/ab.log; RTAMD_PERSIST=0 AB_NS=1,8 timeout -k 10 120 python tools/ab_split.py bunny >> $O/ab.log 2>&1 || { echo F3; exit 1; }
echo "== G1 g8" >> $O/ab.log; RTAMD_PERSIST_G=1 AB_NS=1,8 timeout -k 10 120 python tools/ab_split.py bunny >> $O/ab.log 2>&1 || { echo F4; exit 1; }
echo "== mb16 g16 grid" >> $O/ab.log; RTAMD_LIB=$V AB_GROUP=16 AB_NS=1,8 timeout -k 10 120 python tools/ab_split.py grid >> $O/ab.log 2>&1 || { echo F5; exit 1; }
echo "== base g8 grid" >> $O/ab.log; AB_NS=1,8 timeout -k 10 120 python tools/ab_split.py grid >> $O/ab.log 2>&1 || { echo F6; exit 1; }
done
echo ALLOK
