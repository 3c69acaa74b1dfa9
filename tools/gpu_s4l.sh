set -o pipefail
# per-rank compute at N=2,4: block dispatch vs work queue
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4l
mkdir -p $O
for wl in bunny grid mesh_large; do
echo "== persist1 $wl" >> $O/ab.log; AB_NS=1,2,4 timeout -k 10 150 python tools/ab_split.py $wl >> $O/ab.log 2>&1 || { echo F1; exit 1; }
echo "== persist0 $wl" >> $O/ab.log; RTAMD_PERSIST=0 AB_NS=1,2,4 timeout -k 10 150 python tools/ab_split.py $wl >> $O/ab.log 2>&1 || { echo F2; exit 1; }
done
echo ALLOK
