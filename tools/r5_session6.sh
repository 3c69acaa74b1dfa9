# round-5 session 6: full GPU suite, driver bench, 20-frame split after the event fixes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5h; mkdir -p $O
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests -k "not fullsize" > $O/gpu_tests.log 2>&1; tail -1 $O/gpu_tests.log
echo "== bench"; timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1; grep "^{" $O/bench.log | tail -1 > $O/bench.json
echo "== split 20"; for g in 16 8; do
  echo "-- group $g"; AB_STEPS=20 AB_GROUP=$g AB_NS=8 timeout -k 10 200 python tools/ab.py split bunny mesh_large 2>&1 | grep -E "N=8|N=1"
done > $O/split20.txt; grep -E "max over|N=1|group" $O/split20.txt
echo "== done"
