# round-5 session 4: drop-in after the hit-box changes; host issue time of the N=8 band split
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5f; mkdir -p $O
echo "== rowsplit tests"; timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_rowsplit.py > $O/rowsplit_tests.log 2>&1; tail -1 $O/rowsplit_tests.log
echo "== dropin A/B"; for r in 1 2; do for k in 1 2 4; do
  RTAMD_DROPIN_BANDS=$k AB_FRAMES=32 timeout -k 10 120 python tools/ab.py dropin bunny 2>&1 | grep drop-in | sed "s/^/K=$k /"
done; done > $O/dropin_ab.txt; cat $O/dropin_ab.txt
echo "== split 20"; for g in 16 8; do
  echo "-- group $g"; AB_STEPS=20 AB_GROUP=$g AB_NS=8 timeout -k 10 200 python tools/ab.py split bunny 2>&1 | grep -E "N=8|N=1"
done > $O/split20.txt; cat $O/split20.txt
echo "== done"
