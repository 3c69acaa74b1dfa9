# round-5 session 2: banded pageable drop-in (tests + K A/B), band dispatch at the driver's 20 frames
set -e
cd $(dirname $0)/..
export TMPDIR=/tmp
O=gpurun_out/r5d; mkdir -p $O
echo "== dropin tests"; timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_rowsplit.py -k "drop_in" > $O/dropin_tests.log 2>&1; tail -1 $O/dropin_tests.log
echo "== dropin A/B"; for r in 1 2; do for k in 1 2 3 4 6; do
  RTAMD_DROPIN_BANDS=$k AB_FRAMES=32 timeout -k 10 120 python tools/ab.py dropin bunny 2>&1 | grep drop-in | sed "s/^/K=$k /"
done; done > $O/dropin_ab.txt; cat $O/dropin_ab.txt
echo "== split 20"; for r in 1 2; do for v in "" RTAMD_BAND_PERSIST=8; do for g in 8 16; do
  echo "-- $r [$v] group $g"; env $v AB_STEPS=20 AB_GROUP=$g AB_NS=8 timeout -k 10 200 python tools/ab.py split bunny 2>&1 | grep -E "max over|N=1"
done; done; done > $O/split20.txt; cat $O/split20.txt
echo "== done"
