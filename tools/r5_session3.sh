# round-5 session 3: host-frame store scope x drop-in bands; kernel traces of the N=8 band split
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5e; mkdir -p $O
echo "== dropin tests"; timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_rowsplit.py -k "drop_in" > $O/dropin_tests.log 2>&1; tail -1 $O/dropin_tests.log
echo "== dropin A/B"; for r in 1 2; do for hs in sys agent; do for k in 1 2 4; do
  RTAMD_HOST_STORES=$hs RTAMD_DROPIN_BANDS=$k AB_FRAMES=32 timeout -k 10 120 python tools/ab.py dropin bunny 2>&1 | grep drop-in | sed "s/^/$hs K=$k /"
done; done; done > $O/dropin_ab.txt; cat $O/dropin_ab.txt
for v in block queue; do
  e=""; [ $v = queue ] && e="RTAMD_BAND_PERSIST=8"
  echo "== trace split $v"
  env $e AB_STEPS=20 AB_GROUP=16 AB_NS=8 AB_WARM=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o p -- python3 tools/ab.py split bunny > $O/tr_$v.log 2>&1
  grep -E "max over|N=1" $O/tr_$v.log
done
echo "== done"
