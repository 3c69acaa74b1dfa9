# round-5 session 5: pageable drop-in with per-row spans
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5g; mkdir -p $O
echo "== rowsplit tests"; timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_rowsplit.py > $O/rowsplit_tests.log 2>&1; tail -1 $O/rowsplit_tests.log
echo "== dropin A/B"; for r in 1 2 3; do
  AB_FRAMES=32 timeout -k 10 120 python tools/ab.py dropin bunny 2>&1 | grep drop-in
done > $O/dropin_ab.txt; cat $O/dropin_ab.txt
echo "== done"
