# round-5 session 10: fast reciprocal behind the per-scene direction bound -- parity and A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5n; mkdir -p $O
echo "== parity"; timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_fullsize.py tests/test_rowsplit.py > $O/parity.log 2>&1; tail -1 $O/parity.log
echo "== A/B"; bash tools/ab_oct.sh "main norcp rcpnofb" 2 "bunny mesh_large default_mode" > $O/rcp_ab.txt 2>&1; grep "2 streams\|round" $O/rcp_ab.txt
echo "== done"
