# round-5 session 11: exact fast division in the ray setup -- checks, parity, A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5p; mkdir -p $O
echo "== division checks + parity"; timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_fullsize.py tests/test_rowsplit.py tests/test_grid_layout.py > $O/parity.log 2>&1; tail -1 $O/parity.log
echo "== A/B"; AB_VARIANTS=8x2 bash tools/ab_oct.sh "main nodiv" 3 "bunny grid grid_shipped octree octree_shipped mesh_large" > $O/div_ab.txt 2>&1; grep -v amdgpu $O/div_ab.txt
echo "== done"
