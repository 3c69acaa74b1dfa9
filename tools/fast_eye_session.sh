set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5r; mkdir -p $O
echo "== parity"; timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_fullsize.py tests/test_rowsplit.py > $O/parity.log 2>&1; tail -1 $O/parity.log
echo "== A/B"; AB_VARIANTS=8x2 bash tools/ab_oct.sh "main main+RTAMD_FAST_EYE=0" 3 "bunny grid grid_shipped octree mesh_large" > $O/eye_ab.txt 2>&1; grep -v amdgpu $O/eye_ab.txt
