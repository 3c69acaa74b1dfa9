# round-5 session 9: fast reciprocal in the triangle test -- exhaustive check, parity, A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5m; mkdir -p $O
echo "== rcp + mesh parity"; timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py > $O/parity.log 2>&1; tail -1 $O/parity.log
echo "== A/B"; bash tools/ab_oct.sh "main norcp" 2 "bunny mesh_large default_mode" > $O/rcp_ab.txt 2>&1; grep -v amdgpu $O/rcp_ab.txt
echo "== done"
