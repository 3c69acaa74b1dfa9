set -o pipefail
# mesh kernel at 4 waves/SIMD by default: full GPU suite, then the distributed bench legs on one GPU
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --dist --no-extra --no-pmc --no-cpu-baseline > $O/dist1_p2p.json 2> $O/dist1_p2p.err || { echo D1FAIL; tail -20 $O/dist1_p2p.err; exit 1; }
RTAMD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 32 --warmup 8 > $O/gloo2_p2p.json 2> $O/gloo2_p2p.err || { echo G2FAIL; tail -20 $O/gloo2_p2p.err; exit 1; }
echo ALLOK
