set -o pipefail
# distributed legs on one GPU for the final build: RCCL at world 1 (p2p and gather), gloo at world 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4r
mkdir -p $O
for ex in p2p gather; do
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --dist --exchange $ex --no-extra --no-pmc --no-cpu-baseline > $O/dist1_$ex.json 2> $O/dist1_$ex.err || { echo D1FAIL; tail -20 $O/dist1_$ex.err; exit 1; }
done
RTAMD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 32 --warmup 8 > $O/gloo2_p2p.json 2> $O/gloo2_p2p.err || { echo G2FAIL; tail -20 $O/gloo2_p2p.err; exit 1; }
echo ALLOK
