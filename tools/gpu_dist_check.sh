mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_rowsplit.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r5/tests.log; exit 1; }
for ex in p2p gather; do
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --dist --exchange $ex --no-extra --no-pmc --no-cpu-baseline > gpurun_out/r5/dist1_$ex.json 2> gpurun_out/r5/dist1_$ex.err || { echo D1FAIL; tail -20 gpurun_out/r5/dist1_$ex.err; exit 1; }
done
RTAMD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 32 --warmup 8 > gpurun_out/r5/gloo2_p2p.json 2> gpurun_out/r5/gloo2_p2p.err || { echo G2FAIL; tail -20 gpurun_out/r5/gloo2_p2p.err; exit 1; }
echo ALLOK
