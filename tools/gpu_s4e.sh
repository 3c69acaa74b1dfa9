set -o pipefail
# full check of the current build: GPU tests, bench, rocprofv3 stats of the bench, host BVH build times
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BFAIL; tail -20 $O/bench.err; exit 1; }
echo BENCH_OK
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r1 --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $O/bench_under_rocprof.json 2> $O/prof.err || { echo PFAIL; tail -20 $O/prof.err; exit 1; }
echo PROF_OK
for t in 1 4 16; do OMP_NUM_THREADS=$t timeout -k 10 120 python tools/bvh_time.py >> $O/bvh_time.log 2>&1 || { echo BVHFAIL; exit 1; }; done
OMP_WAIT_POLICY=passive OMP_NUM_THREADS=16 timeout -k 10 120 python tools/bvh_time.py >> $O/bvh_time.log 2>&1
lscpu | grep -i "model name" >> $O/bvh_time.log
echo ALLOK
