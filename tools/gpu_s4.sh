set -o pipefail
# Round-1 re-entry check: GPU tests, default bench, rocprofv3 kernel stats of the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BFAIL; tail -20 $O/bench.err; exit 1; }
echo BENCH_OK
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r1 --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $O/bench_under_rocprof.json 2> $O/prof.err || { echo PFAIL; tail -20 $O/prof.err; exit 1; }
echo ALLOK
