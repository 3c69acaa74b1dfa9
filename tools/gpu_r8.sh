set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SFAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BFAIL; tail -20 $O/bench.err; exit 1; }
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o r8 --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-pmc > $O/bench_prof.json 2> $O/bench_prof.err || { echo PFAIL; tail -20 $O/bench_prof.err; exit 1; }
echo ALLOK
