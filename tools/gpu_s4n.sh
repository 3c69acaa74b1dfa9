set -o pipefail
# profile refresh for the current build: GPU suite, bench (live PMC), rocprofv3 stats, PMC passes
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
echo TESTS_OK
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BFAIL; tail -20 $O/bench.err; exit 1; }
echo BENCH_OK
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o r1 --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $O/bench_under_rocprof.json 2> $O/prof.err || { echo PFAIL; tail -20 $O/prof.err; exit 1; }
echo PROF_OK
bash tools/pmc.sh $O/pmc_bunny stanford-bunny.obj 32 8 > $O/pmc_bunny.log 2>&1 || { echo PMCFAIL; cat $O/pmc_bunny.log; exit 1; }
bash tools/pmc.sh $O/pmc_grid grid 32 8 > $O/pmc_grid.log 2>&1 || { echo PMCFAIL2; cat $O/pmc_grid.log; exit 1; }
PMC_KERNEL=render_persist_kernel python tools/pmc_summary.py $O/pmc_bunny > $O/pmc_summary.txt 2>&1
PMC_KERNEL=render_batch_kernel python tools/pmc_summary.py $O/pmc_grid >> $O/pmc_summary.txt 2>&1
echo ALLOK
