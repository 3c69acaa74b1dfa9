mkdir -p gpurun_out/r6
timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline > gpurun_out/r6/bench.json 2> gpurun_out/r6/bench.err || { echo BFAIL; tail -20 gpurun_out/r6/bench.err; exit 1; }
bash tools/pmc.sh gpurun_out/r6/pmc_grid grid 16 > gpurun_out/r6/pmc_grid.log 2>&1 || { echo PFAIL; cat gpurun_out/r6/pmc_grid.log; exit 1; }
bash tools/pmc_occ.sh gpurun_out/r6/pmcocc_grid grid 16 > gpurun_out/r6/pmcocc_grid.log 2>&1 || { echo P2FAIL; cat gpurun_out/r6/pmcocc_grid.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r6/pmc_grid gpurun_out/r6/pmcocc_grid > gpurun_out/r6/pmc_grid_summary.txt
echo ALLOK
