set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6_of
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_of/prof -o p -- python3 tools/prof_frames.py --plan bunny:stanford-bunny.obj:1920:1080:primary --group 1 --launches 64 > gpurun_out/r6_of/log.txt 2>&1
rc=$?; echo rc=$rc; tail -3 gpurun_out/r6_of/log.txt
find gpurun_out/r6_of/prof -name "*kernel_stats.csv" | xargs cat | cut -c1-250
