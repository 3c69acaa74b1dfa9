#!/bin/bash
# Occupancy / lane-utilisation counters. usage: tools/pmc_occ.sh <outdir> <workload> [one-frame launches] [W H]
set -e
OUT=${1:-gpurun_out/pmcocc}; WL=${2:-stanford-bunny.obj}; N=${3:-16}; W=${4:-1920}; H=${5:-1080}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p -- \
    python3 tools/prof_frames.py --plan "w:$WL:$W:$H:primary" --launches $N --group 1 > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
}
run a SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LEVEL_WAVES SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAVE_CYCLES
run b SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
echo done
