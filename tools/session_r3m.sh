# PMC issue mix of the final build: two --pmc passes over 2 launches of 8 frames
# per workload on one stream (tools/prof_frames.py), one rocprofv3 run per pass
set -o pipefail
OUT=gpurun_out/r3m; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PLAN=bunny:stanford-bunny.obj:1920:1080:primary,sdf6:sdf_6.octree:3840:2160:primary,grid65:example_grid.grid:1920:1080:primary,large:mesh_large:3840:2160:primary
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/mix -o p -- python3 tools/prof_frames.py --plan $PLAN > $OUT/mix.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/wait -o p -- python3 tools/prof_frames.py --plan $PLAN > $OUT/wait.log 2>&1 || exit 1
python3 tools/issue_mix.py $OUT/mix $OUT/wait > $OUT/issue_mix.txt && tail -n 12 $OUT/issue_mix.txt
