# octree counters: the round-4 SQ set over 2 launches of 8 frames, one stream (tools/prof_frames.py); tools/octree_pmc.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/octree_pmc}; mkdir -p $O
for wl in "sdf6:sdf_6.octree:3840:2160:primary" "d8:octree:3840:2160:primary"; do
  name=${wl%%:*}
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $O/$name -o p -- python3 tools/prof_frames.py --plan "$wl" --group 8 --launches 2 > $O/$name.log 2>&1
  echo "$name done"
done
PMC_KERNEL=render_ python tools/pmc_summary.py $O/sdf6 $O/d8 > $O/summary.txt; cat $O/summary.txt
