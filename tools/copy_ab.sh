# pageable drop-in copy: streaming stores vs memcpy (RTAMD_COPY_NT), two interleaved rounds:
# tools/copy_ab.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/copy_ab}; mkdir -p $O
for r in 1 2; do
  for nt in 1 0; do
    RTAMD_COPY_NT=$nt RTAMD_DROPIN_TRACE=1 AB_FRAMES=16 timeout -k 10 120 python tools/ab.py dropin bunny > $O/ab_${nt}_$r.log 2>&1
    echo "== nt=$nt round $r"; grep "^dropin" $O/ab_${nt}_$r.log | tail -6; grep "drop-in" $O/ab_${nt}_$r.log
  done
done
