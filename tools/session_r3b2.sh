# row-band split, block dispatch vs the persistent queue for every band size,
# re-measured with one-wave persistent workgroups
set -o pipefail
OUT=gpurun_out/r3b2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for wl in bunny mesh_large; do
  for bp in default 8; do
    if [ $bp = default ]; then E=""; else E="RTAMD_BAND_PERSIST=$bp"; fi
    timeout -k 10 400 env $E python tools/ab.py split $wl > $OUT/split_${wl}_$bp.log 2>&1 || exit 1
    echo "== $wl band queue $bp"; grep "max over ranks\|N=1" $OUT/split_${wl}_$bp.log
  done
done
