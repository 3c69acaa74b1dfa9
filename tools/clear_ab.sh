# pageable / pinned drop-in: staging spans reset by the host copy threads vs
# (the switches are read only by A/B builds: first `bash tools/build_variant.sh abenv ""`)
# clear_spans_kernel (RTAMD_HOST_CLEAR), two interleaved rounds: tools/clear_ab.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export RTAMD_LIB=$PWD/triangles-sdf-cpu-raytracing_amd/lib/var_abenv.so
O=${1:-gpurun_out/clear_ab}; mkdir -p $O
for r in 1 2; do
  for hc in 1 0; do
    RTAMD_HOST_CLEAR=$hc RTAMD_DROPIN_TRACE=1 AB_FRAMES=16 timeout -k 10 120 python tools/ab.py dropin bunny > $O/ab_${hc}_$r.log 2>&1
    echo "== host_clear=$hc round $r"; grep "^dropin" $O/ab_${hc}_$r.log | tail -4; grep "drop-in" $O/ab_${hc}_$r.log
  done
done
