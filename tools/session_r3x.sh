# two-stream overlap of persistent launches: per-launch wave stamps (stamps build)
set -o pipefail
OUT=gpurun_out/r3x; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export RTAMD_LIB=$GRAFT_REPO_ROOT/triangles-sdf-cpu-raytracing_amd/lib/var_stamps.so
for a in "bunny 20 2" "bunny 64 2" "bunny 16 1"; do
  echo "== overlap $a"
  timeout -k 10 240 python tools/overlap_probe.py $a > "$OUT/overlap_${a// /_}.log" 2>&1 || { echo FAIL; tail -n 20 "$OUT/overlap_${a// /_}.log"; exit 1; }
done
echo done
