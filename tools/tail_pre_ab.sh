# last-frame prefix of the persistent launches (RTAMD_TAIL_PRE=<items>) vs off,
# the driver's 20 frames as 10 x 2 and 128 frames as 8 x 2, interleaved rounds:
# tools/tail_pre_ab.sh [outdir] [values]
# The recipe of profiles/r05/tail_pre_ab.txt: the RTAMD_TAIL_PRE code was
# measured level and removed, so on the shipping sources
# every value runs the same kernel.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/tail_pre}; mkdir -p $O
V=${2:-"0 256 1024"}
for r in 1 2 3; do
  for p in $V; do
    RTAMD_TAIL_PRE=$p AB_STEPS=20 AB_WARM=5 AB_VARIANTS="10x2" timeout -k 10 120 python tools/ab.py batch bunny mesh_large > $O/ab20_${p}_$r.log 2>&1
    echo "pre=$p round $r (20 frames): $(grep frames $O/ab20_${p}_$r.log | tr '\n' ' ')"
  done
done
for p in $V; do
  RTAMD_TAIL_PRE=$p AB_VARIANTS="8x2" timeout -k 10 120 python tools/ab.py batch bunny > $O/ab128_${p}.log 2>&1
  echo "pre=$p (128 frames): $(grep frames $O/ab128_${p}.log | tr '\n' ' ')"
done
