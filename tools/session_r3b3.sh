# row-band split of the bunny: streams per rank 2 / 3 / 4
set -o pipefail
OUT=gpurun_out/r3b3; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for ns in 2 3 4; do
  timeout -k 10 400 env AB_STREAMS=$ns AB_NS=4,8 python tools/ab.py split bunny > $OUT/split_bunny_s$ns.log 2>&1 || exit 1
  echo "== streams $ns"; grep "max over ranks\|N=1" $OUT/split_bunny_s$ns.log
done
