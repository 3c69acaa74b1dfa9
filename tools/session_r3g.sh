# frames per launch x streams, re-measured with one-wave persistent workgroups
set -o pipefail
OUT=gpurun_out/r3g; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
for gs in "8 2" "4 2" "8 3" "6 2" "8 4"; do
  set -- $gs
  for st in 20 128; do
    timeout -k 10 200 python bench.py --steps $st --warmup 5 --group $1 --streams $2 --no-pmc --no-cpu-baseline --no-extra > $OUT/g$1_s$2_$st_$rep.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('group', $1, 'streams', $2, 'steps', $st, d['ms_per_step'])" $OUT/g$1_s$2_$st_$rep.log
  done
done
done
