# round-5 session 12: the driver's command three times (spread), the 20-frame N = 8 split on the final build
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5q; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$r.log 2>&1
  grep "^{" $O/bench_$r.log | tail -1 > $O/bench_$r.json
  python -c "import json; d=json.load(open('$O/bench_$r.json')); print('run $r', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drop_in']['pageable_cleared_ms'], d['drop_in']['pinned_cleared_ms'], {k: v['frac'] for k, v in d['extra'].items()})"
done
echo "== split 20"; for r in 1 2; do AB_STEPS=20 AB_GROUP=10 AB_NS=8 timeout -k 10 200 python tools/ab.py split bunny mesh_large 2>&1 | grep -E "max over|N=1"; done > $O/split20.txt; cat $O/split20.txt
echo "== done"
