# round-5 session 8: frames per launch = steps split over the streams (bench default), N = 1 and N = 8 split
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5j; mkdir -p $O
for r in 1 2; do for g in default 8; do
  e=""; [ $g != default ] && e="--group $g"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-pmc --no-drop-in $e > $O/bench_$g.log 2>&1
  python -c "import json; d=json.loads([l for l in open('$O/bench_$g.log') if l.startswith('{')][-1]); print('round $r group $g:', d['value'], d['ms_per_step'], d['config'].get('frames_per_launch'))"
done; done | tee $O/bench_group.txt
echo "== split 20 N=8"; for r in 1 2; do for g in 10 16; do
  echo "-- $r group $g"; AB_STEPS=20 AB_GROUP=$g AB_NS=8 timeout -k 10 200 python tools/ab.py split bunny 2>&1 | grep -E "max over|N=1"
done; done > $O/split20_group.txt; cat $O/split20_group.txt
echo "== dist gloo"; timeout -k 10 300 env RTAMD_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 > $O/dist_gloo.log 2>&1; grep "^{" $O/dist_gloo.log | tail -1 > $O/dist_gloo.json; python -c "import json; d=json.load(open('$O/dist_gloo.json')); print(d['value'], d['n_gpus'], d['config'].get('frames_per_launch'), d.get('frame_check'))"
echo "== variants"; bash tools/ab_oct.sh "main w6 lb2w6 oct7" 2 "bunny octree mesh_large" > $O/variants_ab.txt 2>&1; grep -v amdgpu $O/variants_ab.txt
echo "== done"
