# round-5 session 7: bench + 20-frame split + distributed paths after the GC placement fix
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5i; mkdir -p $O
echo "== bench"; timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1; grep "^{" $O/bench.log | tail -1 > $O/bench.json
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['drop_in']['pageable_cleared_ms'], {k: v['frac'] for k, v in d['extra'].items()})"
echo "== split 20"; AB_STEPS=20 AB_GROUP=16 AB_NS=8 timeout -k 10 200 python tools/ab.py split bunny mesh_large > $O/split20.txt 2>&1; grep -E "max over|N=1" $O/split20.txt
echo "== dist gloo 2 ranks"; timeout -k 10 300 env RTAMD_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 > $O/dist_gloo.log 2>&1; grep "^{" $O/dist_gloo.log | tail -1 > $O/dist_gloo.json; python -c "import json; d=json.load(open('$O/dist_gloo.json')); print(d['value'], d['n_gpus'], d.get('frame_check'))"
echo "== single process 0,0"; timeout -k 10 300 python bench.py --gpus 2 --single-process --devices 0,0 --steps 20 --warmup 5 > $O/sp.log 2>&1; grep "^{" $O/sp.log | tail -1 > $O/sp.json; python -c "import json; d=json.load(open('$O/sp.json')); print(d['value'], d['ms_per_step'], d.get('config'))"
echo "== done"
