# the driver's bench command, three times in a row (reproducibility of the headline)
set -o pipefail
mkdir -p gpurun_out/r3h2; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail gpurun_out/r3h2/d$i.json > gpurun_out/r3h2/b$i.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['frame_check'], d['roofline']['one_stream']['ms_per_step'])" gpurun_out/r3h2/b$i.log
done
