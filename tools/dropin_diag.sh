# drop-in phases (RTAMD_DROPIN_TRACE=1) inside the bench and tools/ab.py dropin: tools/dropin_diag.sh [outdir]
# (the switches are read only by A/B builds: first `bash tools/build_variant.sh abenv ""`)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export RTAMD_LIB=$PWD/triangles-sdf-cpu-raytracing_amd/lib/var_abenv.so
O=${1:-gpurun_out/dropin_diag}; mkdir -p $O
for r in 1 2; do
  RTAMD_DROPIN_TRACE=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-pmc > $O/bench_$r.log 2>&1
  python -c "import json; d=json.loads([l for l in open('$O/bench_$r.log') if l.startswith('{')][-1]); print('bench $r', d['drop_in'])"
  grep "^dropin" $O/bench_$r.log | tail -20
done
RTAMD_DROPIN_TRACE=1 AB_FRAMES=16 timeout -k 10 100 python tools/ab.py dropin bunny > $O/ab.log 2>&1; grep -E "^dropin|drop-in" $O/ab.log | tail -8
nproc
