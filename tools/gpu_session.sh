#!/bin/bash
# One gpurun session: GPU tests, the driver's bench command, a long bench run,
# a rocprofv3 kernel-stats pass and A/B legs. usage (on the box):
#   tools/gpu_session.sh OUT step [step ...]
# steps:
#   tests | fulltests | smoke | bench | bench128 | prof | prof_driver | split | split_large
#   dist_gloo          bench.py --gpus 2 as the driver would run it without a launcher
#                      (it spawns its 2 ranks; gloo, both on the one GPU)
#   dist_gloo_run      the same through torch.distributed.run
#   dist_rccl1         RCCL at world size 1 through the distributed path (--dist)
#   bvh                GPU BVH builder tests + build timing (tools/bvh_time.py)
#   benchw=KEY         bench.py --workload KEY (20 steps, headline only)
#   ab=VAR=a,VAR2=b    tools/ab.py batch on $AB_WL (default bunny) under those
#                      settings (RTAMD_LIB=<lib/var_x.so> selects a build variant,
#                      AB_VARIANTS the frames x streams); ab= alone: no settings
#   ptest=VAR=a,...    the GPU tests selected by -k "$AB_K" (default: all but
#                      the full-size ones) under those settings
#   short=VAR=a,...    bench.py at 20 and 128 steps (headline only) under them
#   tail=VAR=a,...     tools/persist_tail.py on $AB_WL (needs the stamps variant:
#                      bash tools/build_variant.sh stamps -DRT_PERSIST_STAMPS)
#   pmc=VAR=a,...      rocprofv3 --pmc $PMC_COUNTERS over tools/prof_frames.py
#                      --plan $PMC_PLAN (one counter pass; see bench.PMC_PASSES);
#                      counters may be joined by '+' (pmc=PMC_COUNTERS=A+B+C)
# Every GPU step runs under its own timeout; the first failure ends the session.
set -o pipefail
OUT=${1:-gpurun_out/s}; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
run() { local name=$1 secs=$2; shift 2
  echo "== $name: $*"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"; return $rc; }
n=0
for step in "$@"; do
  n=$((n + 1))
  arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
  envs=(${arg//,/ })
  tag="$n.${step%%=*}"
  case $step in
    tests) run tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" || exit 1 ;;
    fulltests) run fulltests 600 python -u -m pytest tests/test_fullsize.py -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench) run bench 900 python bench.py --gpus 1 --steps 20 --warmup 5 --detail "$OUT/bench_detail.json" && grep "^{" "$OUT/bench.log" | tail -n 1 > "$OUT/bench.json" || exit 1 ;;
    bench128) run bench128 600 python bench.py --steps 128 --warmup 16 --no-pmc --no-cpu-baseline --no-extra && grep "^{" "$OUT/bench128.log" | tail -n 1 > "$OUT/bench128.json" || exit 1 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o p -- python3 bench.py --steps 128 --warmup 16 --no-pmc --no-cpu-baseline || exit 1 ;;
    prof_driver) run prof_driver 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_driver" -o p -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --detail "$OUT/prof_driver_detail.json" || exit 1
                 grep "^{" "$OUT/prof_driver.log" | tail -n 1 > "$OUT/prof_driver.json"
                 python tools/prof_summary.py $(ls "$OUT"/prof_driver/*/p_kernel_trace.csv "$OUT"/prof_driver/p_kernel_trace.csv 2>/dev/null | head -n 1) 2 "render_persist_kernel<(anonymous namespace)::MeshS, 4, false>" 2 1 20 > "$OUT/prof_driver_phases.txt" 2>&1; cat "$OUT/prof_driver_phases.txt" ;;
    split) run split 600 python tools/ab.py split bunny || exit 1 ;;
    split_large) run split_large 600 python tools/ab.py split mesh_large || exit 1 ;;
    benchw=*) run "bench_$arg" 600 python bench.py --workload "$arg" --steps 20 --warmup 5 --no-extra \
                --no-cpu-baseline --detail "$OUT/bench_${arg}_detail.json" && grep "^{" "$OUT/bench_$arg.log" | tail -n 1 > "$OUT/bench_$arg.json" || exit 1 ;;
    dist_gloo) run dist_gloo 600 env RTAMD_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 \
                 --detail "$OUT/dist_gloo_detail.json" && grep "^{" "$OUT/dist_gloo.log" | tail -n 1 > "$OUT/dist_gloo.json" || exit 1 ;;
    bvh) run bvhtests 400 python -u -m pytest tests/test_bvhgpu.py -x -q --timeout 300 --timeout-method thread || exit 1
         run bvh_time 300 env RTAMD_BVH_TIMING=1 OMP_NUM_THREADS=16 python tools/bvh_time.py || exit 1 ;;
    dist_gloo_run) run dist_gloo_run 600 env RTAMD_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 && grep "^{" "$OUT/dist_gloo_run.log" | tail -n 1 > "$OUT/dist_gloo_run.json" || exit 1 ;;
    dist_rccl1) run dist_rccl1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --steps 20 --warmup 5 --dist && grep "^{" "$OUT/dist_rccl1.log" | tail -n 1 > "$OUT/dist_rccl1.json" || exit 1 ;;
    ab=*) echo "== $tag [$arg]"; run "$tag" 300 env "${envs[@]}" python tools/ab.py batch ${AB_WL:-bunny} || exit 1
          grep -v amdgpu "$OUT/$tag.log" ;;
    ptest=*) run "$tag" 600 env "${envs[@]}" python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${AB_K:-not fullsize}" || exit 1 ;;
    short=*) for st in 20 128; do
               run "$tag.$st" 300 env "${envs[@]}" python bench.py --steps $st --warmup 5 --no-pmc --no-cpu-baseline --no-extra || exit 1
               python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('[$arg] bench steps', sys.argv[2], d['ms_per_step'], 'ms/frame')" "$OUT/$tag.$st.log" $st
             done ;;
    tail=*) run "$tag" 300 env "${envs[@]}" python tools/persist_tail.py ${AB_WL:-bunny} || exit 1
            grep -v amdgpu "$OUT/$tag.log" ;;
    pmc=*) for e in "${envs[@]}"; do [ "${e%%=*}" = PMC_COUNTERS ] && PMC_COUNTERS=${e#*=}; done
           run "$tag" 120 env "${envs[@]}" rocprofv3 --pmc ${PMC_COUNTERS//+/ } --output-format csv -d "$OUT/$tag" -o p -- python3 tools/prof_frames.py --plan "$PMC_PLAN" || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== session done"
