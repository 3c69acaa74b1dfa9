# Round-6 re-sweep of the mesh tail parameters in the driver's shape (headline
# only, 20 steps), three interleaved rounds (profiles/r06/param_sweep_majority.txt).
# Build the variants first:
#   bash tools/build_variant.sh coop12 -DRT_COOP_RAYS=12; ... coop16 -DRT_COOP_RAYS=16;
#   prio8 -DRT_HEAVY_PRIO=8; prio32 -DRT_HEAVY_PRIO=32; prio0 -DRT_HEAVY_PRIO=0
L=$PWD/triangles-sdf-cpu-raytracing_amd/lib
mkdir -p gpurun_out/sweep
for r in 1 2 3; do
  for v in main coop12 coop16 prio8 prio32 prio0; do
    lib=""; [ $v != main ] && lib="RTAMD_LIB=$L/var_$v.so"
    env $lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-extra --no-drop-in --no-single-process-leg > gpurun_out/sweep/$r.$v.log 2>&1 || { echo "fail $v"; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['frame_latency']['kernel_ms_p50'] if 'frame_latency' in d else '')" gpurun_out/sweep/$r.$v.log $r $v
  done
done
