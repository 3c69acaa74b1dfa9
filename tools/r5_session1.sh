# round-5 session: drop-in tests + bench, SLP / oversubscription A/B, band-order split A/B + parity
set -e
cd $(dirname $0)/..
export TMPDIR=/tmp
O=gpurun_out/r5b; mkdir -p $O
L=$PWD/triangles-sdf-cpu-raytracing_amd/lib
echo "== dropin tests"; timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_rowsplit.py -k "drop_in" > $O/dropin_tests.log 2>&1; tail -1 $O/dropin_tests.log
echo "== bench"; timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-pmc > $O/bench.json 2> $O/bench.err
echo "== band-order parity"; RTAMD_LIB=$L/var_border.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_rowsplit.py tests/test_multi.py "tests/test_gpu_parity.py::test_band_order_is_output_neutral" "tests/test_gpu_parity.py::test_row_band_tiles" "tests/test_gpu_parity.py::test_sixteen_frames_per_launch" "tests/test_fullsize.py::test_config5_row_bands_assemble_oracle_frame" -k "not no_fallback and not drop_in" > $O/border_tests.log 2>&1; tail -1 $O/border_tests.log
echo "== split A/B"; for r in 1 2; do
  for v in main border; do
    lib=""; [ $v != main ] && lib="RTAMD_LIB=$L/var_$v.so"
    echo "-- $r $v"; env $lib AB_STEPS=20 AB_GROUP=16 AB_NS=8 timeout -k 10 200 python tools/ab.py split bunny mesh_large 2>&1 | grep -E "max over|N=1"
  done
done > $O/split_ab.txt
echo "== slp A/B"; bash tools/ab_oct.sh "main main+RTAMD_PERSIST_OVERSUB=2 noslp noslp2 noslpw5" 2 "bunny octree octree_shipped grid mesh_large" > $O/slp_ab.txt 2>&1
echo "== done"
