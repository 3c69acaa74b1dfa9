# Interleaved A/B of octree builds: lib/var_$A.so vs the in-tree librtamd.so
# (B), `rounds` times each, 8 x 2 and 8 x 1; output under gpurun_out/.
set -e
A=${1:-base}; ROUNDS=${2:-2}; WL=${3:-"octree octree_shipped"}
cd $(dirname $0)/..
L=triangles-sdf-cpu-raytracing_amd/lib
for r in $(seq $ROUNDS); do
  echo "== round $r: A=$A"; AB_VARIANTS=8x2,8x1 RTAMD_LIB=$PWD/$L/var_$A.so timeout -k 10 200 python tools/ab.py batch $WL
  echo "== round $r: B=librtamd"; AB_VARIANTS=8x2,8x1 timeout -k 10 200 python tools/ab.py batch $WL
done
