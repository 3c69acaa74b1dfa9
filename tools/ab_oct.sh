# Interleaved A/B of builds and switches: ab_oct.sh "<variants>" <rounds> "<workloads>"
# variant "main" = the in-tree librtamd.so, any other name = lib/var_<name>.so;
# a variant may carry environment settings after '+': main+RTAMD_X=1+RTAMD_Y=2.
# 8 x 2 and 8 x 1 (AB_VARIANTS) per workload; output on stdout.
set -e
VARS=${1:-"base main"}; ROUNDS=${2:-2}; WL=${3:-"octree octree_shipped"}
cd $(dirname $0)/..
L=$PWD/triangles-sdf-cpu-raytracing_amd/lib
for r in $(seq $ROUNDS); do
  for v in $VARS; do
    echo "== round $r: $v"
    name=${v%%+*}; envs=""; [ "$name" != "$v" ] && envs=${v#*+}
    envs=${envs//+/ }
    lib=""; [ "$name" != main ] && lib="RTAMD_LIB=$L/var_$name.so"
    env $lib $envs AB_VARIANTS=${AB_VARIANTS:-8x2,8x1} timeout -k 10 200 python tools/ab.py batch $WL
  done
done
