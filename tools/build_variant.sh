# build_variant.sh NAME "-DFLAGS..." [REV]
#   -> triangles-sdf-cpu-raytracing_amd/lib/var_NAME.so (A/B experiments).
# With REV (a git revision), rt_device.hip and its headers are taken from that
# revision instead of the working tree (A/B against a committed state).
set -e
R=$(cd $(dirname $0)/.. && pwd)
P=$R/triangles-sdf-cpu-raytracing_amd
cd $P
mkdir -p build/var lib
SRC=csrc/rt_device.hip
if [ -n "$3" ]; then
  S=build/var/src_$1
  rm -rf $S && mkdir -p $S/include $S/p/csrc
  for f in $(git -C $R ls-tree --name-only $3 triangles-sdf-cpu-raytracing_amd/csrc/); do
    case $f in *.h|*.hip) git -C $R show $3:$f > $S/p/csrc/$(basename $f) ;; esac
  done
  git -C $R show $3:include/rtamd.h > $S/include/rtamd.h
  SRC=$S/p/csrc/rt_device.hip
fi
/opt/rocm/bin/hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC $2 -c -o build/var/rt_device_$1.o $SRC
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o lib/var_$1.so build/rt_host.o build/rt_meshops.o build/var/rt_device_$1.o build/rt_sdfgen.o build/rt_bvhgpu.o -lgomp
