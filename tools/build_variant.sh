# build_variant.sh NAME "-DFLAGS..." [REV]
#   -> triangles-sdf-cpu-raytracing_amd/lib/var_NAME.so (A/B experiments).
# With REV (a git revision), rt_device.hip and its headers are taken from that
# revision instead of the working tree (A/B against a committed state).
# VAR_UNIT=bvhgpu: the flags apply to rt_bvhgpu.hip (the BVH builder) instead.
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
HIPF="-std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC"
if [ "$VAR_UNIT" = bvhgpu ]; then
  /opt/rocm/bin/hipcc $HIPF $2 -c -o build/var/rt_bvhgpu_$1.o csrc/rt_bvhgpu.hip
  DEV=build/rt_device.o BVH=build/var/rt_bvhgpu_$1.o
else
  /opt/rocm/bin/hipcc $HIPF $2 -c -o build/var/rt_device_$1.o $SRC
  DEV=build/var/rt_device_$1.o BVH=build/rt_bvhgpu.o
fi
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o lib/var_$1.so build/rt_host.o build/rt_bvhstage.o build/rt_meshops.o $DEV build/rt_sdfgen.o $BVH build/rt_buildid.o -lgomp
