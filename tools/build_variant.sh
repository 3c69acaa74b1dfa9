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
# the shipping build's flags (the Makefile's HIPFLAGS), plus RT_AB_ENV: a
# variant reads the RTAMD_* A/B switches from the environment (the shipping
# library does not, csrc/rt_host.h ab_env)
HIPF="$(make -s print-hipflags) -DRT_AB_ENV=1"
if [ "$VAR_UNIT" = bvhgpu ]; then
  /opt/rocm/bin/hipcc $HIPF $2 -c -o build/var/rt_bvhgpu_$1.o csrc/rt_bvhgpu.hip
  DEV=build/rt_device.o BVH=build/var/rt_bvhgpu_$1.o
else
  /opt/rocm/bin/hipcc $HIPF $2 -c -o build/var/rt_device_$1.o $SRC
  DEV=build/var/rt_device_$1.o BVH=build/rt_bvhgpu.o
fi
# the variant's own build id: the tree's id + its name and a hash of its
# flags and revision, so a bench line from a variant never passes for the
# shipping library's
make -s build/rt_buildid.o
BASE=$(sed -n 's/.*return "\([0-9a-f]*\)".*/\1/p' build/rt_buildid.cpp)
VH=$(printf '%s|%s|%s|%s' "$2" "$3" "$VAR_UNIT" "$HIPF" | sha256sum | cut -c1-8)
printf 'extern "C" const char *rt_build_id(void) { return "%s+%s:%s"; }\n' "$BASE" "$1" "$VH" > build/var/rt_buildid_$1.cpp
g++ -fPIC -c -o build/var/rt_buildid_$1.o build/var/rt_buildid_$1.cpp
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o lib/var_$1.so build/rt_host.o build/rt_bvhstage.o build/rt_meshops.o $DEV build/rt_sdfgen.o $BVH build/rt_multi.o build/var/rt_buildid_$1.o -lgomp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
