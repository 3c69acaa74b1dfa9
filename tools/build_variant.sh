# build_variant.sh NAME "-DFLAGS..."  -> triangles-sdf-cpu-raytracing_amd/lib/var_NAME.so (A/B experiments)
set -e
P=$(dirname $0)/../triangles-sdf-cpu-raytracing_amd
cd $P
mkdir -p build/var lib
/opt/rocm/bin/hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC $2 -c -o build/var/rt_device_$1.o csrc/rt_device.hip
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o lib/var_$1.so build/rt_host.o build/rt_meshops.o build/var/rt_device_$1.o build/rt_sdfgen.o build/rt_bvhgpu.o -lgomp
