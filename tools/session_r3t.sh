# banded per-XCD item order (RTAMD_QMAP=band) vs interleaved: bit-exactness + A/B;
# BVH builder: wave-scan SAH (default) vs block-scan (RTAMD_SAH=block), serial bound 256 / 512 / 1024
O=gpurun_out/r3t
mkdir -p $O
OUT=r3t bash tools/session_bvh.sh || exit 1
RTAMD_SAH=block RTAMD_BVH_TIMING=1 OMP_NUM_THREADS=16 timeout -k 10 300 python tools/bvh_time.py > $O/bvh_sahblock.log 2>&1 || exit 1
for v in ser512 ser1024; do
  RTAMD_LIB=$PWD/triangles-sdf-cpu-raytracing_amd/lib/var_$v.so timeout -k 10 300 python -u -m pytest tests/test_bvhgpu.py -x -q --timeout 200 --timeout-method thread -k "sort or edge" > $O/bvh_$v.tests.log 2>&1 || exit 1
  RTAMD_LIB=$PWD/triangles-sdf-cpu-raytracing_amd/lib/var_$v.so RTAMD_BVH_TIMING=1 OMP_NUM_THREADS=16 timeout -k 10 300 python tools/bvh_time.py > $O/bvh_$v.log 2>&1 || exit 1
done
AB_K="fullsize or persist or batched or golden" bash tools/gpu_session.sh $O ptest=RTAMD_QMAP=band || exit 1
AB_WL="bunny mesh_large sdf_6.octree" bash tools/gpu_session.sh $O ab= ab=RTAMD_QMAP=band ab= ab=RTAMD_QMAP=band || exit 1
bash tools/gpu_session.sh $O short= short=RTAMD_QMAP=band short= short=RTAMD_QMAP=band
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 tools/issue_cost.py > $O/issue.log 2>&1
