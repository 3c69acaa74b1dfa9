# GPU BVH builder: tests + timing for the main build and an A/B variant library ($1, optional)
O=gpurun_out/${OUT:-r3d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_bvhgpu.py -x -q --timeout 300 --timeout-method thread > $O/bvhtests.log 2>&1 || exit 1
RTAMD_BVH_TIMING=1 OMP_NUM_THREADS=16 timeout -k 10 300 python tools/bvh_time.py > $O/bvh_time.log 2>&1 || exit 1
if [ -n "$1" ]; then
  RTAMD_LIB=$1 timeout -k 10 400 python -u -m pytest tests/test_bvhgpu.py -x -q --timeout 300 --timeout-method thread > $O/bvhtests_var.log 2>&1 || exit 1
  RTAMD_LIB=$1 RTAMD_BVH_TIMING=1 OMP_NUM_THREADS=16 timeout -k 10 300 python tools/bvh_time.py > $O/bvh_time_var.log 2>&1 || exit 1
fi
tail -n 2 $O/bvhtests*.log; grep -hv amdgpu.ids $O/bvh_time*.log
