"""How well consecutive persistent launches overlap on two streams (dev tool).

Every launch of a run of K frames (launches of `batch` frames alternating over
`streams` streams, bench.run_single's issue order) records per-wave stamps
into its own buffer (rtx_set_persist_stamps is re-pointed before each launch,
and a launch keeps the pointer it was issued with). From the stamps: each
launch's first wave start, first wave out (its queue drained), last wave end,
and the number of resident waves of all launches over time, against the
4 x 4 x 256 = 4096 wave slots of the GPU at the kernel's occupancy.
Needs the stamps build:
  bash tools/build_variant.sh stamps -DRT_PERSIST_STAMPS
  RTAMD_LIB=.../lib/var_stamps.so python tools/overlap_probe.py [workload] [frames] [streams]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rtamd  # noqa: E402
from rtamd import workloads as WL  # noqa: E402

L = rtamd.lib()
L.rtx_set_persist_stamps.argtypes = [C.c_void_p, C.c_int64]
CAP = 1 << 14


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ns = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    batch = 8
    src, W, H, mode = bench.WORKLOADS[name][:4]
    sc, _ = WL.scene_for(src)
    sc.set_plane(None)
    prm = bench.orbit_params(64, W, H)
    streams = bench.stream_pool(ns)
    for st in streams:
        rtamd._lib.check(L.rt_stream_prepare(C.c_void_p(st.cuda_stream)))
    dev = torch.device("cuda")
    bufs = [[(torch.empty((H, W), dtype=torch.int32, device=dev), torch.empty((H, W), dtype=torch.float32, device=dev))
             for _ in range(batch)] for _ in range(ns)]

    def issue(j, k, n, stamps=None):
        st = streams[j % ns]
        fb = bufs[j % ns][:n]
        rtamd._lib.check(L.rtx_set_persist_stamps(C.c_void_p(stamps.data_ptr()) if stamps is not None else None,
                                                   CAP if stamps is not None else 0))
        with torch.cuda.stream(st):
            sc.render_device_frames([prm[(k + i) % 64] for i in range(n)], [c.data_ptr() for c, _ in fb],
                                    [t.data_ptr() for _, t in fb], W, H, rtamd.RT_FLAG_CLEAR,
                                    stream=st.cuda_stream)

    for rep in range(2):
        for j, (k, n) in enumerate(bench.split_launches(0, 16, batch)):  # warm every stream
            issue(j, k, n)
        torch.cuda.synchronize()
        timed = bench.split_launches(16, K, batch)
        sb = [torch.zeros(CAP * 8, dtype=torch.int64, device=dev) for _ in timed]
        torch.cuda.synchronize()
        for j, (k, n) in enumerate(timed):
            issue(j, k, n, sb[j])
        rtamd._lib.check(L.rtx_set_persist_stamps(None, 0))
        torch.cuda.synchronize()
        S = [b.view(-1, 8).cpu().numpy() for b in sb]
        S = [s[s[:, 1] > 0] for s in S]
        t0 = min(s[:, 0].min() for s in S)
        ends = []
        print(f"== {name} {K} frames, launches {[n for _, n in timed]}, {ns} streams (rep {rep})")
        for j, s in enumerate(S):
            st, en = (s[:, 0] - t0) / 100.0, (s[:, 1] - t0) / 100.0
            ends.append(en.max())
            print(f"  launch {j} (stream {j % ns}, {timed[j][1]} frames): {len(s)} waves, first start {st.min():.1f}"
                  f" us, start p50/p90 {np.median(st):.1f}/{np.percentile(st, 90):.1f}, first out (drained) "
                  f"{en.min():.1f}, ends p50/p90 {np.median(en):.1f}/{np.percentile(en, 90):.1f}, last end "
                  f"{en.max():.1f} us")
        span = max(ends)
        # resident waves of all launches over time, 10 us bins
        edges = np.arange(0.0, span + 10.0, 10.0)
        act = np.zeros(len(edges) - 1)
        for s in S:
            st, en = (s[:, 0] - t0) / 100.0, (s[:, 1] - t0) / 100.0
            for a, b in zip(st, en):
                lo, hi = np.clip((edges[:-1], edges[1:]), a, b)
                act += np.maximum(0.0, hi - lo) / 10.0
        print(f"  span {span:.1f} us = {span / K * 1e-3:.4f} ms/frame; resident waves per 10 us bin (of 4096):")
        for i in range(0, len(act), 5):
            print("   " + " ".join(f"{edges[i + q]:6.0f}:{act[i + q]:5.0f}" for q in range(5) if i + q < len(act)))
        print(f"  mean resident waves {act.mean():.0f} = {act.mean() / 4096:.3f} of the slots")
    sc.close()


if __name__ == "__main__":
    main()
