"""Host time of each launch issued right after a device synchronisation (dev
tool): the driver's 20-frame runs issue only 2-3 launches per timed region,
so the first calls' cost is what a rank at N = 8 pays. For row-band tiles
(8 ranks) and whole frames, 16 frames per launch, two streams: per call, the
pieces of bench.run_single's issue() -- stream context + start event, the
params / pointer marshalling and rt_render_device_frames itself.
usage: python tools/issue_probe.py [workload]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import rtamd  # noqa: E402
from rtamd import _lib  # noqa: E402
from rtamd import workloads as WL  # noqa: E402
from rtamd.api import RenderParams  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
    src, W, H, mode = bench.WORKLOADS[name][:4]
    sc, _ = WL.scene_for(src)
    sc.set_plane(None)
    G, reps = 16, 6
    prm = bench.orbit_params(64, W, H)
    dev = torch.device("cuda")
    streams = bench.stream_pool(2)
    for st in streams:
        _lib.check(rtamd.lib().rt_stream_prepare(C.c_void_p(st.cuda_stream)))
    bufs = [[(torch.empty((H, W), dtype=torch.int32, device=dev), torch.empty((H, W), dtype=torch.float32, device=dev))
             for _ in range(G)] for _ in range(2)]
    L = rtamd.lib()
    # timing events as bench.run_single records them (enable_timing=True),
    # created (first record) before the probe
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
           for _ in range(reps)]
    for row in evs:
        for a, b in row:
            a.record(streams[0])
            b.record(streams[0])
    for label, tile in (("band 0 of 8", _lib.Tile(8, 0, 8, 0)), ("whole frame", None)):
        for rep in range(reps):
            torch.cuda.synchronize()
            out = []
            for j in range(3):
                st, fb = streams[j % 2], bufs[j % 2]
                p = prm[(j * G) % 48:(j * G) % 48 + G]
                ev0, ev1 = evs[rep][j]
                t0 = time.perf_counter()
                ctx = torch.cuda.stream(st)
                ctx.__enter__()
                ev0.record(st)
                t1 = time.perf_counter()
                arr = (RenderParams * G)(*p)
                cp = (C.c_void_p * G)(*[c.data_ptr() for c, _ in fb])
                tp = (C.c_void_p * G)(*[t.data_ptr() for _, t in fb])
                t2 = time.perf_counter()
                _lib.check(L.rt_render_device_frames(sc._handle(), arr, G, cp, tp, W, H, rtamd.RT_FLAG_CLEAR,
                                                     C.byref(tile) if tile is not None else None,
                                                     C.c_void_p(st.cuda_stream)))
                t3 = time.perf_counter()
                ev1.record(st)
                ctx.__exit__(None, None, None)
                t4 = time.perf_counter()
                out.append(f"call {j}: ctx+event {1e6 * (t1 - t0):.0f} + marshal {1e6 * (t2 - t1):.0f} + "
                           f"rt_render_device_frames {1e6 * (t3 - t2):.0f} + event+exit {1e6 * (t4 - t3):.0f} us")
            torch.cuda.synchronize()
            print(f"{name} {label} rep {rep}: " + "; ".join(out), flush=True)
    sc.close()


if __name__ == "__main__":
    main()
