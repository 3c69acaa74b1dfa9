"""bench.run_single's timed issue loop replayed with switches (dev tool): which
step makes the first launch after the pre-timing synchronisation cost ~130 us
of host time (tools/ab.py split: host issue [first, second] launch).
  PROBE_GC=0      no gc.collect() / gc.disable() before the timed region
  PROBE_EVENTS=0  no timing events around the launches
  PROBE_TILE=0    whole frames instead of band 0 of 8
usage: python tools/issue_probe2.py"""
import ctypes as C
import gc
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


def flag(name, default="1"):
    return os.environ.get(name, default) == "1"


def main():
    src, W, H, _ = bench.WORKLOADS["bunny"][:4]
    sc, _ = WL.scene_for(src)
    sc.set_plane(None)
    G = 16
    tile = _lib.Tile(8, 0, 8, 0) if flag("PROBE_TILE") else None
    prm = bench.orbit_params(64, W, H)
    dev = torch.device("cuda")
    streams = bench.stream_pool(2)
    for st in streams:
        _lib.check(rtamd.lib().rt_stream_prepare(C.c_void_p(st.cuda_stream)))
    bufs = [[(torch.empty((H, W), dtype=torch.int32, device=dev), torch.empty((H, W), dtype=torch.float32, device=dev))
             for _ in range(G)] for _ in range(2)]

    def issue(j, p, ev=None):
        st, fb = streams[j % 2], bufs[j % 2][:len(p)]
        with torch.cuda.stream(st):
            if ev:
                ev[0].record(st)
            sc.render_device_frames(p, [c.data_ptr() for c, _ in fb], [t.data_ptr() for _, t in fb], W, H,
                                    rtamd.RT_FLAG_CLEAR, tile=tile, stream=st.cuda_stream)
            if ev:
                ev[1].record(st)

    for rep in range(6):
        for j in range(2):  # warm-up launches, as run_single
            issue(j, prm[j * G:(j + 1) * G])
        evs = None
        if flag("PROBE_EVENTS"):
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(2)]
            for j, (a, b) in enumerate(evs):
                a.record(streams[j % 2])
                b.record(streams[j % 2])
        if flag("PROBE_GC"):
            gc.collect()
            gc.disable()
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        issue(0, prm[32:48], evs[0] if evs else None)
        t.append(time.perf_counter())
        issue(1, prm[48:52], evs[1] if evs else None)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        gc.enable()
        print(f"rep {rep}: issue {1e6 * (t[1] - t[0]):.0f} + {1e6 * (t[2] - t[1]):.0f} us, wall "
              f"{1e6 * (t[3] - t[0]):.0f} us", flush=True)
    sc.close()


if __name__ == "__main__":
    main()
