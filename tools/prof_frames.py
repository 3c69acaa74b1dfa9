"""Render orbit frames of one or more workloads back to back (profiling driver).

Run under `rocprofv3 --pmc ...` by bench.py (one process per counter pass, all
workloads in it) and by hand. Every workload issues exactly `--launches`
launches of `--group` frames on ONE stream (the bench's launch shape; counters
are per dispatch), in the order given, so a reader can map the render-kernel
dispatches to workloads by dispatch order.

--plan key:src:W:H:mode[,key:src:W:H:mode...]  (src: a shipped input file or a
stand-in key of rtamd.workloads.STANDINS; mode: primary | default).
calib:<width>:<MiB>:0:- issues one rtx_calib_read dispatch instead (the byte
calibration of the L1/L2 counters, bench.py).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))
import torch  # noqa: E402  (one HIP runtime)
import rtamd  # noqa: E402
from rtamd import workloads as WL  # noqa: E402


def frames_for(W, H, mode, n):
    orbit = WL.orbit_positions(64)
    sm = rtamd.ShadingMode.Normal if mode == "primary" else rtamd.ShadingMode.Lambert
    return [WL.params_for(orbit[k % 64], W, H, sm) for k in range(n)]


def run(src, W, H, mode, group, launches):
    s, off = WL.scene_for(src)
    s.set_plane(None if mode == "primary" else rtamd.Plane((0.0, 1.0, 0.0), off))
    P = frames_for(W, H, mode, group * launches)
    dev = torch.device("cuda")
    st = torch.cuda.current_stream()
    bufs = [(torch.empty((H, W), dtype=torch.int32, device=dev), torch.empty((H, W), dtype=torch.float32, device=dev))
            for _ in range(group)]
    rtamd.lib().rt_stream_prepare(st.cuda_stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(st)
    for j in range(launches):
        fr = P[j * group:(j + 1) * group]
        if group == 1:
            s.render_device(fr[0], bufs[0][0].data_ptr(), bufs[0][1].data_ptr(), W, H, clear=True,
                            stream=st.cuda_stream)
        else:
            s.render_device_frames(fr, [c.data_ptr() for c, _ in bufs], [t.data_ptr() for _, t in bufs], W, H,
                                   rtamd.RT_FLAG_CLEAR, stream=st.cuda_stream)
    ev[1].record(st)
    torch.cuda.synchronize()
    s.close()
    return ev[0].elapsed_time(ev[1]) / launches


def calib(width, mib=256):
    """rtx_calib_read: one read pass over `mib` MiB, `width` bytes per lane (the
    PMC calibration dispatch, kernel calib_read_kernel)."""
    import ctypes as C
    L = rtamd.lib()
    L.rtx_calib_read.argtypes = [C.c_int64, C.c_int32, C.POINTER(C.c_uint32)]
    sink = C.c_uint32(0)
    rtamd._lib.check(L.rtx_calib_read(mib << 20, width, C.byref(sink)))
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", default="bunny:stanford-bunny.obj:1920:1080:primary")
    ap.add_argument("--group", type=int, default=8)
    ap.add_argument("--launches", type=int, default=2)
    a = ap.parse_args()
    for item in a.plan.split(","):
        key, src, W, H, mode = item.split(":")
        if key == "calib":  # calib:<width>:<MiB>:0:- (one calibration dispatch)
            calib(int(src), int(W))
            print(f"calib: {W} MiB read at {src} B per lane", flush=True)
            continue
        ms = run(src, int(W), int(H), mode, a.group, a.launches)
        print(f"{key} ({src} {W}x{H} {mode}): {ms:.4f} ms per launch of {a.group} frames", flush=True)


if __name__ == "__main__":
    main()
