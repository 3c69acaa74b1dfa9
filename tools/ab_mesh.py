"""A/B: single-kernel vs two-kernel (wavefront) mesh primary path, interleaved rounds."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))
import torch  # noqa
import rtamd
from rtamd import workloads as WL

L = rtamd.lib()
L.rtx_set_wavefront.argtypes = [C.c_void_p, C.c_int]
for name, W, H in [("stanford-bunny.obj", 1920, 1080), ("stanford-bunny.obj", 3840, 2160), ("spot.obj", 1920, 1080)]:
    kind, payload, off = WL.load_input(name)
    s = WL.make_scene(kind, payload)
    s.set_plane(None)
    P = [WL.params_for(p, W, H, rtamd.ShadingMode.Normal) for p in WL.orbit_positions(64)]
    res = {0: [], 1: []}
    for rnd in range(4):
        for mk in (0, 1):
            L.rtx_set_wavefront(s._h, 1 - mk)
            s.bench_frames(P[:4], W, H)
            res[mk].append(s.bench_frames(P, W, H)[0])
    print(f"{name} {W}x{H}: wavefront {min(res[0]):.4f} ms  megakernel {min(res[1]):.4f} ms", flush=True)
