"""A/B of the mesh wave-priority knob (rtx_set_prio) on bunny 1080p / mesh_large 4K (dev tool)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))
import torch  # noqa: F401
import rtamd
from rtamd import data
from rtamd import workloads as WL

L = rtamd.lib()
L.rtx_set_prio.argtypes = [C.c_void_p, C.c_int]
bunny = rtamd.load_mesh_from_obj(data.path("stanford-bunny.obj"))
cases = [("bunny", rtamd.BVHBuilder(bunny), 1920, 1080),
         ("bunny4k", rtamd.BVHBuilder(bunny), 3840, 2160)]
for name, s, W, H in cases:
    s.set_plane(None)
    P = [WL.params_for(p, W, H, rtamd.ShadingMode.Normal) for p in WL.orbit_positions(64)]
    for it in (0, 8, 16, 32, 64, 0):
        L.rtx_set_prio(s._h, it)
        s.bench_frames(P[:5], W, H)
        best = min(s.bench_frames(P, W, H)[0] for _ in range(3))
        print(f"{name:8s} prio_iter {it:3d}: {best:.4f} ms/frame", flush=True)
