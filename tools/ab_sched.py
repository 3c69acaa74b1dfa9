"""A/B of the cost-ordered block schedule (rtx_set_schedule) on the bench workloads (dev tool)."""
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
L.rtx_set_schedule.argtypes = [C.c_void_p, C.c_int]
bunny = rtamd.load_mesh_from_obj(data.path("stanford-bunny.obj"))
sm = rtamd.SDFMesh(bunny)
cases = [("bunny", lambda: rtamd.BVHBuilder(bunny), 1920, 1080),
         ("grid65", lambda: WL.make_scene(*WL.load_input("example_grid.grid")[:2]), 1920, 1080),
         ("grid256", lambda: rtamd.SDFGrid(*sm.grid(256)), 1920, 1080),
         ("sdf6_4k", lambda: WL.make_scene(*WL.load_input("sdf_6.octree")[:2]), 3840, 2160),
         ("oct8_4k", lambda: rtamd.SDFOctree(sm.octree(8)), 3840, 2160),
         ("bunny4k", lambda: rtamd.BVHBuilder(bunny), 3840, 2160)]
modes = sys.argv[1:] or ["primary", "default"]
for name, mk, W, H in cases:
    s = mk()
    for mode in modes:
        if mode == "primary":
            s.set_plane(None)
            P = [WL.params_for(p, W, H, rtamd.ShadingMode.Normal) for p in WL.orbit_positions(64)]
        else:
            s.set_plane(rtamd.Plane((0.0, 1.0, 0.0), -1.0))
            P = [WL.params_for(p, W, H, rtamd.ShadingMode.Lambert) for p in WL.orbit_positions(64)]
        res = []
        for on in (0, 1, 0, 1):
            L.rtx_set_schedule(s._h, on)
            s.bench_frames(P[:8], W, H)
            res.append(min(s.bench_frames(P, W, H)[0] for _ in range(2)))
        print(f"{name:8s} {mode:8s} off {min(res[0], res[2]):.4f}  on {min(res[1], res[3]):.4f} ms/frame",
              flush=True)
    s.close()
