"""Quick GPU timing of the primary-ray path on the BASELINE configs (dev tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))
import rtamd
from rtamd import workloads as WL

for name, W, H in [("stanford-bunny.obj", 1920, 1080), ("example_grid.grid", 1920, 1080),
                   ("sdf_6.octree", 3840, 2160), ("sdf_6.octree", 1920, 1080)]:
    kind, payload, off = WL.load_input(name)
    s = WL.make_scene(kind, payload)
    for mode in ("primary", "default"):
        if mode == "default":
            s.set_plane(rtamd.Plane((0.0, 1.0, 0.0), off))
            P = [WL.params_for(p, W, H, rtamd.ShadingMode.Lambert) for p in WL.orbit_positions(64)]
        else:
            s.set_plane(None)
            P = [WL.params_for(p, W, H, rtamd.ShadingMode.Normal) for p in WL.orbit_positions(64)]
        s.bench_frames(P[:5], W, H)
        mean, total = s.bench_frames(P, W, H)
        print(f"{name:22s} {W}x{H} {mode:8s} {mean:8.3f} ms/frame  {W*H/mean/1e3:9.1f} Mrays/s(primary)",
              flush=True)
