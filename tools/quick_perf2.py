"""Quick primary/default timing of all workloads incl. stand-ins (dev tool; best of 3 x 64 frames)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))
import torch  # noqa: F401
import rtamd
from rtamd import data
from rtamd import workloads as WL

bunny = rtamd.load_mesh_from_obj(data.path("stanford-bunny.obj"))
sm = rtamd.SDFMesh(bunny)
cases = [("bunny", lambda: rtamd.BVHBuilder(bunny), 1920, 1080, bunny.vPos4f[:, 1].min()),
         ("grid65", lambda: WL.make_scene(*WL.load_input("example_grid.grid")[:2]), 1920, 1080, -1.0),
         ("grid256", lambda: rtamd.SDFGrid(*sm.grid(256)), 1920, 1080, -1.0),
         ("sdf6_4k", lambda: WL.make_scene(*WL.load_input("sdf_6.octree")[:2]), 3840, 2160, -1.0),
         ("oct8_4k", lambda: rtamd.SDFOctree(sm.octree(8)), 3840, 2160, -1.0)]
only = sys.argv[1:]
for name, mk, W, H, off in cases:
    if only and name not in only:
        continue
    s = mk()
    out = []
    for mode in ("primary", "default"):
        if mode == "primary":
            s.set_plane(None)
            P = [WL.params_for(p, W, H, rtamd.ShadingMode.Normal) for p in WL.orbit_positions(64)]
        else:
            s.set_plane(rtamd.Plane((0.0, 1.0, 0.0), float(off)))
            P = [WL.params_for(p, W, H, rtamd.ShadingMode.Lambert) for p in WL.orbit_positions(64)]
        s.bench_frames(P[:8], W, H)
        out.append(min(s.bench_frames(P, W, H)[0] for _ in range(3)))
    print(f"{name:8s} {W}x{H}  primary {out[0]:.4f}  default {out[1]:.4f} ms/frame", flush=True)
    s.close()
