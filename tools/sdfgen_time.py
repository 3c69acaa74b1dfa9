"""Time the GPU mesh -> SDF generator on the config 3/4/5 stand-ins (diagnostic)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "triangles-sdf-cpu-raytracing_amd"))
import numpy as np  # noqa: E402

import rtamd  # noqa: E402
from rtamd import data  # noqa: E402

out = {}
m = rtamd.load_mesh_from_obj(data.path("stanford-bunny.obj"))
t0 = time.perf_counter()
sm = rtamd.SDFMesh(m)
out["prep_s"] = time.perf_counter() - t0
for n in (64, 128, 256):
    t0 = time.perf_counter()
    size, vals = sm.grid(n)
    out[f"grid{n}_s"] = time.perf_counter() - t0
    out[f"grid{n}_neg_frac"] = float((vals < 0).mean())
for d in (6, 7, 8):
    t0 = time.perf_counter()
    nodes = sm.octree(d)
    out[f"oct{d}_s"] = time.perf_counter() - t0
    out[f"oct{d}_nodes"] = nodes.size // 36
t0 = time.perf_counter()
big = rtamd.subdivide_mesh(m, 2)
out["subdiv2_s"] = time.perf_counter() - t0
t0 = time.perf_counter()
b = rtamd.BVHBuilder(big)
out["bvh_1M_s"] = time.perf_counter() - t0
out["bvh_1M_stats"] = b.tree_stats() if hasattr(b, "tree_stats") else None
print(json.dumps(out))
