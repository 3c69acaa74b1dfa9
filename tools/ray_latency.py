"""Latency decomposition of heavy rays through the ray-batch kernel (rocprof times it)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("triangles-sdf-cpu-raytracing_amd", "oracle", "tests")]
import torch  # noqa
import cpuref
import scenes as S
from rtamd.workloads import orbit_positions

name = sys.argv[1] if len(sys.argv) > 1 else "stanford-bunny.obj"
W, H = 1920, 1080
pos = orbit_positions(64)[0]
P = S.params(name, W, H, "primary", pos)
rs = S.ref_scene(name)
rs.set_plane(False)
cost = rs.pixel_cost(P, W, H)
dirs = cpuref.primary_rays(P, W, H)
y, x = np.unravel_index(np.argmax(cost), cost.shape)
ty, tx = (y // 8) * 8, (x // 8) * 8
print(f"heaviest pixel ({y},{x}) cost {cost[y, x]}; its 8x8 tile cost max {cost[ty:ty+8, tx:tx+8].max()} "
      f"sum {cost[ty:ty+8, tx:tx+8].sum()}", flush=True)
gs = S.gpu_scene(name)
gs.set_plane(None)
o1 = np.array([pos], np.float32)
cases = {
    "1 heavy ray": (o1, dirs[y, x][None]),
    "64 copies of the heavy ray": (np.repeat(o1, 64, 0), np.repeat(dirs[y, x][None], 64, 0)),
    "its 8x8 tile (64 rays)": (np.repeat(o1, 64, 0), dirs[ty:ty+8, tx:tx+8].reshape(-1, 3)),
    "full frame as a ray batch": (np.repeat(o1, W * H, 0), dirs.reshape(-1, 3)),
}
for label, (o, d) in cases.items():
    for rep in range(3):
        gs.intersect(o, d, 0.01, 100.0)
    print("case:", label, len(o), flush=True)
