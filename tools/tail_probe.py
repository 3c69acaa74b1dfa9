"""Dev probe (not product code): how the work of the heaviest 8x8 wave tiles is
spread over their rays, from the oracle's per-pixel primary-ray work units
(cpuref_pixel_cost: node visits + leaf visits + triangle tests, the same units
the bench's byte model counts) on the bench's camera orbit at 1920x1080.

A wave runs its 64 rays in lockstep, so a tile takes about as many traversal
iterations as its heaviest ray; rays that finish early leave lanes idle. A
scheme that speeds up only the LAST k rays of a wave (the cooperative tail at
k <= 8, or evaluating a late ray's pending subtrees in parallel at k = 1-4)
can shorten a heavy tile by at most (max - kth largest) / max of its units:
the 2nd / 4th / 9th heaviest rays set the wave's time while they run.

  python tools/tail_probe.py [frames ...]   (default: orbit frames 5, 8, ..., 23)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd")]

import cpuref  # noqa: E402  (the oracle: dev tooling only)
from rtamd import data  # noqa: E402
from rtamd import workloads as WL  # noqa: E402


def main():
    frames = [int(x) for x in sys.argv[1:]] or list(range(5, 25, 3))
    v, i = cpuref.load_obj(data.path("stanford-bunny.obj"))
    rs = cpuref.RefScene.mesh(v, i)
    W, H = 1920, 1080
    orbit = WL.orbit_positions(64)
    rows = []
    for k in frames:
        vi, pi = cpuref.camera_matrices(orbit[k], aspect=W / H)
        c = rs.pixel_cost(cpuref.make_params(orbit[k], vi, pi, mode=0), W, H)
        t = c.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        s = np.sort(t, axis=1)[:, ::-1]
        for j in np.argsort(s[:, 0])[::-1][:20]:  # the 20 heaviest tiles of the frame
            rows.append((k, *(int(s[j, r]) for r in (0, 1, 3, 8, 16)), int(s[j].sum())))
        print(f"frame {k}: mean units per ray {c.mean():.2f}, heaviest ray {c.max()}, "
              f"tiles {len(t)}, mean tile max {s[:, 0].mean():.2f}")
    rows.sort(key=lambda r: -r[1])
    print("\nheaviest tiles (units of the 1st / 2nd / 4th / 9th / 17th heaviest ray, tile sum):")
    print("frame   1st  2nd  4th  9th 17th   sum")
    for r in rows[:25]:
        print("%5d %5d %4d %4d %4d %4d %6d" % r)
    a = np.array([r[1:6] for r in rows], float)
    share = lambda q: np.median((a[:, 0] - a[:, q]) / a[:, 0])  # noqa: E731
    print(f"\nover the {len(rows)} tiles (20 heaviest per frame), median of (1st - kth) / 1st, the most a "
          f"scheme that speeds up only the last k rays of the wave can take off the tile:")
    print(f"  k = 1: {share(1):.3f}   k = 3: {share(2):.3f}   k = 8: {share(3):.3f}   k = 16: {share(4):.3f}")


if __name__ == "__main__":
    main()
