"""A/B: frames per launch (batch) x launches in flight (streams) on the N=1 path.
usage: python tools/ab_batch.py [workload ...]   (workload: bunny | grid | octree | mesh_large | a file)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import rtamd  # noqa: E402
from rtamd import workloads as WL  # noqa: E402

SIZES = {"bunny": (1920, 1080), "grid": (1920, 1080), "example_grid.grid": (1920, 1080),
         "octree": (3840, 2160), "sdf_6.octree": (3840, 2160), "mesh_large": (3840, 2160)}
VARIANTS = [tuple(int(x) for x in v.split("x")) for v in
            os.environ.get("AB_VARIANTS", "1x1,1x3,2x2,4x1,4x2,8x1,8x2,8x3").split(",")]


def scene_for(name):
    if name == "bunny":
        kind, payload, _ = WL.load_input("stanford-bunny.obj")
        return WL.make_scene(kind, payload)
    if "." in name:
        kind, payload, _ = WL.load_input(name)
        return WL.make_scene(kind, payload)
    return bench.standin_scenes(name)


def main():
    names = sys.argv[1:] or ["bunny"]
    rtamd.lib().rt_set_device(0)
    for name in names:
        sc = scene_for(name)
        sc.set_plane(None)
        W, H = SIZES.get(name, (1920, 1080))
        orbit = WL.orbit_positions(64)
        prm = [WL.params_for(orbit[k % 64], W, H, rtamd.ShadingMode.Normal) for k in range(16 + 128)]
        for b, inf in VARIANTS:
            wall, kms, _ = bench.run_single(sc, prm, 16, 128, W, H, inflight=inf, batch=b)
            print(f"{name:14s} batch {b} inflight {inf}: {wall * 1e3 / 128:.4f} ms/frame, "
                  f"{kms:.4f} ms/launch, {W * H * 128 / wall / 1e6:.0f} Mrays/s", flush=True)
        sc.close()
        torch.cuda.synchronize()
        time.sleep(0.1)


if __name__ == "__main__":
    main()
