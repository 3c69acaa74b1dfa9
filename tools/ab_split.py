"""Per-rank compute of the row-split renderer, on one GPU: rank r of N renders
its 8-row bands (packed) for the bench's orbit, 8 frames per launch over 2
streams. Bounds the N-GPU strong scaling from the compute side (no exchange).
usage: python tools/ab_split.py [workload]   (bunny | grid | a file)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402,F401

import bench  # noqa: E402
import rtamd  # noqa: E402
from ab_batch import scene_for  # noqa: E402
from rtamd import _lib  # noqa: E402
from rtamd import workloads as WL  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
    group = int(os.environ.get("AB_GROUP", "8"))
    streams = int(os.environ.get("AB_STREAMS", "2"))
    rtamd.lib().rt_set_device(0)
    sc = scene_for(name)
    sc.set_plane(None)
    W, H = 1920, 1080
    orbit = WL.orbit_positions(64)
    prm = [WL.params_for(orbit[k % 64], W, H, rtamd.ShadingMode.Normal) for k in range(16 + 128)]
    base = None
    for n in (int(x) for x in os.environ.get("AB_NS", "1,2,4,8").split(",")):
        for r in sorted({0, n - 1}):
            tile = None if n == 1 else _lib.Tile(8, r, n, 0)
            wall, kms, _ = bench.run_single(sc, prm, 16, 128, W, H, inflight=streams, tile=tile, batch=group)
            ms = wall * 1e3 / 128
            base = ms if n == 1 else base
            rel = f"{base / ms:.2f}x of N=1" if base else "-"
            print(f"{name} N={n} rank {r}: {ms:.4f} ms/frame ({rel}), "
                  f"{kms:.4f} ms/launch of {group}", flush=True)


if __name__ == "__main__":
    main()
