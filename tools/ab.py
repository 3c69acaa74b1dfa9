"""One A/B driver for the render path on a single GPU (dev tool; bench.py's
launch machinery, so numbers are comparable with the bench).

  python tools/ab.py batch [workload ...]   frames per launch x streams
                                            (AB_VARIANTS="8x2,8x1,4x2")
  python tools/ab.py split [workload ...]   per-rank compute of the row-split
                                            renderer: EVERY rank r of N renders
                                            its 8-row bands (AB_NS="2,4,8"); the
                                            max over ranks bounds the N-GPU scaling;
                                            AB_STREAMS: streams per rank, default 2;
                                            AB_GROUP: frames per launch, default 8
  python tools/ab.py modes [workload ...]   primary and default shading
  python tools/ab.py dropin [workload ...]  rt_render on host buffers (bench.drop_in:
                                            pageable / pinned, AB_FRAMES frames)

workload: a key of bench.WORKLOADS (bunny, grid, grid_shipped, octree,
octree_shipped, mesh_large, default_mode: rendered in its own shading mode)
or a shipped input file. Build variants are
compared by running this under different RTAMD_LIB libraries
(tools/build_variant.sh) or RTAMD_* switches.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))

import torch  # noqa: E402,F401

import bench  # noqa: E402
import rtamd  # noqa: E402
from rtamd import _lib  # noqa: E402
from rtamd import workloads as WL  # noqa: E402

WARM, STEPS = int(os.environ.get("AB_WARM", "16")), int(os.environ.get("AB_STEPS", "128"))


def resolve(name):
    if name in bench.WORKLOADS:
        src, W, H, mode = bench.WORKLOADS[name][:4]
    else:
        src, W, H, mode = name, 1920, 1080, "primary"
    sc, off = WL.scene_for(src)
    return sc, off, W, H, mode


def timed(sc, prm, W, H, streams, group, tile=None):
    wall, launches, _ = bench.run_single(sc, prm, WARM, STEPS, W, H, inflight=streams, tile=tile, batch=group)
    return wall * 1e3 / STEPS, bench.per_frame_ms(launches) * group


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "batch"
    names = sys.argv[2:] or ["bunny"]
    rtamd.lib().rt_set_device(0)
    for name in names:
        sc, off, W, H, wmode = resolve(name)
        sc.set_plane(None if wmode == "primary" else rtamd.Plane((0.0, 1.0, 0.0), off))
        prm = bench.orbit_params(WARM + STEPS, W, H, wmode)
        if what == "batch":
            for v in os.environ.get("AB_VARIANTS", "8x2,8x1,4x2,1x1").split(","):
                g, s = (int(x) for x in v.split("x"))
                ms, kms = timed(sc, prm, W, H, s, g)
                print(f"{name} {g} frames x {s} streams: {ms:.4f} ms/frame, {kms:.4f} ms/launch", flush=True)
        elif what == "split":
            sc.set_plane(None)
            prm = bench.orbit_params(WARM + STEPS, W, H)
            group = int(os.environ.get("AB_GROUP", "8"))  # frames per launch (<= the build's RT_MAX_BATCH)
            base, _ = timed(sc, prm, W, H, 2, group)
            print(f"{name} N=1: {base:.4f} ms/frame", flush=True)
            for n in (int(x) for x in os.environ.get("AB_NS", "2,4,8").split(",")):
                per = []
                for r in range(n):
                    ms, kms = timed(sc, prm, W, H, int(os.environ.get("AB_STREAMS", "2")), group,
                                    _lib.Tile(8, r, n, 0))
                    per.append((ms, kms))
                    print(f"{name} N={n} rank {r}: {ms:.4f} ms/frame ({base / ms:.2f}x of N=1), "
                          f"{kms:.4f} ms/launch of {group}, host issue "
                          f"{bench.LAST_RUN['issue_s'] * 1e6:.0f} us {bench.LAST_RUN['issue_each_us']}", flush=True)
                worst = max(ms for ms, _ in per)
                print(f"{name} N={n}: max over ranks {worst:.4f} ms/frame -> compute-side bound "
                      f"{base / worst:.2f}x", flush=True)
        elif what == "dropin":
            d = bench.drop_in(sc, prm, W, H, frames=int(os.environ.get("AB_FRAMES", "32")))
            print(f"{name} drop-in: " + ", ".join(f"{k} {v}" for k, v in d.items() if k != "note"), flush=True)
        elif what == "modes":
            for mode in ("primary", "default"):
                sc.set_plane(None if mode == "primary" else rtamd.Plane((0.0, 1.0, 0.0), off))
                p = bench.orbit_params(WARM + STEPS, W, H, mode)
                ms, kms = timed(sc, p, W, H, 2, 8)
                print(f"{name} {mode}: {ms:.4f} ms/frame, {kms:.4f} ms/launch", flush=True)
        sc.close()


if __name__ == "__main__":
    main()
