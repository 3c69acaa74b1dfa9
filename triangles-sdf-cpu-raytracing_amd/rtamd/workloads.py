"""Benchmark / test workloads (BASELINE.json configs).

Camera orbit (synthetic, deterministic): frame k of N looks at the origin from
pos_k = (2.5 sin(2 pi k/N), 0.5, 2.5 cos(2 pi k/N)), up (0,1,0), fovy 45,
near 0.01, far 100, light (2,2,2); ground plane at the model's bbox min y
(grid / octree: -1), as main.cpp:189 sets it.
"""
from __future__ import annotations

import math

import numpy as np

from . import api, data

DEFAULT_EYE = (0.0, 0.0, 2.5)  # main.cpp:89-91


def orbit_positions(n: int = 64, radius: float = 2.5, height: float = 0.5):
    return [(radius * math.sin(2 * math.pi * k / n), height, radius * math.cos(2 * math.pi * k / n))
            for k in range(n)]


def params_for(pos, W, H, mode=api.ShadingMode.Normal, shadows=True, reflections=True,
               light=(2.0, 2.0, 2.0)):
    vi, pi = api.camera_matrices(pos, (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 45.0, W / H, 0.01, 100.0)
    return api.render_params(pos, vi, pi, light, mode, shadows, reflections)


def load_input(name: str):
    """-> (kind, payload, plane_offset). kind in {'mesh','grid','octree'}."""
    if name.endswith(".obj"):
        m = api.load_mesh_from_obj(data.path(name), scale=True)
        return "mesh", m, float(m.vPos4f[:, 1].min() / 1.0)
    if name.endswith(".grid"):
        return "grid", api.load_sdf_grid(data.path(name)), -1.0
    if name.endswith(".octree"):
        return "octree", api.load_sdf_octree(data.path(name)), -1.0
    raise ValueError(name)


def make_scene(kind: str, payload):
    if kind == "mesh":
        return api.BVHBuilder(payload)
    if kind == "grid":
        size, vals = payload
        return api.SDFGrid(size, vals)
    return api.SDFOctree(payload)


STANDINS = {
    # BASELINE configs 3-5 name inputs missing from the reference (.MISSING_LARGE_BLOBS);
    # deterministic stand-ins generated from the shipped stanford-bunny.obj
    "grid": "stanford-bunny SDF on a 256^3 lattice, generated on the GPU "
            "(stand-in for example_grid_large.grid, BASELINE configs[2])",
    "octree": "stanford-bunny SDF octree of depth 8, generated on the GPU "
              "(stand-in for example_octree_large.octree, BASELINE configs[3])",
    "mesh_large": "stanford-bunny midpoint-subdivided twice, 1,111,216 triangles "
                  "(stand-in for MotorcycleCylinderHead.obj, BASELINE configs[4])",
}


def standin_scene(which: str):
    """The config 3-5 stand-ins (rt_sdf_mesh_* / rt_mesh_subdivide) as scenes."""
    bunny = api.load_mesh_from_obj(data.path("stanford-bunny.obj"))
    if which == "mesh_large":
        return api.BVHBuilder(api.subdivide_mesh(bunny, 2))
    sm = api.SDFMesh(bunny)
    try:
        if which == "grid":
            return api.SDFGrid(*sm.grid(256))
        if which == "octree":
            return api.SDFOctree(sm.octree(8))
    finally:
        sm.close()
    raise ValueError(which)


def scene_for(src: str):
    """-> (scene, plane offset) for a shipped input file name or a stand-in key."""
    if src in STANDINS:
        return standin_scene(src), (-1.0 if src != "mesh_large" else
                                    float(api.load_mesh_from_obj(data.path("stanford-bunny.obj"))
                                          .vPos4f[:, 1].min()))
    kind, payload, off = load_input(src)
    return make_scene(kind, payload), off
