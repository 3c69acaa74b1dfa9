"""Shared scene loading for tests: the same input arrays go to the oracle and to the GPU."""
import functools

import numpy as np

import cpuref
import rtamd
from rtamd import data

GOLDEN = {
    # word-wise FNV-1a-64 of the colour buffer, rendered by the
    # reference's unmodified hot-path TUs (camera (0,0,2.5)->0, after clear()).
    ("cube.obj", 256, 256, "primary"): "371a13d286950407",
    ("cube.obj", 256, 256, "default"): "27075cada95bb655",
    ("stanford-bunny.obj", 1920, 1080, "primary"): "8a7af01a77f18d51",
    ("stanford-bunny.obj", 1920, 1080, "default"): "6f4090c7f43ad024",
    ("stanford-bunny.obj", 3840, 2160, "primary"): "d73023ff6d3762a4",
    ("example_grid.grid", 1920, 1080, "primary"): "76d04af253e66449",
    ("example_grid.grid", 1920, 1080, "default"): "642fd2b0425b8cba",
    ("sdf_6.octree", 3840, 2160, "primary"): "b18e7e0bfc294bdf",
    ("sdf_6.octree", 3840, 2160, "default"): "5e8f335223c8b154",
}
COVERAGE = {
    ("stanford-bunny.obj", 1920, 1080, "primary"): 293614,
    ("stanford-bunny.obj", 1920, 1080, "default"): 1116188,
    ("example_grid.grid", 1920, 1080, "primary"): 505347,
    ("sdf_6.octree", 3840, 2160, "primary"): 2684413,
}

MODES = {
    # name: (shading mode, plane, shadows, reflections)
    "primary": (0, False, True, True),
    "default": (1, True, True, True),
    "lambert_noplane": (1, False, True, True),
    "lambert_noshadow": (1, True, False, True),
    "color_plane": (2, True, True, True),
    "normal_plane": (0, True, True, True),
}


@functools.lru_cache(maxsize=None)
def inputs(name):
    """-> (kind, payload, plane_offset) loaded with the ORACLE loaders (payload is
    handed unchanged to both implementations)."""
    p = data.path(name)
    if name.endswith(".obj"):
        v, i = cpuref.load_obj(p)
        bb = (v[:, :3] / v[:, 3:4]).min(0)
        return "mesh", (v, i), float(bb[1])
    if name.endswith(".grid"):
        size = np.fromfile(p, np.uint32, 3)
        vals = np.fromfile(p, np.float32, offset=12)
        return "grid", (size, vals), -1.0
    nodes = np.fromfile(p, np.uint8, offset=4)
    return "octree", nodes, -1.0


@functools.lru_cache(maxsize=None)
def ref_scene(name):
    kind, payload, _ = inputs(name)
    if kind == "mesh":
        return cpuref.RefScene.mesh(*payload)
    if kind == "grid":
        return cpuref.RefScene.grid(*payload)
    return cpuref.RefScene.octree(payload)


@functools.lru_cache(maxsize=None)
def gpu_scene(name):
    kind, payload, _ = inputs(name)
    if kind == "mesh":
        return rtamd.BVHBuilder(rtamd.SimpleMesh(*payload))
    if kind == "grid":
        return rtamd.SDFGrid(*payload)
    return rtamd.SDFOctree(payload)


def params(name, W, H, mode, pos=(0.0, 0.0, 2.5), module="ref"):
    sm, plane, sh, rf = MODES[mode]
    vi, pi = cpuref.camera_matrices(pos, (0, 0, 0), (0, 1, 0), 45.0, W / H, 0.01, 100.0)
    if module == "ref":
        return cpuref.make_params(pos, vi, pi, (2, 2, 2), sm, sh, rf)
    return rtamd.render_params(pos, vi, pi, (2, 2, 2), sm, sh, rf)


def set_planes(name, mode, *scenes):
    _, plane, _, _ = MODES[mode]
    off = inputs(name)[2]
    for s in scenes:
        if isinstance(s, cpuref.RefScene):
            s.set_plane(plane, (0, 1, 0), off)
        else:
            s.set_plane(rtamd.Plane((0.0, 1.0, 0.0), off) if plane else None)


def ref_frame(name, W, H, mode, pos=(0.0, 0.0, 2.5)):
    s = ref_scene(name)
    set_planes(name, mode, s)
    c, t, _, _ = s.render(params(name, W, H, mode, pos, "ref"), W, H)
    return c, t


def gpu_frame(name, W, H, mode, pos=(0.0, 0.0, 2.5), clear=True, color=None, t=None):
    s = gpu_scene(name)
    set_planes(name, mode, s)
    if color is None:
        color = np.zeros((H, W), np.uint32)
        t = np.full((H, W), np.inf, np.float32)
    s.render(params(name, W, H, mode, pos, "gpu"), color, t, clear=clear)
    return color, t


def edge_mesh(seed, ntri, mode):
    """test_host.py's tie-heavy triangle soups (vPos4f, one vertex per corner):
    "same" duplicate triangles (all keys tie), "grid" integer lattices (many
    equal keys), "flat" (zero-area boxes on one axis), "signed0" lattices whose
    zero coordinates are a random mix of -0.0 and +0.0, "rand" small random
    triangles."""
    rng = np.random.default_rng(seed)
    if mode == "signed0":
        g = rng.integers(-2, 3, size=(ntri, 3)).astype(np.float64)
        v = np.concatenate([g, g + [1, 0, 0], g + [0, 1, 0]], axis=1).reshape(-1, 3)
        z = (v == 0) & (rng.random(v.shape) < 0.5)
        v[z] = -0.0
        assert np.signbit(v[v == 0]).any() and (~np.signbit(v[v == 0])).any()
    elif mode == "same":
        v = np.tile(rng.normal(size=(3, 3)), (ntri, 1))
    elif mode == "grid":
        g = rng.integers(0, 6, size=(ntri, 3)).astype(np.float64)
        v = np.concatenate([g, g + [1, 0, 0], g + [0, 1, 0]], axis=1).reshape(-1, 3)
    elif mode == "flat":
        v = rng.normal(size=(ntri * 3, 3))
        v[:, 1] = 0.25
    else:
        c = rng.normal(size=(ntri, 1, 3))
        v = (c + 0.05 * rng.normal(size=(ntri, 3, 3))).reshape(-1, 3)
    return np.concatenate([v, np.ones((len(v), 1))], axis=1).astype(np.float32)
