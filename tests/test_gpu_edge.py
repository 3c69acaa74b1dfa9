"""Edge cases of the frame path on the GPU, against the oracle, bit for bit.

Tiny and degenerate meshes (root leaf, duplicate and flat triangles), frame
sizes that do not fill a 16x16 tile or an 8x8 wave, very wide / tall frames,
cameras inside the model and looking straight down an axis (1/d infinite: the
exact ISPC slab path), and frames rendered with tPrev from a previous frame.
"""
import numpy as np
import pytest

import cpuref
import rtamd

pytestmark = pytest.mark.gpu


def tri_mesh(seed, ntri, mode):
    rng = np.random.default_rng(seed)
    if mode == "same":
        v = np.tile(rng.normal(size=(3, 3)) * 0.5, (ntri, 1))
    elif mode == "flat":
        v = rng.uniform(-0.8, 0.8, size=(ntri * 3, 3))
        v[:, 1] = -0.25
    elif mode == "grid":
        g = rng.integers(-3, 3, size=(ntri, 3)).astype(np.float64) * 0.25
        v = np.concatenate([g, g + [0.25, 0, 0], g + [0, 0.25, 0]], axis=1).reshape(-1, 3)
    else:
        c = rng.uniform(-0.7, 0.7, size=(ntri, 1, 3))
        v = (c + 0.15 * rng.normal(size=(ntri, 3, 3))).reshape(-1, 3)
    v4 = np.concatenate([v, np.ones((len(v), 1))], axis=1).astype(np.float32)
    return v4, np.arange(len(v), dtype=np.uint32)


def frames(ref_s, gpu_s, W, H, pos, mode, plane_y=-1.0, target=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0)):
    sm, plane = {"primary": (0, False), "default": (1, True), "color": (2, True)}[mode]
    vi, pi = cpuref.camera_matrices(pos, target, up, 45.0, W / H, 0.01, 100.0)
    ref_s.set_plane(plane, (0.0, 1.0, 0.0), plane_y)
    gpu_s.set_plane(rtamd.Plane((0.0, 1.0, 0.0), plane_y) if plane else None)
    rc, rt_, _, _ = ref_s.render(cpuref.make_params(pos, vi, pi, (2, 2, 2), sm, True, True), W, H)
    gc = np.zeros((H, W), np.uint32)
    gt = np.full((H, W), np.inf, np.float32)
    gpu_s.render(rtamd.render_params(pos, vi, pi, (2, 2, 2), sm, True, True), gc, gt, clear=True)
    return (rc, rt_), (gc, gt)


def same(a, b, what):
    (rc, rt_), (gc, gt) = a, b
    assert np.array_equal(np.isfinite(rt_), np.isfinite(gt)), f"{what}: coverage"
    assert np.array_equal(rc, gc), f"{what}: {(rc != gc).sum()} colour px differ"
    assert np.array_equal(rt_.view(np.uint32), gt.view(np.uint32)), f"{what}: depth"


@pytest.mark.parametrize("seed,ntri,mode", [(1, 1, "rand"), (2, 3, "rand"), (3, 9, "rand"), (4, 300, "rand"),
                                            (5, 64, "same"), (6, 200, "grid"), (7, 120, "flat")])
@pytest.mark.parametrize("mode_", ["primary", "default"])
def test_small_meshes(gpu, seed, ntri, mode, mode_):
    v, i = tri_mesh(seed, ntri, mode)
    ref_s, gpu_s = cpuref.RefScene.mesh(v, i), rtamd.BVHBuilder(rtamd.SimpleMesh(v, i))
    for pos in [(0.0, 0.3, 2.5), (1.7, 1.2, -1.1)]:
        same(*frames(ref_s, gpu_s, 96, 72, pos, mode_), f"{mode} n={ntri} {mode_} {pos}")


@pytest.mark.parametrize("W,H", [(1, 1), (7, 5), (17, 13), (1, 300), (1000, 3)])
@pytest.mark.parametrize("name", ["stanford-bunny.obj", "example_grid.grid", "sdf_5.octree"])
def test_odd_frame_sizes(gpu, name, W, H):
    import scenes as S
    ref_s, gpu_s = S.ref_scene(name), S.gpu_scene(name)
    for mode in ("primary", "default"):
        same(*frames(ref_s, gpu_s, W, H, (0.3, 0.2, 2.5), mode, S.inputs(name)[2]), f"{name} {W}x{H} {mode}")


@pytest.mark.parametrize("name", ["stanford-bunny.obj", "example_grid.grid", "sdf_6.octree"])
def test_axis_aligned_and_inside_cameras(gpu, name):
    """Straight down an axis (rays with d.x = d.z = 0 exactly at the centre
    pixel column: 1/d infinite), and a camera inside the model."""
    import scenes as S
    ref_s, gpu_s = S.ref_scene(name), S.gpu_scene(name)
    off = S.inputs(name)[2]
    for pos, up in [((0.0, 3.0, 0.0), (0.0, 0.0, 1.0)), ((0.0, 0.0, 3.0), (0.0, 1.0, 0.0)),
                    ((3.0, 0.0, 0.0), (0.0, 1.0, 0.0)), ((0.05, 0.1, 0.02), (0.0, 1.0, 0.0))]:
        for mode in ("primary", "default", "color"):
            same(*frames(ref_s, gpu_s, 65, 49, pos, mode, off, up=up), f"{name} {pos} {mode}")


def test_empty_and_invalid_scenes(gpu):
    with pytest.raises(rtamd.RtError):
        rtamd.BVHBuilder(rtamd.SimpleMesh(np.zeros((3, 4), np.float32), np.array([0, 1, 5], np.uint32)))
    with pytest.raises(rtamd.RtError):
        rtamd.SDFGrid(np.array([0, 4, 4], np.uint32), np.zeros(0, np.float32))


@pytest.mark.parametrize("name", ["stanford-bunny.obj", "spot.obj", "example_grid.grid", "sdf_6.octree"])
def test_random_cameras(gpu, name):
    """24 seeded random cameras per scene (radius 0.3-4, any direction, random
    up vector and shading mode), 96x64 frames: bit-exact vs the oracle."""
    import scenes as S
    rng = np.random.default_rng(sum(map(ord, name)))
    ref_s, gpu_s = S.ref_scene(name), S.gpu_scene(name)
    off = S.inputs(name)[2]
    for k in range(24):
        dirv = rng.normal(size=3)
        pos = tuple((dirv / np.linalg.norm(dirv) * rng.uniform(0.3, 4.0)).astype(np.float32).tolist())
        up = (0.0, 1.0, 0.0) if k % 3 else tuple(rng.normal(size=3).astype(np.float32).tolist())
        mode = ("primary", "default", "color")[k % 3]
        same(*frames(ref_s, gpu_s, 96, 64, pos, mode, off, up=up), f"{name} cam {k} {pos} {mode}")


@pytest.mark.parametrize("force", [0, 1, 2, 3])
def test_grid_address_paths(gpu, force):
    """Every grid_mode branch (linear / bricked layout x 32-bit buffer / 64-bit
    address loads), forced on the shipped 65^3 grid with rtx_set_grid_force:
    frames and IScene::intersect bitwise equal to the oracle's."""
    import ctypes as C

    import scenes as S
    from rtamd import _lib
    L = rtamd.lib()
    L.rtx_set_grid_force.argtypes = [C.c_int]
    name = "example_grid.grid"
    size, vals = S.inputs(name)[1]
    ref_s = S.ref_scene(name)
    _lib.check(L.rtx_set_grid_force(force))
    try:
        gpu_s = rtamd.SDFGrid(size, vals)  # created under the forced layout
        for mode in ("primary", "default"):
            same(*frames(ref_s, gpu_s, 160, 90, (0.4, 0.3, 2.4), mode), f"force {force} {mode}")
        rng = np.random.default_rng(7 + force)
        o = rng.uniform(-2.5, 2.5, (4000, 3)).astype(np.float32)
        d = rng.normal(size=(4000, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
        ref_s.set_plane(False, (0, 1, 0), 0.0)
        gpu_s.set_plane(None)
        rh, rt_, rn, rp = ref_s.intersect_rays(o, d, 0.01, 100.0)
        g = gpu_s.intersect(o, d, 0.01, 100.0)
        assert np.array_equal(rh.astype(bool), g.hitten)
        assert np.array_equal(rp, g.prim)
        h = g.hitten
        assert np.array_equal(rt_[h].view(np.uint32), g.t[h].view(np.uint32))
        assert np.array_equal(rn[h].view(np.uint32), g.normal[h].view(np.uint32))
        gpu_s.close()
    finally:
        _lib.check(L.rtx_set_grid_force(0))


@pytest.mark.parametrize("seed,ntri,mode", [(11, 2000, "grid"), (12, 3000, "rand"), (13, 1500, "same"),
                                            (14, 2500, "flat")])
def test_overlapping_meshes_random_rays(gpu, seed, ntri, mode):
    """IScene::intersect on meshes whose BVH8 boxes overlap heavily and whose
    triangles tie (axis-aligned lattice, duplicates, one plane): the traversal's
    per-frame local best, its fold on return (or at a tail-call descent) and
    the first-found tie rule must give the oracle's hit, t, normal and id."""
    v, i = tri_mesh(seed, ntri, mode)
    ref_s, gpu_s = cpuref.RefScene.mesh(v, i), rtamd.BVHBuilder(rtamd.SimpleMesh(v, i))
    rng = np.random.default_rng(seed)
    n = 30000
    o = rng.uniform(-2.0, 2.0, (n, 3)).astype(np.float32)
    inside = rng.random(n) < 0.4
    o[inside] = rng.uniform(-0.6, 0.6, (int(inside.sum()), 3)).astype(np.float32)
    d = (rng.uniform(-0.7, 0.7, (n, 3)) - o).astype(np.float32)  # mostly towards the model
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    for tn, tf in ((0.01, 100.0), (-3.0, 100.0)):
        rh, rt_, rn, rp = ref_s.intersect_rays(o, d, tn, tf)
        g = gpu_s.intersect(o, d, tn, tf)
        assert rh.sum() > n // 10
        assert np.array_equal(rh.astype(bool), g.hitten), f"{mode} tn={tn}: hit mask"
        assert np.array_equal(rp, g.prim), f"{mode} tn={tn}: primitive ids"
        h = g.hitten
        assert np.array_equal(rt_[h].view(np.uint32), g.t[h].view(np.uint32)), f"{mode} tn={tn}: t"
        assert np.array_equal(rn[h].view(np.uint32), g.normal[h].view(np.uint32)), f"{mode} tn={tn}: normal"
