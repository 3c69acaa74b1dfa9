"""Device grid layouts (rt_scenes.h GridDev) against the oracle, bit for bit.

Grids larger than one XCD's L2 (4 MiB) are stored as 4x4x4 bricks on the
device; smaller ones keep the reference's x-major array (SDFGrid,
src/grid_raytracing.hpp:10-21). Only addresses change, so frames, hit
primitive ids (the c0 sample's REFERENCE index), t and normals must equal the
oracle's on both layouts, including sizes that are not multiples of the brick
(padding samples are never read) and non-cubic grids.
"""
import zlib

import numpy as np
import pytest

import cpuref
import rtamd

pytestmark = pytest.mark.gpu


def sdf_grid(size, seed):
    """A deterministic SDF-like field on the reference lattice: a sphere unioned
    with a torus plus a little seeded noise, sampled at 2i/(n-1)-1."""
    sx, sy, sz = size
    rng = np.random.default_rng(seed)
    x = np.linspace(-1.0, 1.0, sx)[:, None, None]
    y = np.linspace(-1.0, 1.0, sy)[None, :, None]
    z = np.linspace(-1.0, 1.0, sz)[None, None, :]
    sphere = np.sqrt((x - 0.2) ** 2 + y ** 2 + z ** 2) - 0.45
    q = np.sqrt(x ** 2 + z ** 2) - 0.55
    torus = np.sqrt(q ** 2 + (y + 0.1) ** 2) - 0.15
    v = np.minimum(sphere, torus) + 0.002 * rng.standard_normal((sx, sy, sz))
    return np.asarray(size, np.uint32), v.astype(np.float32).ravel()


SIZES = [(103, 97, 130), (128, 128, 128), (65, 200, 90), (24, 24, 24)]


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("mode", ["primary", "default"])
def test_grid_layout_frames(gpu, size, mode):
    sz, vals = sdf_grid(size, zlib.crc32(repr(size).encode()))
    assert (4 * vals.size > 4 << 20) == (size != (24, 24, 24))  # bricked except the small one
    ref_s, gpu_s = cpuref.RefScene.grid(sz, vals), rtamd.SDFGrid(sz, vals)
    sm, plane = {"primary": (0, False), "default": (1, True)}[mode]
    W, H = 200, 150
    for pos in [(0.0, 0.5, 2.5), (2.0, -0.7, -1.2), (0.3, 0.2, 0.4)]:
        vi, pi = cpuref.camera_matrices(pos, (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 45.0, W / H, 0.01, 100.0)
        ref_s.set_plane(plane, (0.0, 1.0, 0.0), -0.8)
        gpu_s.set_plane(rtamd.Plane((0.0, 1.0, 0.0), -0.8) if plane else None)
        rc, rt_, _, _ = ref_s.render(cpuref.make_params(pos, vi, pi, (2, 2, 2), sm, True, True), W, H)
        gc = np.zeros((H, W), np.uint32)
        gt = np.full((H, W), np.inf, np.float32)
        gpu_s.render(rtamd.render_params(pos, vi, pi, (2, 2, 2), sm, True, True), gc, gt, clear=True)
        assert np.isfinite(rt_).sum() > 1000, "the camera sees the surface"
        assert np.array_equal(rc, gc), f"{size} {mode} {pos}: {(rc != gc).sum()} colour px differ"
        assert np.array_equal(rt_.view(np.uint32), gt.view(np.uint32)), f"{size} {mode} {pos}: depth"


@pytest.mark.parametrize("size", SIZES[:3])
def test_grid_layout_rays(gpu, size):
    """IScene::intersect on random rays: hit, t, normal and the reference-index
    primitive id exact on the bricked layout."""
    sz, vals = sdf_grid(size, 7)
    rs, gs = cpuref.RefScene.grid(sz, vals), rtamd.SDFGrid(sz, vals)
    rng = np.random.default_rng(11)
    n = 20000
    o = rng.uniform(-2.5, 2.5, size=(n, 3)).astype(np.float32)
    d = (rng.uniform(-0.5, 0.5, size=(n, 3)) - o * 0.3).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    d = d.astype(np.float32)
    rh, rt_, rn, rp = rs.intersect_rays(o, d, 0.01, 100.0)
    g = gs.intersect(o, d, 0.01, 100.0)
    assert rh.sum() > 1000
    assert np.array_equal(rh.astype(bool), g.hitten), "hit mask differs"
    assert np.array_equal(rp, g.prim), "primitive ids differ"
    h = g.hitten
    assert np.array_equal(rt_[h].view(np.uint32), g.t[h].view(np.uint32)), "t differs"
    assert np.array_equal(rn[h].view(np.uint32), g.normal[h].view(np.uint32)), "normal differs"


def _batch_frames(gs, params, W, H):
    """Frames through rt_render_device_frames (the multi-frame block dispatch the
    bench times), read back to the host."""
    import torch
    n = len(params)
    cs = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in range(n)]
    ts = [torch.empty((H, W), dtype=torch.float32, device="cuda") for _ in range(n)]
    gs.render_device_frames(params, [c.data_ptr() for c in cs], [t.data_ptr() for t in ts], W, H, rtamd.RT_FLAG_CLEAR)
    torch.cuda.synchronize()
    return [(c.cpu().numpy().view(np.uint32), t.cpu().numpy()) for c, t in zip(cs, ts)]


@pytest.mark.parametrize("size", [(103, 97, 130), (24, 24, 24), (65, 65, 65)])
@pytest.mark.parametrize("mode", ["primary", "default"])
def test_grid_multi_frame_launches(gpu, size, mode):
    """Multi-frame launches on the bricked (103x97x130) and linear (24^3,
    65^3) layouts equal the oracle's frames bit for bit, including the default
    mode's shadow and reflection rays. (Round 4 ran this with the per-wave LDS
    block cache on and off; the cache was removed in round 5.)"""
    sz, vals = sdf_grid(size, zlib.crc32(repr(size).encode()) + 1)
    ref_s, gpu_s = cpuref.RefScene.grid(sz, vals), rtamd.SDFGrid(sz, vals)
    sm, plane = {"primary": (0, False), "default": (1, True)}[mode]
    ref_s.set_plane(plane, (0.0, 1.0, 0.0), -0.8)
    gpu_s.set_plane(rtamd.Plane((0.0, 1.0, 0.0), -0.8) if plane else None)
    W, H = 160, 120
    poses = [(0.0, 0.5, 2.5), (2.0, -0.7, -1.2), (0.3, 0.2, 0.4), (-1.1, 1.4, 1.7), (0.9, 0.0, -2.2)]
    gp, rp = [], []
    for pos in poses:
        vi, pi = cpuref.camera_matrices(pos, (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 45.0, W / H, 0.01, 100.0)
        gp.append(rtamd.render_params(pos, vi, pi, (2, 2, 2), sm, True, True))
        rp.append(cpuref.make_params(pos, vi, pi, (2, 2, 2), sm, True, True))
    refs = [ref_s.render(p, W, H)[:2] for p in rp]
    gpu_s.render(gp[0], np.zeros((H, W), np.uint32), np.full((H, W), np.inf, np.float32), clear=True)  # create
    for k, ((gc, gt), (rc, rt_)) in enumerate(zip(_batch_frames(gpu_s, gp, W, H), refs)):
        assert np.array_equal(rc, gc), f"{size} {mode} frame {k}: {(rc != gc).sum()} px differ"
        assert np.array_equal(rt_.view(np.uint32), gt.view(np.uint32)), f"{size} {mode} frame {k}: t"
