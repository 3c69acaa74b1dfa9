"""The ray pump (render_pump_kernel: persistent waves with ballot/prefix-sum
active-ray compaction, the primary-ray path of rt_render_device_frames) gives
the same frames as the one-frame render_kernel and as the oracle, bit for bit:
every refill threshold, frame sizes with partial tiles and fewer pixels than
the grid has lanes, tPrev accumulation (no clear), cameras whose rays have
zero direction components (the exact slab form), and 8 frames of different
cameras mixed in one launch (lanes of one wave on different frames). The
octrees and the SDF grid (linear 65^3 and the bricked 256^3 stand-in) are
pumped."""
import numpy as np
import pytest
import torch

import scenes as S

pytestmark = pytest.mark.gpu
PUMPED = ["sdf_6.octree", "sdf_5.octree", "example_grid.grid"]


def pump(sc, on=True):
    import ctypes as C

    from rtamd import _lib
    L = _lib.lib()
    L.rtx_set_pump.argtypes = [C.c_void_p, C.c_int]
    _lib.check(L.rtx_set_pump(sc._h, int(on)))


def batch(sc, prm, W, H, clear=True, init=None):
    """rt_render_device_frames on the ray pump (switched on for this call only)."""
    from rtamd import _lib
    bufs = []
    for k in range(len(prm)):
        if init is None:
            c = torch.full((H, W), 7, dtype=torch.int32, device="cuda")
            t = torch.zeros((H, W), dtype=torch.float32, device="cuda")
        else:
            c, t = init[k][0].clone(), init[k][1].clone()
        bufs.append((c, t))
    pump(sc, True)
    try:
        sc.render_device_frames(prm, [c.data_ptr() for c, _ in bufs], [t.data_ptr() for _, t in bufs], W, H,
                                _lib.RT_FLAG_CLEAR if clear else 0)
        torch.cuda.synchronize()
    finally:
        pump(sc, False)
    return bufs


def single(sc, prm, W, H, clear=True, init=None):
    out = []
    for k, p in enumerate(prm):
        if init is None:
            c = torch.zeros((H, W), dtype=torch.int32, device="cuda")
            t = torch.zeros((H, W), dtype=torch.float32, device="cuda")
        else:
            c, t = init[k][0].clone(), init[k][1].clone()
        sc.render_device(p, c.data_ptr(), t.data_ptr(), W, H, clear=clear)
        out.append((c, t))
    torch.cuda.synchronize()
    return out


def same(a, b, what):
    for k, ((c1, t1), (c2, t2)) in enumerate(zip(a, b)):
        assert torch.equal(c1, c2), f"{what} frame {k}: {(c1 != c2).sum().item()} colour px differ"
        assert torch.equal(t1.view(torch.int32), t2.view(torch.int32)), f"{what} frame {k}: t differs"


def cams(W, H, n, seed=0, radius=2.5):
    import rtamd
    from rtamd import workloads as WL
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        th, h = rng.uniform(0, 2 * np.pi), rng.uniform(-1.5, 1.5)
        out.append(WL.params_for((radius * np.sin(th), h, radius * np.cos(th)), W, H, rtamd.ShadingMode.Normal))
    return out


@pytest.mark.parametrize("name", PUMPED)
@pytest.mark.parametrize("W,H", [(320, 180), (131, 77), (9, 7), (1, 1)])
def test_pump_equals_single_frame_path(gpu, name, W, H):
    sc = S.gpu_scene(name)
    sc.set_plane(None)
    prm = cams(W, H, 8, seed=W)
    same(batch(sc, prm, W, H), single(sc, prm, W, H), f"{name} {W}x{H}")


@pytest.mark.parametrize("name", PUMPED)
def test_pump_equals_oracle(gpu, name):
    sc = S.gpu_scene(name)
    sc.set_plane(None)
    W, H = 320, 240
    from rtamd import workloads as WL
    orbit = WL.orbit_positions(64)
    pos = [orbit[k] for k in (3, 17, 29, 44, 60)]
    prm = [WL.params_for(p, W, H, gpu.ShadingMode.Normal) for p in pos]
    got = batch(sc, prm, W, H)
    for k, p in enumerate(pos):
        rc, rt_ = S.ref_frame(name, W, H, "primary", p)
        assert np.array_equal(got[k][0].cpu().numpy().view(np.uint32), rc), f"frame {k}"
        assert np.array_equal(got[k][1].cpu().numpy().view(np.uint32), rt_.view(np.uint32)), f"frame {k}"


@pytest.mark.parametrize("name", PUMPED)
def test_pump_tprev_accumulation(gpu, name):
    """Without RT_FLAG_CLEAR every lane reads its pixel's tPrev (raytracing.cpp:89-94)."""
    sc = S.gpu_scene(name)
    sc.set_plane(None)
    W, H = 200, 150
    first = single(sc, cams(W, H, 6, seed=1), W, H)
    prm = cams(W, H, 6, seed=2, radius=2.2)
    same(batch(sc, prm, W, H, clear=False, init=first), single(sc, prm, W, H, clear=False, init=first),
         f"{name} tPrev")


@pytest.mark.parametrize("name", PUMPED)
def test_pump_axis_aligned_cameras(gpu, name):
    """Cameras on the axes: rays with zero direction components (1/d = inf) put
    the wave on the exact slab form."""
    from rtamd import workloads as WL
    sc = S.gpu_scene(name)
    sc.set_plane(None)
    W, H = 64, 64
    prm = [WL.params_for(p, W, H, gpu.ShadingMode.Normal)
           for p in [(0.0, 0.0, 2.5), (2.5, 0.0, 0.0), (0.0, 0.0, -2.0), (0.3, 0.2, 0.1)]]
    same(batch(sc, prm, W, H), single(sc, prm, W, H), f"{name} axis-aligned")


def refill(lanes):
    """The pump's refill threshold (rtx_set_refill; 0 restores the default)."""
    import ctypes as C

    from rtamd import _lib
    L = _lib.lib()
    L.rtx_set_refill.argtypes = [C.c_int32]
    _lib.check(L.rtx_set_refill(lanes))


@pytest.mark.parametrize("lanes", [1, 8, 32, 64])
def test_pump_refill_thresholds(gpu, lanes):
    """Every refill threshold gives the same frames."""
    sc = S.gpu_scene("sdf_6.octree")
    sc.set_plane(None)
    prm = cams(160, 96, 8, seed=4)
    refill(lanes)
    try:
        same(batch(sc, prm, 160, 96), single(sc, prm, 160, 96), f"refill {lanes}")
    finally:
        refill(0)


def test_pump_bricked_grid_stand_in(gpu):
    """The 256^3 stand-in (configs[2]; bricked layout, buffer loads) on the
    pump equals the one-frame path."""
    from rtamd import workloads as WL
    sc, _ = WL.scene_for("grid")
    sc.set_plane(None)
    W, H = 256, 144
    prm = cams(W, H, 8, seed=7)
    same(batch(sc, prm, W, H), single(sc, prm, W, H), "grid 256^3")


@pytest.mark.parametrize("lanes", [1, 32, 64])
def test_pump_grid_refill_thresholds(gpu, lanes):
    sc = S.gpu_scene("example_grid.grid")
    sc.set_plane(None)
    prm = cams(160, 96, 8, seed=5)
    refill(lanes)
    try:
        same(batch(sc, prm, 160, 96), single(sc, prm, 160, 96), f"grid refill {lanes}")
    finally:
        refill(0)
