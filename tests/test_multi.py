"""Single-process multi-GPU rendering through the C ABI (rt_multi_*,
include/rtamd.h): Renderer::draw (raytracing.cpp:67-102) over several devices
of one process, the frame split into row bands as the reference's draw splits
rows over OpenMP threads (raytracing.cpp:77-96), assembled on devices[0] by one
gather per frame (RCCL ncclGather, or peer copies when a device repeats).

The test box has one GPU, so slots share device 0: (0,) runs the RCCL path
with a one-rank communicator, (0, 0) / (0, 0, 0) the peer-copy path. Every
frame is compared bitwise with the single-device rt_render of the same frame
(itself oracle-exact, tests/test_gpu_parity.py) and, at least once per
configuration, with the oracle. Configs[4] at full size: test_fullsize.py."""
import numpy as np
import pytest

import cpuref
import scenes as S


def _frame(sc, P, W, H, flags_kw, init=None):
    c = np.zeros((H, W), np.uint32) if init is None else init[0].copy()
    t = np.full((H, W), np.inf, np.float32) if init is None else init[1].copy()
    sc.render(P, c, t, **flags_kw)
    return c, t


def _eq(a, b, what):
    assert np.array_equal(a[0], b[0]), f"{what}: {(a[0] != b[0]).sum()} colour px differ"
    assert np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32)), f"{what}: t differs"


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0)])
@pytest.mark.parametrize("band_rows", [8, 5])
def test_multi_matches_single_device(gpu, devices, band_rows):
    """Bunny (plane + Lambert + shadows + reflection, and primary rays) at a
    ragged size (H not a multiple of bands x slots): cleared, clear+draw and
    tPrev frames over the same caller buffers equal rt_render's."""
    rt = gpu
    name, W, H = "stanford-bunny.obj", 333, 197
    sc = S.gpu_scene(name)
    for mode in ("default", "primary"):
        S.set_planes(name, mode, sc)
        P0 = S.params(name, W, H, mode, (0.0, 0.3, 2.5), "gpu")
        P1 = S.params(name, W, H, mode, (0.8, 0.2, 2.1), "gpu")
        with rt.MultiRenderer(sc, devices, band_rows=band_rows) as mr:
            for kw in ({"cleared": True}, {"clear": True}):
                _eq(_frame(mr, P0, W, H, kw), _frame(sc, P0, W, H, kw), f"{devices} {mode} {kw}")
            # tPrev: a second draw from another camera over a kept frame (raytracing.cpp:89-94),
            # with a sentinel region the first frame did not touch
            base = _frame(sc, P0, W, H, {"clear": True})
            base[0][:20, :30] = 0x11223344
            _eq(_frame(mr, P1, W, H, {}, base), _frame(sc, P1, W, H, {}, base), f"{devices} {mode} tPrev")


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0)])
@pytest.mark.parametrize("pinned", [False, True])
def test_multi_cleared_zero_copy(gpu, devices, pinned):
    """The cleared frame (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY, the app's clear()
    + draw) takes no gather: every slot stores its bands' hits at their own rows
    straight into host memory -- the caller's pinned buffers, or the handle's
    staging frame whose stored spans the host copies. A sequence of frames
    (sizes growing and shrinking, ragged band counts, cameras with no hit,
    default and primary shading, band heights 8 and 3) equals rt_render's."""
    import ctypes as C
    rt = gpu
    L = rt.lib()
    name = "stanford-bunny.obj"
    sc = S.gpu_scene(name)
    seq = [(320, 180, "default", (0.0, 0.3, 2.5), 8), (333, 197, "primary", (0.2, 0.1, 0.9), 8),
           (200, 120, "default", (0.0, 0.0, -30.0), 8), (400, 241, "default", (1.2, 0.4, 1.9), 3),
           (333, 197, "primary", (-0.7, 0.5, 2.2), 3), (64, 7, "default", (0.1, 0.2, 2.4), 8)]
    bufs = {}
    try:
        for W, H, mode, pos, br in seq:
            if (W, H) not in bufs:
                bufs[(W, H)] = (np.zeros((H, W), np.uint32), np.full((H, W), np.inf, np.float32))
                if pinned:
                    for a in bufs[(W, H)]:
                        rt._lib.check(L.rt_host_pin(C.c_void_p(a.ctypes.data), a.nbytes))
            c, t = bufs[(W, H)]
            c[:] = 0
            t[:] = np.inf
            S.set_planes(name, mode, sc)
            P = S.params(name, W, H, mode, pos, "gpu")
            with rt.MultiRenderer(sc, devices, band_rows=br) as mr:
                mr.render(P, c, t, cleared=True)
                _eq((c, t), _frame(sc, P, W, H, {"clear": True}), f"{devices} {W}x{H} {mode} {pos} br {br}")
                # a second frame on the same handle (staging frame and spans reused)
                c[:] = 0
                t[:] = np.inf
                P2 = S.params(name, W, H, mode, (pos[0] + 0.3, pos[1], pos[2]), "gpu")
                mr.render(P2, c, t, cleared=True)
                _eq((c, t), _frame(sc, P2, W, H, {"clear": True}), f"{devices} {W}x{H} second frame")
    finally:
        if pinned:
            for c, t in bufs.values():
                L.rt_host_unpin(C.c_void_p(c.ctypes.data))
                L.rt_host_unpin(C.c_void_p(t.ctypes.data))


@pytest.mark.gpu
def test_multi_against_oracle_and_plane_changes(gpu):
    """(0, 0): the assembled frame equals the oracle's Renderer::draw, and a
    plane set on the root scene after the handle was made reaches every slot."""
    rt = gpu
    name, W, H = "stanford-bunny.obj", 320, 180
    sc = S.gpu_scene(name)
    rs = S.ref_scene(name)
    with rt.MultiRenderer(sc, (0, 0)) as mr:
        for mode in ("primary", "default"):
            S.set_planes(name, mode, sc)
            S.set_planes(name, mode, rs)
            c, t = _frame(mr, S.params(name, W, H, mode, (0.2, 0.4, 2.4), "gpu"), W, H, {"cleared": True})
            rc, rt_, _, _ = rs.render(S.params(name, W, H, mode, (0.2, 0.4, 2.4), "ref"), W, H)
            _eq((c, t), (rc, rt_), f"oracle {mode}")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["grid", "octree"])
def test_multi_sdf_scenes_device_frames(gpu, kind):
    """The SDF grid and octree through rt_multi_render_device_frames (frames
    left on devices[0], stream-ordered), 5 frames, against single-device frames."""
    import torch

    import rtamd
    name = "example_grid.grid" if kind == "grid" else "sdf_6.octree"
    W, H = 256, 160
    sc = S.gpu_scene(name)
    S.set_planes(name, "default", sc)
    poses = [(0.0, 0.5, 2.5), (1.7, 0.4, 1.6), (-2.0, 0.9, 0.5), (0.3, -0.2, 2.2), (-1.0, 1.2, -1.9)]
    P = [S.params(name, W, H, "default", p, "gpu") for p in poses]
    cs = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in P]
    ts = [torch.empty((H, W), dtype=torch.float32, device="cuda") for _ in P]
    with rtamd.MultiRenderer(sc, (0, 0, 0), band_rows=4) as mr:
        st = torch.cuda.current_stream()
        mr.render_device_frames(P, [c.data_ptr() for c in cs], [t.data_ptr() for t in ts], W, H,
                                stream=st.cuda_stream)
        torch.cuda.synchronize()
    for k, p in enumerate(P):
        ref = _frame(sc, p, W, H, {"clear": True})
        _eq((cs[k].cpu().numpy().view(np.uint32), ts[k].cpu().numpy()), ref, f"{kind} frame {k}")


@pytest.mark.gpu
def test_multi_argument_errors(gpu):
    rt = gpu
    sc = S.gpu_scene("cube.obj")
    with pytest.raises(rt.RtError, match="not visible"):
        rt.MultiRenderer(sc, (0, rt.device_count()))
    with pytest.raises(rt.RtError, match="bad arguments"):
        rt.MultiRenderer(sc, ())
    with rt.MultiRenderer(sc, (0, 0)) as mr:
        c = np.zeros((16, 16), np.uint32)
        t = np.full((16, 16), np.inf, np.float32)
        from rtamd import _lib
        import ctypes as C
        L = rt.lib()
        P = S.params("cube.obj", 16, 16, "primary", module="gpu")
        rc = L.rt_multi_render(mr._h, C.byref(P), C.c_void_p(c.ctypes.data), C.c_void_p(t.ctypes.data), 16, 16,
                               _lib.RT_FLAG_TILE_NATURAL, None)
        assert rc < 0 and b"flags" in L.rt_last_error()


def test_multi_create_without_device_fails_cleanly(rt):
    """CPU: with no HIP device the multi-GPU entry points return an error, never crash."""
    import ctypes as C
    if rt.device_count() > 0:
        pytest.skip("a device is visible")
    L = rt.lib()
    devs = (C.c_int32 * 2)(0, 0)
    h = C.c_void_p()
    assert L.rt_multi_create(None, devs, 2, 8, C.byref(h)) < 0
    assert L.rt_multi_destroy(None) == 0
