"""Queue order of the persistent multi-frame kernel (render_persist_kernel,
PersistQ::band): frame after frame, or bands of item rows taken from every
frame in turn. The order only decides which wave traces which tile when, so
every order gives the single-frame render_kernel's frames bit for bit: band
sizes that divide the frame, that leave a partial remainder band per frame,
that exceed the frame (natural order), one-row bands, batches of 2-8 frames
and frame sizes with partial tiles. Also against the oracle on the bunny."""
import ctypes as C

import numpy as np
import pytest

import scenes as S
from test_pump import cams, same, single

pytestmark = pytest.mark.gpu
SCENES = ["stanford-bunny.obj", "sdf_6.octree"]


def set_band(rows):
    from rtamd import _lib
    L = _lib.lib()
    L.rtx_set_queue_band.argtypes = [C.c_int]
    _lib.check(L.rtx_set_queue_band(int(rows)))


def batch(sc, prm, W, H, rows):
    import torch

    from rtamd import _lib
    bufs = [(torch.full((H, W), 7, dtype=torch.int32, device="cuda"),
             torch.zeros((H, W), dtype=torch.float32, device="cuda")) for _ in prm]
    set_band(rows)
    try:
        sc.render_device_frames(prm, [c.data_ptr() for c, _ in bufs], [t.data_ptr() for _, t in bufs], W, H,
                                _lib.RT_FLAG_CLEAR)
        torch.cuda.synchronize()
    finally:
        set_band(-1)
    return bufs


@pytest.mark.parametrize("name", SCENES)
@pytest.mark.parametrize("W,H,n", [(320, 180, 8), (131, 77, 3), (640, 360, 2), (17, 9, 5)])
@pytest.mark.parametrize("rows", [0, 1, 3, 8, 1000])
def test_band_orders_equal_single_frame_path(gpu, name, W, H, n, rows):
    sc = S.gpu_scene(name)
    sc.set_plane(None)
    prm = cams(W, H, n, seed=W + rows)
    same(batch(sc, prm, W, H, rows), single(sc, prm, W, H), f"{name} {W}x{H} x{n} band {rows}")


def test_band_order_equals_oracle(gpu):
    from rtamd import workloads as WL
    name = "stanford-bunny.obj"
    sc = S.gpu_scene(name)
    sc.set_plane(None)
    W, H = 320, 240
    orbit = WL.orbit_positions(64)
    pos = [orbit[k] for k in (0, 9, 21, 33, 47, 58)]
    prm = [WL.params_for(p, W, H, gpu.ShadingMode.Normal) for p in pos]
    got = batch(sc, prm, W, H, 4)
    for k, p in enumerate(pos):
        rc, rt_ = S.ref_frame(name, W, H, "primary", p)
        assert np.array_equal(got[k][0].cpu().numpy().view(np.uint32), rc), f"frame {k}"
        assert np.array_equal(got[k][1].cpu().numpy().view(np.uint32), rt_.view(np.uint32)), f"frame {k}"
