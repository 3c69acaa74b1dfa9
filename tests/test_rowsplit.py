"""Row-split rendering (rtamd.rowsplit, BASELINE north_star's multi-GPU path).

GPU, one process: every rank's bands rendered with RT_FLAG_TILE_NATURAL |
RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY into ONE cleared frame (what the p2p
exchange does over xGMI) reassemble the whole-frame render bit for bit, for
meshes, grids and octrees, primary and default shading, ragged band sizes.

GPU, two processes sharing the card (gloo signals): the full RowSplitRenderer
protocol -- IPC-mapped slots, hit-only peer stores, groups, partial last group,
slot reuse -- for both exchanges; rank 0's last frame equals a whole-frame
render.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch

import scenes as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _flags(rt):
    from rtamd import _lib
    return _lib.RT_FLAG_CLEAR | _lib.RT_FLAG_HITS_ONLY | _lib.RT_FLAG_TILE_NATURAL


@pytest.mark.parametrize("name,W,H", [("stanford-bunny.obj", 320, 180), ("example_grid.grid", 250, 131),
                                      ("sdf_6.octree", 203, 97)])
@pytest.mark.parametrize("mode", ["primary", "default"])
@pytest.mark.parametrize("world,band", [(2, 8), (3, 5), (8, 16)])
def test_natural_hits_only_bands_assemble_frame(gpu, name, W, H, mode, world, band):
    from rtamd import _lib
    rt = gpu
    dev = torch.device("cuda")
    sc = S.gpu_scene(name)
    S.set_planes(name, mode, sc)
    P = S.params(name, W, H, mode, pos=(0.4, 0.3, 2.4), module="gpu")
    full_c = torch.empty((H, W), dtype=torch.int32, device=dev)
    full_t = torch.empty((H, W), dtype=torch.float32, device=dev)
    sc.render_device(P, full_c.data_ptr(), full_t.data_ptr(), W, H, clear=True)
    c = torch.full((H, W), 12345, dtype=torch.int32, device=dev)
    t = torch.zeros((H, W), dtype=torch.float32, device=dev)
    _lib.check(rt.lib().rt_clear_device(C.c_void_p(c.data_ptr()), C.c_void_p(t.data_ptr()), W * H, None))
    torch.cuda.synchronize()
    assert int((c != 0).sum()) == 0 and bool(torch.isinf(t).all())
    for r in range(world):
        sc.render_device(P, c.data_ptr(), t.data_ptr(), W, H, clear=False, tile=rt.Tile(band, r, world, 0),
                         flags=_flags(rt))
    torch.cuda.synchronize()
    assert torch.equal(c, full_c)
    assert torch.equal(t.view(torch.int32), full_t.view(torch.int32))
    # the oracle agrees with the whole-frame render
    rc, rt_ = S.ref_frame(name, W, H, mode, pos=(0.4, 0.3, 2.4))
    assert np.array_equal(full_c.cpu().numpy().view(np.uint32), rc)
    assert np.array_equal(full_t.cpu().numpy().view(np.uint32), rt_.view(np.uint32))


@pytest.mark.parametrize("name,W,H", [("stanford-bunny.obj", 240, 136), ("example_grid.grid", 161, 90),
                                      ("sdf_6.octree", 130, 77)])
@pytest.mark.parametrize("mode", ["primary", "default"])
@pytest.mark.parametrize("tiled", [False, True])
def test_batched_frames_equal_single_frames(gpu, name, W, H, mode, tiled):
    """rt_render_device_frames (up to 8 frames per launch, blockIdx.z = frame;
    11 frames = a launch of 8 + one of 3) == one rt_render_device per frame."""
    from rtamd import _lib
    from rtamd import workloads as WL
    rt = gpu
    sc = S.gpu_scene(name)
    S.set_planes(name, mode, sc)
    sm = {"primary": rt.ShadingMode.Normal, "default": rt.ShadingMode.Lambert}[mode]
    orbit = WL.orbit_positions(64)
    prm = [WL.params_for(orbit[(7 * k) % 64], W, H, sm) for k in range(11)]
    tile = rt.Tile(8, 1, 3, 0) if tiled else None
    flags = _lib.RT_FLAG_CLEAR
    bufs = [(torch.full((H, W), 5, dtype=torch.int32, device="cuda"),
             torch.zeros((H, W), dtype=torch.float32, device="cuda")) for _ in prm]
    sc.render_device_frames(prm, [c.data_ptr() for c, _ in bufs], [t.data_ptr() for _, t in bufs], W, H, flags,
                            tile=tile)
    for k, p in enumerate(prm):
        c = torch.full((H, W), 5, dtype=torch.int32, device="cuda")
        t = torch.zeros((H, W), dtype=torch.float32, device="cuda")
        sc.render_device(p, c.data_ptr(), t.data_ptr(), W, H, clear=True, tile=tile)
        torch.cuda.synchronize()
        assert torch.equal(c, bufs[k][0]), f"frame {k}"
        assert torch.equal(t.view(torch.int32), bufs[k][1].view(torch.int32)), f"frame {k}"


@pytest.mark.parametrize("name,W,H", [("stanford-bunny.obj", 200, 120), ("example_grid.grid", 9, 7),
                                      ("sdf_6.octree", 130, 77)])
def test_batched_launches_repeat_across_streams(gpu, name, W, H):
    """The batch path's per-stream work queues: launches back to back on two
    streams (each launch's last wave resets its stream's queue for the next)
    give the same frames as one rt_render_device per frame; 9x7 has fewer
    8x8 tiles than the grid has waves."""
    from rtamd import _lib
    from rtamd import workloads as WL
    sc = S.gpu_scene(name)
    sc.set_plane(None)
    orbit = WL.orbit_positions(64)
    prm = [WL.params_for(orbit[(5 * k) % 64], W, H, gpu.ShadingMode.Normal) for k in range(8)]
    ref = []
    for p in prm:
        c = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        t = torch.zeros((H, W), dtype=torch.float32, device="cuda")
        sc.render_device(p, c.data_ptr(), t.data_ptr(), W, H, clear=True)
        ref.append((c, t))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for rep in range(6):
        st = streams[rep % 2]
        n = 8 if rep % 3 else 5
        bufs = [(torch.full((H, W), 7, dtype=torch.int32, device="cuda"),
                 torch.zeros((H, W), dtype=torch.float32, device="cuda")) for _ in range(n)]
        torch.cuda.synchronize()
        sc.render_device_frames(prm[:n], [c.data_ptr() for c, _ in bufs], [t.data_ptr() for _, t in bufs], W, H,
                                _lib.RT_FLAG_CLEAR, stream=st.cuda_stream)
        outs.append(bufs)
    torch.cuda.synchronize()
    for rep, bufs in enumerate(outs):
        for k, (c, t) in enumerate(bufs):
            assert torch.equal(c, ref[k][0]), f"launch {rep} frame {k}"
            assert torch.equal(t.view(torch.int32), ref[k][1].view(torch.int32)), f"launch {rep} frame {k}"


@pytest.mark.parametrize("name,W,H", [("stanford-bunny.obj", 240, 136), ("sdf_6.octree", 130, 77)])
@pytest.mark.parametrize("rank", [0, 1])
@pytest.mark.parametrize("natural", [False, True])
def test_two_rank_bands_take_the_work_queue(gpu, name, W, H, rank, natural):
    """Row bands with enough pixels per frame (band_takes_queue; the threshold
    is lowered here so these small frames qualify) take the persistent
    work-queue kernel in rt_render_device_frames; single-frame
    rt_render_device never does. Both must give the same pixels: batched ==
    per-frame == the untiled full frame at the band's rows (natural layout)
    or packed (RT_FLAG_TILE_NATURAL off)."""
    from rtamd import _lib
    from rtamd import workloads as WL
    rt = gpu
    sc = S.gpu_scene(name)
    sc.set_plane(None)
    orbit = WL.orbit_positions(64)
    prm = [WL.params_for(orbit[(9 * k) % 64], W, H, rt.ShadingMode.Normal) for k in range(8)]
    tile = rt.Tile(8, rank, 2, 0)
    flags = _lib.RT_FLAG_CLEAR | (_lib.RT_FLAG_TILE_NATURAL if natural else 0)
    npx = rt.lib().rt_tile_pixels(W, H, C.byref(tile))
    shape = (H, W) if natural else (npx,)
    bufs = [(torch.full(shape, 5, dtype=torch.int32, device="cuda"),
             torch.zeros(shape, dtype=torch.float32, device="cuda")) for _ in prm]
    rt.lib().rtx_set_band_queue_px(C.c_int64(1))
    try:
        sc.render_device_frames(prm, [c.data_ptr() for c, _ in bufs], [t.data_ptr() for _, t in bufs], W, H, flags,
                                tile=tile)
        torch.cuda.synchronize()
    finally:
        rt.lib().rtx_set_band_queue_px(C.c_int64(-1))
    rows = np.array([y for y in range(H) if (y // 8) % 2 == rank])
    for k, p in enumerate(prm):
        c = torch.full(shape, 5, dtype=torch.int32, device="cuda")
        t = torch.zeros(shape, dtype=torch.float32, device="cuda")
        sc.render_device(p, c.data_ptr(), t.data_ptr(), W, H, clear=True, tile=tile,
                         flags=_lib.RT_FLAG_TILE_NATURAL if natural else 0)
        fc = torch.empty((H, W), dtype=torch.int32, device="cuda")
        ft = torch.empty((H, W), dtype=torch.float32, device="cuda")
        sc.render_device(p, fc.data_ptr(), ft.data_ptr(), W, H, clear=True)
        torch.cuda.synchronize()
        assert torch.equal(c, bufs[k][0]), f"frame {k}: batched != single"
        assert torch.equal(t.view(torch.int32), bufs[k][1].view(torch.int32)), f"frame {k}: batched != single"
        bc, bt = bufs[k][0].cpu().numpy(), bufs[k][1].cpu().numpy()
        fcn, ftn = fc.cpu().numpy(), ft.cpu().numpy()
        if natural:
            assert np.array_equal(bc[rows], fcn[rows]) and np.array_equal(bt[rows].view(np.int32),
                                                                          ftn[rows].view(np.int32))
            other = np.setdiff1d(np.arange(H), rows)
            assert (bc[other] == 5).all() and (bt[other] == 0).all(), "rows of the other rank were written"
        else:
            assert np.array_equal(bc, fcn[rows].reshape(-1))
            assert np.array_equal(bt.view(np.int32), ftn[rows].reshape(-1).view(np.int32))


def test_drop_in_render_host_buffers(gpu):
    """rt_render (Renderer::draw on host buffers) with pageable and pinned
    (rt_host_pin) framebuffers: cleared frames equal the oracle's, and a
    second draw over a kept frame reads t as tPrev and writes only hits
    (raytracing.cpp:89-94), exactly as the oracle's draw over the same buffers."""
    rt = gpu
    L = rt.lib()
    name, W, H = "stanford-bunny.obj", 320, 180
    sc = S.gpu_scene(name)
    S.set_planes(name, "default", sc)
    rs = S.ref_scene(name)
    S.set_planes(name, "default", rs)
    for pinned in (False, True):
        c = np.zeros((H, W), np.uint32)
        t = np.full((H, W), np.inf, np.float32)
        if pinned:
            rt._lib.check(L.rt_host_pin(c.ctypes.data, c.nbytes))
            rt._lib.check(L.rt_host_pin(t.ctypes.data, t.nbytes))
        try:
            sc.render(S.params(name, W, H, "default", (0.0, 0.3, 2.5), "gpu"), c, t, clear=True)
            rc, rt_, _, _ = rs.render(S.params(name, W, H, "default", (0.0, 0.3, 2.5), "ref"), W, H)
            assert np.array_equal(c, rc) and np.array_equal(t.view(np.uint32), rt_.view(np.uint32))
            # second draw from another camera over the kept frame: tPrev semantics
            sc.render(S.params(name, W, H, "default", (0.7, 0.2, 2.3), "gpu"), c, t, clear=False)
            rs.render(S.params(name, W, H, "default", (0.7, 0.2, 2.3), "ref"), W, H, color=rc, t=rt_)
            assert np.array_equal(c, rc) and np.array_equal(t.view(np.uint32), rt_.view(np.uint32))
        finally:
            if pinned:
                L.rt_host_unpin(c.ctypes.data)
                L.rt_host_unpin(t.ctypes.data)


@pytest.mark.parametrize("pinned", [False, True])
def test_drop_in_partial_download(gpu, pinned):
    """rt_render copies back only the bounding box of the stored hits when the
    caller's buffers hold a cleared frame (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY)
    or a tPrev frame (no flag): every other pixel keeps the caller's value,
    exactly as Renderer::draw over the same buffers leaves it. Narrow boxes go
    as 2-D copies, wide ones as whole rows, no hit copies nothing."""
    rt = gpu
    L = rt.lib()
    name, W, H = "stanford-bunny.obj", 320, 180
    sc = S.gpu_scene(name)
    S.set_planes(name, "primary", sc)
    rs = S.ref_scene(name)
    S.set_planes(name, "primary", rs)
    c = np.zeros((H, W), np.uint32)
    t = np.full((H, W), np.inf, np.float32)
    if pinned:
        rt._lib.check(L.rt_host_pin(c.ctypes.data, c.nbytes))
        rt._lib.check(L.rt_host_pin(t.ctypes.data, t.nbytes))
    try:
        # far camera: narrow box (2-D copy); near: wide (rows); away: no hit
        for pos in ((0.0, 0.1, 3.5), (0.2, 0.1, 0.9), (0.0, 0.0, -30.0)):
            c[:] = 0
            t[:] = np.inf
            sc.render(S.params(name, W, H, "primary", pos, "gpu"), c, t, cleared=True)
            rc, rt_, _, _ = rs.render(S.params(name, W, H, "primary", pos, "ref"), W, H)
            assert np.array_equal(c, rc) and np.array_equal(t.view(np.uint32), rt_.view(np.uint32)), pos
        # tPrev over a frame holding other values everywhere (a sentinel region included)
        c[:] = 0x11223344
        t[:] = 1.5
        t[:40, :60] = np.inf
        rc, rt_ = c.copy(), t.copy()
        pos = (0.6, 0.2, 2.2)
        sc.render(S.params(name, W, H, "primary", pos, "gpu"), c, t, clear=False)
        rs.render(S.params(name, W, H, "primary", pos, "ref"), W, H, color=rc, t=rt_)
        assert np.array_equal(c, rc) and np.array_equal(t.view(np.uint32), rt_.view(np.uint32))
    finally:
        if pinned:
            L.rt_host_unpin(c.ctypes.data)
            L.rt_host_unpin(t.ctypes.data)


def test_drop_in_failure_leaves_no_copy_in_flight(gpu):
    """An rt_render that fails after queueing its uploads (injected) returns
    only after synchronising both copy streams, so pinned buffers can be
    unpinned and freed at once; the next call renders normally."""
    import ctypes as C
    rt = gpu
    L = rt.lib()
    L.rtx_render_inject_failure.argtypes = [C.c_int32]
    L.rtx_render_drain_count.restype = C.c_int64
    name, W, H = "stanford-bunny.obj", 1920, 1080
    sc = S.gpu_scene(name)
    S.set_planes(name, "primary", sc)
    c = np.zeros((H, W), np.uint32)
    t = np.full((H, W), np.inf, np.float32)
    rt._lib.check(L.rt_host_pin(c.ctypes.data, c.nbytes))
    rt._lib.check(L.rt_host_pin(t.ctypes.data, t.nbytes))
    P = S.params(name, W, H, "primary", (0.0, 0.0, 2.5), "gpu")
    try:
        L.rtx_render_inject_failure(1)
        n0 = L.rtx_render_drain_count()
        with pytest.raises(rt.RtError, match="injected"):
            sc.render(P, c, t, clear=False)  # tPrev: both uploads queued before the failure
        # the failing return synchronised both copy streams (successfully)
        assert L.rtx_render_drain_count() == n0 + 1
    finally:
        L.rtx_render_inject_failure(0)
        L.rt_host_unpin(c.ctypes.data)
        L.rt_host_unpin(t.ctypes.data)
    sc.render(P, c, t, clear=True)
    rc, rt_ = S.ref_frame(name, W, H, "primary")
    assert np.array_equal(c, rc)


@pytest.mark.parametrize("pinned", [False, True])
def test_drop_in_cleared_frames_zero_copy(gpu, pinned):
    """rt_render of a cleared frame (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY, the
    app's frameBuf.clear() + draw) stores the hits straight into HOST memory:
    into the caller's buffers when rt_host_pin pinned them, else into the
    scene's pinned staging frame, whose per-row spans of stored pixels are
    then copied to the caller and cleared again. A sequence of frames --
    cameras with narrow, wide and no hits, size changes (a taller frame
    regrows the span buffers), default and primary shading, an injected
    failure -- each equals the same frame through the device-frame path
    (RT_FLAG_CLEAR alone: every pixel written on the device and downloaded)."""
    import ctypes as C
    rt = gpu
    L = rt.lib()
    L.rtx_render_inject_failure.argtypes = [C.c_int32]
    name = "stanford-bunny.obj"
    sc = S.gpu_scene(name)
    seq = [(320, 180, "default", (0.0, 0.3, 2.5)), (320, 180, "primary", (0.0, 0.1, 3.5)),
           (320, 180, "primary", (0.2, 0.1, 0.9)), (320, 180, "default", (0.0, 0.0, -30.0)),
           (200, 120, "default", (1.2, 0.4, 1.9)), ("fail", None, None, None),
           (320, 180, "primary", (-0.7, 0.5, 2.2)), (200, 120, "default", (0.4, -0.1, 2.6)),
           (203, 61, "default", (0.1, 0.2, 2.4)), (160, 240, "primary", (0.3, 0.0, 2.0)),
           (320, 180, "default", (0.0, 0.3, 2.5))]
    bufs = {}
    try:
        for W, H, mode, pos in seq:
            if W == "fail":
                L.rtx_render_inject_failure(1)
                c, t = bufs[(320, 180)]
                with pytest.raises(rt.RtError, match="injected"):
                    sc.render(S.params(name, 320, 180, "primary", (0.0, 0.0, 2.5), "gpu"), c, t, cleared=True)
                continue
            if (W, H) not in bufs:
                bufs[(W, H)] = (np.zeros((H, W), np.uint32), np.full((H, W), np.inf, np.float32))
                if pinned:
                    for a in bufs[(W, H)]:
                        rt._lib.check(L.rt_host_pin(a.ctypes.data, a.nbytes))
            c, t = bufs[(W, H)]
            c[:] = 0
            t[:] = np.inf
            S.set_planes(name, mode, sc)
            P = S.params(name, W, H, mode, pos, "gpu")
            sc.render(P, c, t, cleared=True)
            rc = np.zeros((H, W), np.uint32)
            rt_ = np.full((H, W), np.inf, np.float32)
            sc.render(P, rc, rt_, clear=True)
            assert np.array_equal(c, rc), (W, H, mode, pos, int((c != rc).sum()))
            assert np.array_equal(t.view(np.uint32), rt_.view(np.uint32)), (W, H, mode, pos)
    finally:
        L.rtx_render_inject_failure(0)
        if pinned:
            for c, t in bufs.values():
                L.rt_host_unpin(c.ctypes.data)
                L.rt_host_unpin(t.ctypes.data)


@pytest.mark.parametrize("name", ["stanford-bunny.obj", "example_grid.grid", "sdf_6.octree"])
@pytest.mark.parametrize("pinned", [False, True])
def test_drop_in_cleared_pair_flush_layouts(gpu, pinned, name):
    """The one-frame kernel writes a cleared host frame's 16-pixel bands as
    64-byte row pieces from LDS (the pair flush) only for bands inside the
    frame with 16-byte aligned rows; every other band stores per pixel. Frames
    whose buffers start 0, 4, 8 and 12 bytes past an aligned address, widths
    that are and are not multiples of 4, and heights that end inside a band
    all equal the device-frame path bitwise (and the oracle's frame for the
    aligned case)."""
    rt = gpu
    L = rt.lib()
    sc = S.gpu_scene(name)
    S.set_planes(name, "default", sc)
    rs = S.ref_scene(name)
    S.set_planes(name, "default", rs)
    pos = (0.1, 0.2, 2.2)
    sizes = ((320, 180), (322, 181), (336, 96)) if name.endswith(".obj") else ((320, 180), (322, 181))
    for W, H in sizes:
        P = S.params(name, W, H, "default", pos, "gpu")
        rc = np.zeros((H, W), np.uint32)
        rt_ = np.full((H, W), np.inf, np.float32)
        sc.render(P, rc, rt_, clear=True)
        if (W, H) == (320, 180):
            oc, ot, _, _ = rs.render(S.params(name, W, H, "default", pos, "ref"), W, H)
            assert np.array_equal(rc, oc) and np.array_equal(rt_.view(np.uint32), ot.view(np.uint32))
        for off in (0, 1, 2, 3):  # words past a 64-byte aligned base
            rawc = np.zeros(H * W + 32, np.uint32)
            rawt = np.zeros(H * W + 32, np.float32)
            bc = (-(rawc.ctypes.data // 4)) % 16 + off
            bt = (-(rawt.ctypes.data // 4)) % 16 + off
            c = rawc[bc:bc + H * W].reshape(H, W)
            t = rawt[bt:bt + H * W].reshape(H, W)
            c[:] = 0
            t[:] = np.inf
            if pinned:
                rt._lib.check(L.rt_host_pin(c.ctypes.data, c.nbytes))
                rt._lib.check(L.rt_host_pin(t.ctypes.data, t.nbytes))
            try:
                sc.render(P, c, t, cleared=True)
            finally:
                if pinned:
                    L.rt_host_unpin(c.ctypes.data)
                    L.rt_host_unpin(t.ctypes.data)
            assert np.array_equal(c, rc), (W, H, off, int((c != rc).sum()))
            assert np.array_equal(t.view(np.uint32), rt_.view(np.uint32)), (W, H, off)


def test_hits_only_needs_clear(gpu):
    from rtamd import _lib
    sc = S.gpu_scene("cube.obj")
    sc.set_plane(None)
    P = S.params("cube.obj", 16, 16, "primary", module="gpu")
    c = torch.zeros((16, 16), dtype=torch.int32, device="cuda")
    t = torch.zeros((16, 16), dtype=torch.float32, device="cuda")
    with pytest.raises(gpu.RtError, match="HITS_ONLY"):
        sc.render_device(P, c.data_ptr(), t.data_ptr(), 16, 16, clear=False, flags=_lib.RT_FLAG_HITS_ONLY)
    with pytest.raises(gpu.RtError, match="unknown render flag"):
        sc.render_device(P, c.data_ptr(), t.data_ptr(), 16, 16, clear=True, flags=64)


def test_clear_device_ragged_sizes(gpu):
    from rtamd import _lib
    for n in (1, 3, 4, 5, 1023, 4097):
        c = torch.full((n + 8,), 7, dtype=torch.int32, device="cuda")
        t = torch.zeros((n + 8,), dtype=torch.float32, device="cuda")
        _lib.check(gpu.lib().rt_clear_device(C.c_void_p(c.data_ptr()), C.c_void_p(t.data_ptr()), n, None))
        torch.cuda.synchronize()
        assert int((c[:n] != 0).sum()) == 0 and bool(torch.isinf(t[:n]).all())
        assert bool((c[n:] == 7).all()) and bool((t[n:] == 0).all())


def test_exchange_alloc_and_ipc_handle(gpu):
    L = gpu.lib()
    p = C.c_void_p()
    assert L.rt_exchange_alloc(1 << 20, C.byref(p)) == 0 and p.value
    h = (C.c_uint8 * 64)()
    assert L.rt_ipc_get_handle(p, h) == 0
    assert any(h)
    assert L.rt_exchange_free(p) == 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, exchange, out_path):
    import sys
    sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "oracle", "triangles-sdf-cpu-raytracing_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import rtamd
    from rtamd import workloads as WL
    from rtamd.rowsplit import RowSplitRenderer
    import scenes as S
    W, H = 200, 120
    name = "stanford-bunny.obj"
    sc = S.gpu_scene(name)
    S.set_planes(name, "default", sc)
    orbit = WL.orbit_positions(64)
    prm = [WL.params_for(orbit[(5 * k) % 64], W, H, rtamd.ShadingMode.Lambert) for k in range(11)]
    rs = RowSplitRenderer(sc, W, H, band_rows=8, group=3, depth=2, exchange=exchange)
    rs.render(prm[:4])
    rs.drain()
    rs.render(prm[4:])  # 7 more: groups of 3, the last one partial
    rs.drain()
    result = "rank"
    if rank == 0:
        c = torch.empty((H, W), dtype=torch.int32, device="cuda")
        t = torch.empty((H, W), dtype=torch.float32, device="cuda")
        sc.render_device(prm[-1], c.data_ptr(), t.data_ptr(), W, H, clear=True)
        torch.cuda.synchronize()
        fc, ft = rs.last()
        ok = torch.equal(c, fc) and torch.equal(t.view(torch.int32), ft.view(torch.int32))
        nz = int((fc != 0).sum())
        result = f"{'ok' if ok else 'mismatch'} {rs.exchange} {nz}"
    dist.barrier()
    rs.close()
    if rank == 0:
        with open(out_path, "w") as f:
            f.write(result)
    dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["p2p", "gather"])
def test_rowsplit_two_ranks_one_gpu(gpu, tmp_path, exchange):
    import torch.multiprocessing as mp
    out = tmp_path / "r.txt"
    mp.start_processes(_worker, args=(2, _free_port(), exchange, str(out)), nprocs=2, join=True,
                       start_method="spawn")
    res = out.read_text().split()
    assert res[0] == "ok", res
    assert res[1] == exchange  # the IPC path did not silently fall back
    assert int(res[2]) > 1000  # a real frame (plane + bunny), not an empty one
