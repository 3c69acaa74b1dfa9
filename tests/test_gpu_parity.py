"""HIP kernels vs the oracle (parity proper), through the C ABI (librtamd.so).

Bar (BASELINE.json north_star): hit coverage and hit-primitive ids bit-exact;
depth / normal / colour within 1e-5 relative fp32. The kernels reproduce the
reference arithmetic op for op, so these tests demand MORE: packed colour and
t buffers must be bitwise identical to the oracle's.
"""
import zlib

import numpy as np
import pytest

import cpuref
import scenes as S

pytestmark = pytest.mark.gpu

SMALL = [
    ("cube.obj", 256, 256),
    ("stanford-bunny.obj", 480, 270),
    ("spot.obj", 320, 240),
    ("example_grid.grid", 480, 270),
    ("sdf_5.octree", 400, 300),
    ("sdf_6.octree", 480, 270),
]
MODES = list(S.MODES)


def assert_same(ref, got, what):
    rc, rt = ref
    gc, gt = got
    assert gc.shape == rc.shape
    cov_r, cov_g = np.isfinite(rt), np.isfinite(gt)
    assert np.array_equal(cov_r, cov_g), f"{what}: coverage differs in {int((cov_r != cov_g).sum())} px"
    dc = int((rc != gc).sum())
    assert dc == 0, f"{what}: {dc} colour pixels differ"
    dt = int((rt.view(np.uint32) != gt.view(np.uint32)).sum())
    assert dt == 0, f"{what}: {dt} depth values differ bitwise"


@pytest.mark.parametrize("name,W,H", SMALL)
@pytest.mark.parametrize("mode", MODES)
def test_frame_bitexact_small(gpu, name, W, H, mode):
    pos = (0.0, 0.0, 2.5)
    ref = S.ref_frame(name, W, H, mode, pos)
    got = S.gpu_frame(name, W, H, mode, pos)
    assert_same(ref, got, f"{name} {W}x{H} {mode}")


@pytest.mark.parametrize("name,W,H", [("stanford-bunny.obj", 320, 180), ("example_grid.grid", 320, 180),
                                      ("sdf_6.octree", 320, 180)])
@pytest.mark.parametrize("k", [0, 7, 21, 40])
def test_orbit_frames(gpu, name, W, H, k):
    from rtamd.workloads import orbit_positions
    pos = orbit_positions(64)[k]
    for mode in ("primary", "default"):
        assert_same(S.ref_frame(name, W, H, mode, pos), S.gpu_frame(name, W, H, mode, pos),
                    f"{name} orbit {k} {mode}")


@pytest.mark.parametrize("key", sorted(S.GOLDEN))
def test_golden_hash_full_res(gpu, key):
    """Full BASELINE resolutions: the GPU frame hashes to the reference's golden value."""
    name, W, H, mode = key
    c, t = S.gpu_frame(name, W, H, mode)
    assert cpuref.fnv1a64_words(c) == S.GOLDEN[key]
    if key in S.COVERAGE:
        assert int(np.isfinite(t).sum()) == S.COVERAGE[key]


@pytest.mark.parametrize("name", ["stanford-bunny.obj", "example_grid.grid", "sdf_6.octree"])
def test_tprev_accumulation(gpu, name):
    """Without clear(), t is read as tPrev and pixels are overwritten only on hit
    (raytracing.cpp:89-94): render two cameras into the same framebuffer."""
    W, H = 320, 180
    rs = S.ref_scene(name)
    S.set_planes(name, "default", rs)
    rc = np.zeros((H, W), np.uint32)
    rt_ = np.full((H, W), np.inf, np.float32)
    gc = rc.copy()
    gt = rt_.copy()
    for pos in [(0.0, 0.0, 2.5), (0.7, 0.4, 2.2)]:
        rs.render(S.params(name, W, H, "default", pos, "ref"), W, H, rc, rt_)
        S.gpu_frame(name, W, H, "default", pos, clear=False, color=gc, t=gt)
    assert_same((rc, rt_), (gc, gt), f"{name} tPrev")


def _random_rays(n, seed, inside_frac=0.5):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-3, 3, (n, 3)).astype(np.float32)
    m = rng.random(n) < inside_frac
    o[m] = rng.uniform(-0.9, 0.9, (int(m.sum()), 3)).astype(np.float32)  # inside the model box
    d = rng.normal(size=(n, 3)).astype(np.float32)
    # axis-aligned directions (1/d = +-inf slabs) and exact zeros
    k = n // 8
    axis = rng.integers(0, 3, k)
    d[:k] = 0.0
    d[np.arange(k), axis] = rng.choice([-1.0, 1.0], k).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    return o, d.astype(np.float32)


@pytest.mark.parametrize("name", ["cube.obj", "stanford-bunny.obj", "spot.obj", "example_grid.grid",
                                  "sdf_5.octree", "sdf_6.octree"])
@pytest.mark.parametrize("plane", [False, True])
@pytest.mark.parametrize("tn,tf", [(0.01, 100.0), (-5.0, 100.0), (0.5, 2.0)])
def test_intersect_rays(gpu, name, plane, tn, tf):
    """IScene::intersect on random rays (origins inside the model box too, where
    BVH leaf hits may have negative t): hit, t, normal and primitive id exact."""
    o, d = _random_rays(20000, zlib.crc32(f"{name}{plane}{tn}".encode()))
    rs, gs = S.ref_scene(name), S.gpu_scene(name)
    off = S.inputs(name)[2]
    rs.set_plane(plane, (0, 1, 0), off)
    gs.set_plane(__import__("rtamd").Plane((0.0, 1.0, 0.0), off) if plane else None)
    rh, rt_, rn, rp = rs.intersect_rays(o, d, tn, tf)
    g = gs.intersect(o, d, tn, tf)
    assert np.array_equal(rh.astype(bool), g.hitten), "hit mask differs"
    assert np.array_equal(rp, g.prim), "primitive ids differ"
    h = g.hitten
    assert np.array_equal(rt_[h].view(np.uint32), g.t[h].view(np.uint32)), "t differs"
    assert np.array_equal(rn[h].view(np.uint32), g.normal[h].view(np.uint32)), "normal differs"


def _centre_plane_rays(seed):
    """Rays between dyadic points (exact in float32, d unnormalised): aimed at
    octree box corners, centres, edge and face midpoints at depths 0-6, from
    dyadic origins, many of them on centre planes. Their centre-plane
    distances tie (a ray through a centre edge or point) or tie with the entry,
    the cases where oct_expand must take the exact slab + sort8 path."""
    rng = np.random.default_rng(seed)
    n = 20000
    depth = rng.integers(0, 7, n)
    s = np.ldexp(2.0, -depth)                       # node size 2^(1-k)
    cells = np.ldexp(1.0, depth).astype(np.int64)    # 2^k cells per axis
    idx = rng.integers(0, cells[:, None], (n, 3))
    frac = rng.choice([0.0, 0.5, 1.0], (n, 3), p=[0.25, 0.5, 0.25])
    tgt = -1.0 + (idx + frac) * s[:, None]
    o = rng.choice(np.arange(-12, 13) / 4.0, (n, 3))
    far = rng.random(n) < 0.7                        # most origins outside the [-1, 1] box
    o[far] = o[far] * 2.0 + np.sign(o[far] + 0.125) * 1.5
    d = tgt - o
    d[np.all(d == 0, axis=1)] = (0.25, -0.5, 1.0)
    return o.astype(np.float32), d.astype(np.float32)


@pytest.mark.parametrize("name", ["sdf_5.octree", "sdf_6.octree"])
@pytest.mark.parametrize("tn,tf", [(0.01, 100.0), (-5.0, 100.0)])
def test_octree_centre_plane_rays(gpu, name, tn, tf):
    """SDFOctree::intersect on rays whose slab distances tie at node centres
    (crossing-order path vs sort8 fallback in oct_expand): hit, t, normal and
    node id exact."""
    o, d = _centre_plane_rays(zlib.crc32(f"{name}{tn}".encode()))
    rs, gs = S.ref_scene(name), S.gpu_scene(name)
    rs.set_plane(False, (0, 1, 0), 0.0)
    gs.set_plane(None)
    rh, rt_, rn, rp = rs.intersect_rays(o, d, tn, tf)
    g = gs.intersect(o, d, tn, tf)
    assert rh.sum() > 1000, "too few hits to be a test"
    assert np.array_equal(rh.astype(bool), g.hitten), "hit mask differs"
    assert np.array_equal(rp, g.prim), "node ids differ"
    h = g.hitten
    assert np.array_equal(rt_[h].view(np.uint32), g.t[h].view(np.uint32)), "t differs"
    assert np.array_equal(rn[h].view(np.uint32), g.normal[h].view(np.uint32)), "normal differs"


@pytest.mark.parametrize("nranks,band", [(2, 16), (3, 7), (8, 16), (5, 1000)])
def test_row_band_tiles(gpu, nranks, band):
    """Row-band tiling (multi-GPU split): every rank's packed bands, untiled on the
    device, reassemble the single-GPU frame bit for bit."""
    import ctypes as C

    import rtamd
    from rtamd._lib import check, lib
    torch = pytest.importorskip("torch")
    name, W, H = "stanford-bunny.obj", 640, 360
    s = S.gpu_scene(name)
    S.set_planes(name, "default", s)
    P = S.params(name, W, H, "default", module="gpu")
    full_c = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    full_t = torch.zeros((H, W), dtype=torch.float32, device="cuda")
    s.render_device(P, full_c.data_ptr(), full_t.data_ptr(), W, H, clear=True)
    per = max(lib().rt_tile_pixels(W, H, C.byref(rtamd.Tile(band, r, nranks, 0))) for r in range(nranks))
    pc = torch.zeros((nranks, per), dtype=torch.int32, device="cuda")
    pt = torch.zeros((nranks, per), dtype=torch.float32, device="cuda")
    for r in range(nranks):
        tile = rtamd.Tile(band, r, nranks, 0)
        s.render_device(P, pc[r].data_ptr(), pt[r].data_ptr(), W, H, clear=True, tile=tile)
    out_c = torch.zeros_like(full_c)
    out_t = torch.zeros_like(full_t)
    check(lib().rt_untile_device(C.c_void_p(pc.data_ptr()), C.c_void_p(pt.data_ptr()), per,
                                 C.c_void_p(out_c.data_ptr()), C.c_void_p(out_t.data_ptr()), W, H,
                                 C.byref(rtamd.Tile(band, 0, nranks, 0)), None))
    torch.cuda.synchronize()
    assert torch.equal(out_c, full_c)
    assert torch.equal(out_t.view(torch.int32), full_t.view(torch.int32))
    # and the full frame equals the oracle
    rc, rt_ = S.ref_frame(name, W, H, "default")
    assert np.array_equal(full_c.cpu().numpy().view(np.uint32), rc)


def test_no_fallback_library_loaded(gpu):
    """The HIP library is the code path: its kernels ran on the device."""
    import os

    import rtamd
    # an A/B run under RTAMD_LIB (a build variant, tools/build_variant.sh) loads that library
    want = os.path.basename(os.environ.get("RTAMD_LIB") or "librtamd.so")
    assert rtamd.lib()._name.endswith(want)
    assert rtamd.device_count() >= 1
    if not os.environ.get("RTAMD_LIB"):  # the shipped binary was built from this tree's sources
        assert rtamd.lib().rt_build_id().decode() == rtamd._lib.source_build_id()


def test_golden_fixture_frames(gpu):
    """GPU frames equal the committed oracle fixtures (tests/golden/frames.npz)."""
    import importlib.util
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(here, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    data = np.load(os.path.join(here, "frames.npz"))
    index = json.load(open(os.path.join(here, "frames.json")))
    for case, ent in zip(mg.CASES, index):
        name, W, H, mode, pos = case
        c, t = S.gpu_frame(name, W, H, mode, pos)
        assert_same((data[ent["color"]], data[ent["t"]]), (c, t), ent["case"])


def test_schedule_state_is_output_neutral(gpu):
    """The cost-ordered block schedule (per-scene state carried from frame to
    frame) never changes the image: frames rendered while alternating frame
    sizes, row-band tiles, two HIP streams and the schedule switch equal the
    oracle / each other bit for bit."""
    import ctypes as C

    import rtamd
    from rtamd._lib import lib
    torch = pytest.importorskip("torch")
    from rtamd.workloads import orbit_positions
    L = lib()
    L.rtx_set_schedule.argtypes = [C.c_void_p, C.c_int]
    name = "stanford-bunny.obj"
    s = S.gpu_scene(name)
    S.set_planes(name, "primary", s)
    sizes = [(320, 180), (256, 256), (320, 180)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = {}
    for rep in range(2):
        L.rtx_set_schedule(s._h, rep)  # rep 0: off, rep 1: on (state reused across frames)
        for k, pos in enumerate(orbit_positions(64)[:6]):
            W, H = sizes[k % 3]
            P = S.params(name, W, H, "primary", pos, module="gpu")
            c = torch.zeros((H, W), dtype=torch.int32, device="cuda")
            t = torch.zeros((H, W), dtype=torch.float32, device="cuda")
            st = streams[k % 2]
            with torch.cuda.stream(st):
                s.render_device(P, c.data_ptr(), t.data_ptr(), W, H, clear=True, stream=st.cuda_stream)
                if k % 2 == 1:  # a row-band tile frame in between, on the same scene
                    tile = rtamd.Tile(16, 1, 3, 0)
                    n = L.rt_tile_pixels(W, H, C.byref(tile))
                    pc = torch.zeros(n, dtype=torch.int32, device="cuda")
                    pt = torch.zeros(n, dtype=torch.float32, device="cuda")
                    s.render_device(P, pc.data_ptr(), pt.data_ptr(), W, H, clear=True, tile=tile,
                                    stream=st.cuda_stream)
            torch.cuda.synchronize()
            outs[(rep, k)] = (c.cpu().numpy().view(np.uint32), t.cpu().numpy())
    L.rtx_set_schedule(s._h, 1)
    for k, pos in enumerate(orbit_positions(64)[:6]):
        W, H = sizes[k % 3]
        for rep in range(2):
            assert np.array_equal(outs[(rep, k)][0], outs[(0, k)][0])
        if k < 3:
            assert_same(S.ref_frame(name, W, H, "primary", pos), outs[(1, k)], f"schedule frame {k}")


def test_sixteen_frames_per_launch(gpu):
    """16 frames in ONE rt_render_device_frames launch (the multi-GPU ranks'
    launch size): whole frames through the persistent kernel and one rank's
    packed row bands through the block dispatch equal the frames rendered
    one at a time, bit for bit (and the first whole frames equal the oracle)."""
    import ctypes as C

    import rtamd
    from rtamd._lib import lib
    torch = pytest.importorskip("torch")
    from rtamd.workloads import orbit_positions
    L = lib()
    name = "stanford-bunny.obj"
    s = S.gpu_scene(name)
    S.set_planes(name, "primary", s)
    W, H, n = 320, 180, 16
    pos = orbit_positions(64)[:n]
    P = [S.params(name, W, H, "primary", p, module="gpu") for p in pos]
    single = []
    for prm in P:
        c = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        t = torch.zeros((H, W), dtype=torch.float32, device="cuda")
        s.render_device(prm, c.data_ptr(), t.data_ptr(), W, H, clear=True)
        torch.cuda.synchronize()
        single.append((c.cpu().numpy().view(np.uint32), t.cpu().numpy().view(np.uint32)))
    cs = [torch.zeros((H, W), dtype=torch.int32, device="cuda") for _ in P]
    ts = [torch.zeros((H, W), dtype=torch.float32, device="cuda") for _ in P]
    s.render_device_frames(P, [c.data_ptr() for c in cs], [t.data_ptr() for t in ts], W, H, rtamd.RT_FLAG_CLEAR)
    torch.cuda.synchronize()
    for k in range(n):
        assert np.array_equal(cs[k].cpu().numpy().view(np.uint32), single[k][0]), k
        assert np.array_equal(ts[k].cpu().numpy().view(np.uint32), single[k][1]), k
    for k in range(2):
        assert_same(S.ref_frame(name, W, H, "primary", pos[k]), (cs[k].cpu().numpy().view(np.uint32),
                                                                  ts[k].cpu().numpy()), f"16-frame launch {k}")
    tile = rtamd.Tile(8, 1, 3, 0)
    npx = L.rt_tile_pixels(W, H, C.byref(tile))
    pc = [torch.zeros(npx, dtype=torch.int32, device="cuda") for _ in P]
    pt = [torch.zeros(npx, dtype=torch.float32, device="cuda") for _ in P]
    s.render_device_frames(P, [c.data_ptr() for c in pc], [t.data_ptr() for t in pt], W, H, rtamd.RT_FLAG_CLEAR,
                           tile=tile)
    torch.cuda.synchronize()
    rows = [y for y in range(H) if (y // 8) % 3 == 1]
    for k in range(n):
        assert np.array_equal(pc[k].cpu().numpy().view(np.uint32), single[k][0][rows].reshape(-1)), k
        assert np.array_equal(pt[k].cpu().numpy().view(np.uint32), single[k][1][rows].reshape(-1)), k


@pytest.mark.parametrize("mode", ["primary", "default"])
def test_band_order_is_output_neutral(gpu, mode):
    """The heavy-first tile order of row-band launches (band_sched: each
    stream's previous band launch's tile costs order its next one) changes
    only the dispatch order: consecutive multi-frame band launches on one
    stream (the first unordered, the next ones ordered) equal the same bands
    rendered one frame at a time, bit for bit; a change of band geometry on
    the stream drops the order and still renders right. The order is opt-in
    (RTAMD_BAND_ORDER=1); the test switches it on for its launches."""
    from rtamd._lib import lib
    torch = pytest.importorskip("torch")
    from rtamd.workloads import orbit_positions
    L = lib()
    name = "stanford-bunny.obj"
    s = S.gpu_scene(name)
    S.set_planes(name, mode, s)
    st = torch.cuda.Stream()
    orbit = orbit_positions(64)
    L.rtx_set_band_order(1)  # opt-in (RTAMD_BAND_ORDER=1)
    try:
        _band_order_cases(L, s, name, mode, st, orbit)
    finally:
        L.rtx_set_band_order(-1)


def _band_order_cases(L, s, name, mode, st, orbit):
    import ctypes as C

    import rtamd
    torch = pytest.importorskip("torch")
    for W, H, tile, launches in ((320, 240, rtamd.Tile(8, 1, 4, 0), 4), (256, 200, rtamd.Tile(8, 0, 3, 0), 2),
                                 (320, 240, rtamd.Tile(8, 1, 4, 0), 2)):
        npx = L.rt_tile_pixels(W, H, C.byref(tile))
        for j in range(launches):
            P = [S.params(name, W, H, mode, orbit[(7 * j + 3 * i) % 64], module="gpu") for i in range(3)]
            pc = [torch.zeros(npx, dtype=torch.int32, device="cuda") for _ in P]
            pt = [torch.zeros(npx, dtype=torch.float32, device="cuda") for _ in P]
            with torch.cuda.stream(st):
                s.render_device_frames(P, [c.data_ptr() for c in pc], [t.data_ptr() for t in pt], W, H,
                                       rtamd.RT_FLAG_CLEAR, tile=tile, stream=st.cuda_stream)
            st.synchronize()
            for k, prm in enumerate(P):
                c1 = torch.zeros(npx, dtype=torch.int32, device="cuda")
                t1 = torch.zeros(npx, dtype=torch.float32, device="cuda")
                s.render_device(prm, c1.data_ptr(), t1.data_ptr(), W, H, clear=True, tile=tile)
                torch.cuda.synchronize()
                assert torch.equal(pc[k], c1), (W, H, j, k)
                assert torch.equal(pt[k].view(torch.int32), t1.view(torch.int32)), (W, H, j, k)


SORT8_PAIRS = [(0, 1), (2, 3), (4, 5), (6, 7), (0, 2), (1, 3), (4, 6), (5, 7), (1, 2), (5, 6),
               (0, 4), (3, 7), (1, 5), (2, 6), (1, 4), (3, 6), (2, 4), (3, 5), (3, 4)]


def test_group_primitives_match_scalar_forms(gpu):
    """The cooperative tail's 8-lane primitives (DPP exchanges) equal the scalar
    forms: the sort8 network (raytracing.hpp:188-213) including its tie order,
    the first-wins min of a leaf scan, and the OR reduction."""
    import ctypes as C

    from rtamd._lib import check, lib
    rng = np.random.default_rng(9)
    n = 4000
    keys = rng.choice(np.array([-1.0, 0.5, 0.5, 1.0, 2.0, 2.0, 3.0, np.inf], np.float32), size=(n, 8))
    keys[: n // 2] = rng.normal(size=(n // 2, 8)).astype(np.float32)
    keys[: n // 4, ::3] = -1.0
    keys = np.ascontiguousarray(keys, np.float32)
    st = np.zeros((n, 8), np.float32)
    sid = np.zeros((n, 8), np.uint32)
    mt = np.zeros(n, np.float32)
    mk = np.zeros(n, np.uint32)
    orv = np.zeros(n, np.uint32)
    L = lib()
    L.rtx_grp_test.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 5
    check(L.rtx_grp_test(keys.ctypes.data, n, st.ctypes.data, sid.ctypes.data, mt.ctypes.data,
                         mk.ctypes.data, orv.ctypes.data))
    for g in range(n):
        t = list(keys[g])
        ids = list(range(8))
        for a, b in SORT8_PAIRS:
            if t[a] > t[b]:
                t[a], t[b] = t[b], t[a]
                ids[a], ids[b] = ids[b], ids[a]
        assert st[g].tolist() == [float(x) for x in t] and sid[g].tolist() == ids, (g, keys[g])
        lt, lk = np.float32(np.inf), 8
        for k in range(8):
            if lt > keys[g, k]:
                lt, lk = keys[g, k], k
        if lk < 8:
            assert mt[g] == lt and mk[g] == lk, (g, keys[g], mt[g], mk[g])
        else:
            assert mt[g] == np.inf
    assert np.all(orv == 0o11111111)


def test_fast_reciprocal_exhaustive(gpu):
    """tri_t's reciprocal (rt_rcp.h rcp_rn: v_rcp_f32 + one fused Newton step)
    equals the IEEE division 1 / x bit for bit for EVERY float x with
    1e-8 <= |x| < 2^126 -- the range where the triangle test uses it (below,
    the triangle is a miss whatever the value; above, inf and NaN take the
    division). Exhaustive over all 2^32 bit patterns, on this GPU."""
    import ctypes as C

    from rtamd._lib import lib
    L = lib()
    checked, bad, first = C.c_uint64(0), C.c_uint64(0), C.c_uint32(0)
    L.rtx_rcp_check.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
    assert L.rtx_rcp_check(C.byref(checked), C.byref(bad), C.byref(first)) == 0
    # 2 signs x 2^23 mantissas x (the 152 binades 2^-26 .. 2^125, and the part of 2^-27's binade
    # from 1e-8 up)
    assert 2 * 152 * (1 << 23) < checked.value < 2 * 153 * (1 << 23)
    assert bad.value == 0, f"{bad.value} mismatches, e.g. x bits 0x{first.value:08x}"


@pytest.mark.parametrize("log2_scale", [0, 20])
def test_triangle_reciprocal_scene_bound(gpu, log2_scale):
    """The fast reciprocal of the triangle test (tri_t<true>) is taken by rays
    whose direction keeps every |det| of the scene below 2^125
    (MeshDev::dmax2); axis-parallel rays (1/d infinite) take the division.
    The bunny at scale 1 and scaled by 2^20 (exact: a power of two), rays with
    |d| from 1 to 2^14: hit, t, normal and primitive id equal the oracle's bit
    for bit. (|det| near 2^125 needs coordinates or directions large enough
    that the test's other products overflow too; there the reference can
    report a hit at t = inf or NaN, which this path reports as a miss:
    DESIGN.md section 2.)"""
    import rtamd
    from rtamd import data
    m = rtamd.load_mesh_from_obj(data.path("stanford-bunny.obj"))
    v = m.vPos4f.copy()
    v[:, :3] = np.ldexp(v[:, :3], log2_scale)
    gs = rtamd.BVHBuilder(rtamd.SimpleMesh(v, m.indices))
    rs = cpuref.RefScene.mesh(v, m.indices)
    o, d = _random_rays(20000, 77 + log2_scale, inside_frac=0.3)
    o = np.ldexp(o, log2_scale).astype(np.float32)
    rng = np.random.default_rng(5)
    d = np.ldexp(d, rng.integers(0, 15, (len(d), 1))).astype(np.float32)
    tn, tf = 0.0, 1e30
    rh, rt_, rn, rp = rs.intersect_rays(o, d, tn, tf)
    g = gs.intersect(o, d, tn, tf)
    assert rh.sum() > 1000
    assert np.array_equal(rh.astype(bool), g.hitten), "hit mask differs"
    assert np.array_equal(rp, g.prim), "primitive ids differ"
    h = g.hitten
    assert np.array_equal(rt_[h].view(np.uint32), g.t[h].view(np.uint32)), "t differs"
    assert np.array_equal(rn[h].view(np.uint32), g.normal[h].view(np.uint32)), "normal differs"
    gs.close()


@pytest.mark.parametrize("mode,n", [(0, 0), (1, 1 << 32)])
def test_fast_eye_division(gpu, mode, n):
    """eye_ray_fast's divisions (rt_rcp.h div_mk: the checked reciprocal and one
    fused correction) give the IEEE division's bits: (0) 2 (x + 1/2) / W for
    EVERY x < W <= 32768; (1) 2^32 random pairs over the ranges fast_eye_ok
    guarantees (|a| in [2^-72, 2^24] or +-0, |b| in [2^-20, 2^24])."""
    import ctypes as C

    from rtamd._lib import lib
    L = lib()
    out = (C.c_uint64 * 3)()
    L.rtx_div_check.argtypes = [C.c_int32, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]
    assert L.rtx_div_check(mode, n, 2024, out) == 0
    assert out[0] == (32768 * 32769 // 2 if mode == 0 else n)
    assert out[1] == 0, f"{out[1]} mismatches, e.g. a, b bits 0x{out[2] & 0xFFFFFFFF:08x}, 0x{out[2] >> 32:08x}"


@pytest.mark.parametrize("variant", ["reference", "offcenter", "scaled"])
def test_eye_ray_projections(gpu, variant):
    """Frames equal the oracle's bit for bit whichever eye-ray path the
    projection selects: the reference's perspective and an off-centre one take
    eye_ray_fast (fast_eye_ok), the same perspective scaled by 2^12 (the same
    rays, entries out of its range) takes the divisions."""
    import ctypes as C

    import rtamd
    name, W, H = "stanford-bunny.obj", 320, 180
    sm, plane, sh, rf = S.MODES["default"]
    pos = (0.3, 0.2, 2.4)
    vi, pi = cpuref.camera_matrices(pos, (0, 0, 0), (0, 1, 0), 45.0, W / H, 0.01, 100.0)
    pi = np.array(pi, np.float32).reshape(-1).copy()
    if variant == "offcenter":
        pi[12] += np.float32(0.25)
        pi[13] -= np.float32(0.125)
    elif variant == "scaled":
        pi *= np.float32(2.0 ** 12)
    L = rtamd.lib()
    L.rtx_fast_eye_ok.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
    assert L.rtx_fast_eye_ok(pi.ctypes.data, W, H) == (0 if variant == "scaled" else 1)
    rs, gs = S.ref_scene(name), S.gpu_scene(name)
    S.set_planes(name, "default", rs, gs)
    rc, rt_, _, _ = rs.render(cpuref.make_params(pos, vi, pi, (2, 2, 2), sm, sh, rf), W, H)
    c = np.zeros((H, W), np.uint32)
    t = np.full((H, W), np.inf, np.float32)
    gs.render(rtamd.render_params(pos, vi, pi, (2, 2, 2), sm, sh, rf), c, t, clear=True)
    assert np.array_equal(c, rc), int((c != rc).sum())
    assert np.array_equal(t.view(np.uint32), rt_.view(np.uint32))
