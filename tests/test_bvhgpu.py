"""The device BVH8 builder (rt_bvhgpu.hip) builds the
same tree as BVHBuilder::perform (triangles_raytracing.cpp:12-258): its
canonical export (topology, leaf ranges, child boxes bitwise) and triangle
permutation equal the host builder's, which tests/test_host.py pins to the
oracle's restatement of the reference builder. The device sort is checked
against libstdc++'s std::sort permutation itself (ties included, the
heapsort fallback forced with small depth limits)."""
import ctypes as C

import numpy as np
import pytest

import scenes as S

pytestmark = pytest.mark.gpu


def sort_check(keys, depth=-1):
    from rtamd import _lib
    L = _lib.lib()
    L.rtx_sort_check.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.POINTER(C.c_int64)]
    keys = np.ascontiguousarray(keys, np.float32)
    ids = np.zeros(len(keys), np.uint32)
    bad = C.c_int64(-1)
    _lib.check(L.rtx_sort_check(keys.ctypes.data, len(keys), depth, ids.ctypes.data, C.byref(bad)))
    return ids, bad.value


@pytest.mark.parametrize("n,kind", [(2, "rand"), (17, "rand"), (1024, "ties"), (1025, "ties"), (3079, "rand"),
                                    (50_000, "ties"), (200_000, "rand"), (200_000, "few"), (1_000_003, "ties"),
                                    (70_000, "sorted"), (70_000, "reversed"), (70_000, "equal"),
                                    (300_000, "organ")])
def test_device_sort_is_std_sort(gpu, n, kind):
    rng = np.random.default_rng(n)
    if kind == "rand":
        k = rng.normal(size=n)
    elif kind == "ties":
        k = rng.integers(0, max(2, n // 20), n).astype(np.float64) * 0.25
    elif kind == "few":
        k = rng.integers(0, 3, n).astype(np.float64)
    elif kind == "sorted":
        k = np.arange(n) // 3
    elif kind == "reversed":
        k = -(np.arange(n) // 5)
    elif kind == "equal":
        k = np.zeros(n)
    else:  # organ pipe
        k = np.minimum(np.arange(n), n - np.arange(n)).astype(np.float64)
    ids, bad = sort_check(k.astype(np.float32))
    assert bad == 0, f"{bad} of {n} positions differ from std::sort"
    kk = k.astype(np.float32)[ids]
    assert np.all(kk[:-1] <= kk[1:])


@pytest.mark.parametrize("n,depth", [(5000, 2), (100_000, 3), (100_000, 10), (40_000, 0)])
def test_device_sort_heapsort_fallback(gpu, n, depth):
    """Depth limits small enough that the introsort loop falls back to
    std::__partial_sort (heapsort) on big ranges: still std::sort's permutation."""
    rng = np.random.default_rng(depth)
    k = rng.integers(0, 50, n).astype(np.float32)
    _, bad = sort_check(k, depth)
    assert bad == 0


def export(v, i, mode):
    import rtamd
    L = rtamd.lib()
    rtamd._lib.check(L.rt_set_bvh_builder(mode))
    try:
        nn, md = C.c_int64(0), C.c_int32(0)
        v = np.ascontiguousarray(v, np.float32)
        i = np.ascontiguousarray(i, np.uint32)
        rtamd._lib.check(L.rt_bvh_export(v.ctypes.data, len(v), i.ctypes.data, len(i), None, C.byref(nn), None,
                                         None))
        canon = np.zeros((nn.value, 52), np.uint32)
        perm = np.zeros(len(i) // 3, np.uint32)
        rtamd._lib.check(L.rt_bvh_export(v.ctypes.data, len(v), i.ctypes.data, len(i), canon.ctypes.data,
                                         C.byref(nn), perm.ctypes.data, C.byref(md)))
        return canon, perm, md.value
    finally:
        rtamd._lib.check(L.rt_set_bvh_builder(0))


def same_tree(v, i):
    ch, ph, dh = export(v, i, 1)
    cd, pd, dd = export(v, i, 2)
    assert ch.shape == cd.shape, f"{len(cd)} nodes on the device vs {len(ch)} on the host"
    bad = np.flatnonzero((ch != cd).any(1))
    assert bad.size == 0, f"{bad.size} nodes differ, first {bad[:5]}"
    assert np.array_equal(ph, pd) and dh == dd


@pytest.mark.parametrize("name", ["cube.obj", "spot.obj", "stanford-bunny.obj"])
def test_device_builder_shipped_meshes(gpu, name):
    _, (v, i), _ = S.inputs(name)
    same_tree(v, i)


@pytest.mark.parametrize("seed,ntri,mode", [(1, 1, "rand"), (3, 9, "rand"), (4, 300, "rand"), (6, 64, "same"),
                                            (7, 500, "grid"), (8, 100, "flat"), (9, 30000, "grid"),
                                            (10, 12000, "same"), (11, 40000, "rand"), (12, 150000, "grid"),
                                            (13, 3000, "signed0"), (14, 40000, "signed0")])
def test_device_builder_edge_meshes(gpu, seed, ntri, mode):
    """test_host.py's tie-heavy meshes: duplicate triangles (all keys tie),
    integer lattices (many equal keys), flat meshes (zero-area boxes), and
    lattices whose zero coordinates are a random mix of -0.0 and +0.0: a child
    box bound that is 0 must carry the sign bit calc_bbox gives it when the
    node is created (triangles_raytracing.cpp:199), before the children's
    sorts reorder the range."""
    v4 = S.edge_mesh(seed, ntri, mode)
    same_tree(v4, np.arange(len(v4), dtype=np.uint32))


def test_device_builder_config5_standin(gpu):
    """The 1,111,216-triangle stand-in of BASELINE configs[4]."""
    import rtamd
    _, (v, i), _ = S.inputs("stanford-bunny.obj")
    m = rtamd.subdivide_mesh(rtamd.SimpleMesh(v, i), 2)
    same_tree(m.vPos4f, m.indices)


def test_device_built_scene_renders_golden_frame(gpu):
    """A scene whose BVH8 the device built renders the reference's golden 1080p hash."""
    import cpuref
    import rtamd
    _, (v, i), _ = S.inputs("stanford-bunny.obj")
    rtamd._lib.check(rtamd.lib().rt_set_bvh_builder(2))
    try:
        sc = rtamd.BVHBuilder(rtamd.SimpleMesh(v, i))
    finally:
        rtamd._lib.check(rtamd.lib().rt_set_bvh_builder(0))
    sc.set_plane(None)
    W, H = 1920, 1080
    c = np.zeros((H, W), np.uint32)
    t = np.full((H, W), np.inf, np.float32)
    sc.render(S.params("stanford-bunny.obj", W, H, "primary", module="gpu"), c, t, clear=True)
    assert cpuref.fnv1a64_words(c) == S.GOLDEN[("stanford-bunny.obj", 1920, 1080, "primary")]


def test_auto_mode_falls_back_to_host_on_device_failure(gpu):
    """AUTO mode (the default) builds meshes from 32,768 triangles on the device;
    a device failure there (simulated by rtx_bvh_inject_failure) must not fail
    scene creation: the host builder gives the identical tree. The forced
    device mode reports the failure as RT_E_DEVICE with the HIP error text."""
    import cpuref
    import rtamd
    L = rtamd.lib()
    _, (v, i), _ = S.inputs("stanford-bunny.obj")
    assert len(i) // 3 >= 32768
    L.rtx_bvh_inject_failure(1)
    try:
        sc = rtamd.BVHBuilder(rtamd.SimpleMesh(v, i))
    finally:
        L.rtx_bvh_inject_failure(0)
    assert L.rtx_bvh_last_builder() == 3  # host, after the device build failed
    sc.set_plane(None)
    W, H = 1920, 1080
    c = np.zeros((H, W), np.uint32)
    t = np.full((H, W), np.inf, np.float32)
    sc.render(S.params("stanford-bunny.obj", W, H, "primary", module="gpu"), c, t, clear=True)
    assert cpuref.fnv1a64_words(c) == S.GOLDEN[("stanford-bunny.obj", 1920, 1080, "primary")]
    sc.close()
    # without injection AUTO uses the device
    sc2 = rtamd.BVHBuilder(rtamd.SimpleMesh(v, i))
    assert L.rtx_bvh_last_builder() == 2
    sc2.close()
    # DEVICE mode: no fallback, a device error
    rtamd._lib.check(L.rt_set_bvh_builder(2))
    L.rtx_bvh_inject_failure(1)
    try:
        with pytest.raises(rtamd.RtError, match=r"error -3: GPU BVH build: injected failure: "):
            rtamd.BVHBuilder(rtamd.SimpleMesh(v, i))
    finally:
        L.rtx_bvh_inject_failure(0)
        rtamd._lib.check(L.rt_set_bvh_builder(0))


def test_auto_mode_reports_builder_bounds(gpu):
    """An exceeded bound of the device builder's own stage logic (a builder bug,
    simulated by rtx_bvh_inject_failure(-1)) is reported as RT_E_DEVICE in AUTO
    mode too, not hidden by the host fallback; the next build is unaffected."""
    import rtamd
    L = rtamd.lib()
    _, (v, i), _ = S.inputs("stanford-bunny.obj")
    L.rtx_bvh_inject_failure(-1)
    try:
        with pytest.raises(rtamd.RtError, match=r"error -3: GPU BVH builder bound: injected bound"):
            rtamd.BVHBuilder(rtamd.SimpleMesh(v, i))
    finally:
        L.rtx_bvh_inject_failure(0)
    sc = rtamd.BVHBuilder(rtamd.SimpleMesh(v, i))
    assert L.rtx_bvh_last_builder() == 2
    sc.close()
