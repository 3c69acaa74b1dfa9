"""Host-side logic of the product (no GPU): C-ABI exports, loaders, the BVH8
builder, camera math, octree box arithmetic and row-band tiling -- each
checked against the oracle or an independent restatement."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import scenes as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtamd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol(rt):
    names = header_functions()
    assert len(names) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", rt.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (rt_[a-z0-9_]+)$", out, flags=re.M))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    assert set(names) == set(rt.EXPORTED)
    assert rt.lib().rt_abi_version() == 8


def test_library_build_id_matches_tree(rt):
    """librtamd.so (the binary the GPU box runs) was built from this tree's
    sources: rt_build_id() equals the hash of csrc/ + include/rtamd.h."""
    if os.environ.get("RTAMD_LIB"):
        pytest.skip("a variant library injected through RTAMD_LIB")
    assert rt.lib().rt_build_id().decode() == rt._lib.source_build_id()


@pytest.mark.parametrize("name", ["cube.obj", "spot.obj", "stanford-bunny.obj"])
def test_obj_loader_matches_oracle(rt, ref, name):
    p = rt.data.path(name)
    m = rt.load_mesh_from_obj(p)
    v, i = ref.load_obj(p)
    assert np.array_equal(m.vPos4f.view(np.uint32), v.view(np.uint32))
    assert np.array_equal(m.indices, i)
    m2 = rt.load_mesh_from_obj(p, scale=False)
    v2, i2 = ref.load_obj(p, scale=False)
    assert np.array_equal(m2.vPos4f.view(np.uint32), v2.view(np.uint32))


def test_grid_and_octree_loaders(rt):
    p = rt.data.path("example_grid.grid")
    size, vals = rt.load_sdf_grid(p)
    assert list(size) == list(np.fromfile(p, np.uint32, 3))
    assert np.array_equal(vals, np.fromfile(p, np.float32, offset=12))
    p = rt.data.path("sdf_6.octree")
    nodes = rt.load_sdf_octree(p)
    assert nodes.size == 36417 * 36
    assert np.array_equal(nodes, np.fromfile(p, np.uint8, offset=4))


def test_loader_errors(rt, tmp_path):
    with pytest.raises(rt.RtError, match="-2"):
        rt.load_mesh_from_obj(str(tmp_path / "missing.obj"))
    bad = tmp_path / "short.grid"
    np.array([4, 4, 4], np.uint32).tofile(bad)
    with open(bad, "ab") as f:
        f.write(b"\0" * 16)
    with pytest.raises(rt.RtError, match="truncated"):
        rt.load_sdf_grid(str(bad))


def bvh_export(rt, v, i):
    L = rt.lib()
    nn, md = C.c_int64(0), C.c_int32(0)
    v = np.ascontiguousarray(v, np.float32)
    i = np.ascontiguousarray(i, np.uint32)
    rt._lib.check(L.rt_bvh_export(v.ctypes.data, len(v), i.ctypes.data, len(i), None, C.byref(nn),
                                  None, C.byref(md)))
    canon = np.zeros((nn.value, 52), np.uint32)
    perm = np.zeros(len(i) // 3, np.uint32)
    rt._lib.check(L.rt_bvh_export(v.ctypes.data, len(v), i.ctypes.data, len(i), canon.ctypes.data,
                                  C.byref(nn), perm.ctypes.data, C.byref(md)))
    return canon, perm, md.value


@pytest.mark.parametrize("name", ["cube.obj", "spot.obj", "stanford-bunny.obj"])
def test_bvh8_identical_to_reference_builder(rt, ref, name):
    """BVHBuilder::perform: same topology, leaf ranges, child boxes (bitwise) and
    triangle permutation as the oracle's restatement of the reference builder."""
    kind, (v, i), _ = S.inputs(name)
    canon, perm, depth = bvh_export(rt, v, i)
    rs = ref.RefScene.mesh(v, i)
    assert np.array_equal(canon, rs.bvh_export())
    _, tri = rs.bvh_indices(len(i))
    assert np.array_equal(perm, tri)
    if name == "stanford-bunny.obj":
        assert len(canon) == 12143 and depth == 5


@pytest.mark.parametrize("seed,ntri,mode", [(1, 1, "rand"), (2, 7, "rand"), (3, 9, "rand"), (4, 300, "rand"),
                                            (5, 2000, "rand"), (6, 64, "same"), (7, 500, "grid"),
                                            (8, 100, "flat"), (9, 30000, "grid"), (10, 12000, "same"),
                                            (11, 40000, "rand"), (13, 3000, "signed0"), (14, 40000, "signed0")])
def test_bvh8_edge_cases(rt, ref, seed, ntri, mode):
    """Tiny meshes (root leaf), duplicate triangles (all SAH keys tie), axis-aligned
    grids of triangles (many equal keys) and flat meshes (zero-area boxes). The
    large cases run the parallel sort (ranges >= 4096 ids) and the concurrent
    axes, whose tie order must equal the serial std::sort's."""
    rng = np.random.default_rng(seed)
    if mode == "signed0":  # lattice with -0.0 / +0.0 mixed: child box bounds keep calc_bbox's sign bit
        g = rng.integers(-2, 3, size=(ntri, 3)).astype(np.float64)
        v = np.concatenate([g, g + [1, 0, 0], g + [0, 1, 0]], axis=1).reshape(-1, 3)
        v[(v == 0) & (rng.random(v.shape) < 0.5)] = -0.0
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
    v4 = np.concatenate([v, np.ones((len(v), 1))], axis=1).astype(np.float32)
    idx = np.arange(len(v), dtype=np.uint32)
    canon, perm, _ = bvh_export(rt, v4, idx)
    rs = ref.RefScene.mesh(v4, idx)
    assert np.array_equal(canon, rs.bvh_export())
    assert np.array_equal(perm, rs.bvh_indices(len(idx))[1])


def test_camera_matrices_match_reference(rt, ref):
    from rtamd.workloads import orbit_positions
    for pos in orbit_positions(64) + [(0.0, 0.0, 2.5), (0.0, 3.0, 1e-3), (-2.0, -1.0, 0.5)]:
        for aspect in (16 / 9, 1.0, 4 / 3):
            a = rt.camera_matrices(pos, aspect=aspect)
            b = ref.camera_matrices(pos, aspect=aspect)
            assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
            assert np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))


def _divide_chain_boxes(nodes36):
    """Every node's box by the reference's float32 divide_box_8 chain
    (ray_pack.ispc:220-239 from the root box [-1,1]^3), plus its depth and
    integer coordinates."""
    f32 = np.float32
    n = nodes36.size // 36
    rec = nodes36.reshape(n, 36)
    off = rec[:, 32:36].copy().view(np.uint32).ravel()
    out = {0: (np.full(3, -1, f32), np.full(3, 1, f32), 0, (0, 0, 0))}
    stack = [0]
    while stack:
        i = stack.pop()
        bmin, bmax, d, ijk = out[i]
        if off[i] == 0:
            continue
        center = (bmin + bmax) / f32(2.0)
        diff = center - bmin
        for c in range(8):
            x, y, z = c >> 2, (c & 3) >> 1, c & 1
            mn = np.array([bmin[0] if x == 0 else center[0], bmin[1] if y == 0 else center[1],
                           bmin[2] if z == 0 else center[2]], f32)
            out[int(off[i]) + c] = (mn, mn + diff, d + 1, (2 * ijk[0] + x, 2 * ijk[1] + y, 2 * ijk[2] + z))
            stack.append(int(off[i]) + c)
    return out


@pytest.mark.parametrize("name", ["sdf_5.octree", "sdf_6.octree"])
def test_octree_box_arithmetic_is_exact(rt, name):
    """The kernels compute a node's box from its depth and integer coordinates
    ([-1 + i*s, -1 + i*s + s], s = 2^(1-depth)); the reference derives it by
    repeated float divide_box_8. Equal bit for bit on every node."""
    nodes = rt.load_sdf_octree(rt.data.path(name))
    boxes = _divide_chain_boxes(nodes)
    for i, (bmin, bmax, d, ijk) in boxes.items():
        s = np.float32(np.ldexp(2.0, -d))
        mn = (np.float32(-1.0) + np.asarray(ijk, np.float32) * s).astype(np.float32)
        mx = (mn + s).astype(np.float32)
        assert np.array_equal(mn.view(np.uint32), bmin.view(np.uint32)), (i, d)
        assert np.array_equal(mx.view(np.uint32), bmax.view(np.uint32)), (i, d)


@pytest.mark.parametrize("W,H,band,n", [(1920, 1080, 16, 1), (1920, 1080, 16, 2), (1920, 1080, 16, 8),
                                        (640, 360, 7, 3), (100, 5, 16, 4), (33, 1000, 1, 7)])
def test_row_band_tiling(rt, W, H, band, n):
    from rtamd.tiles import rank_rows
    rows = [rank_rows(H, band, r, n) for r in range(n)]
    allr = np.sort(np.concatenate(rows))
    assert np.array_equal(allr, np.arange(H))  # every row exactly once
    for r in range(n):
        t = rt.Tile(band, r, n, 0)
        assert rt.lib().rt_tile_pixels(W, H, C.byref(t)) == len(rows[r]) * W
