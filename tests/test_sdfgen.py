"""Mesh -> SDF construction and the config 3-5 stand-ins.

The reference renders SDF grids / octrees but has no generator for them, so
the definition lives in the oracle (oracle/cpuref.cpp `sdfref`, brute force
over every triangle; oracle/cpuref.py for lattice, octree assembly and
subdivision). Parity of that definition against the reference is unpinned; the
GPU generator must equal it bit for bit.
"""
import numpy as np
import pytest

import cpuref
import scenes as S


def mesh(name):
    kind, (v, i), _ = S.inputs(name)
    assert kind == "mesh"
    return v, i


# ------------------------------------------------------------- CPU (host) --
@pytest.mark.parametrize("name,levels", [("cube.obj", 1), ("cube.obj", 3), ("spot.obj", 1),
                                         ("stanford-bunny.obj", 1)])
def test_subdivision_matches_oracle(rt, name, levels):
    v, i = mesh(name)
    got = rt.subdivide_mesh(rt.SimpleMesh(v, i), levels)
    rv, ri = cpuref.subdivide(v, i, levels)
    assert got.indices.size == i.size * 4 ** levels
    assert np.array_equal(got.indices, ri)
    assert np.array_equal(got.vPos4f.view(np.uint32), rv.view(np.uint32))


def test_config5_standin_size(rt):
    """BASELINE configs[4] stand-in: stanford-bunny subdivided twice = 1,111,216 triangles."""
    v, i = mesh("stanford-bunny.obj")
    m = rt.subdivide_mesh(rt.SimpleMesh(v, i), 2)
    assert m.TrianglesNum() == 1_111_216
    # every original vertex is kept, edge midpoints are shared (closed under welding)
    assert np.array_equal(m.vPos4f[:len(v)], v)
    assert int(m.indices.max()) == len(m.vPos4f) - 1


def test_subdivision_errors(rt):
    v, i = mesh("cube.obj")
    with pytest.raises(rt.RtError):
        rt.subdivide_mesh(rt.SimpleMesh(v, i[:-1]), 1)
    with pytest.raises(rt.RtError):
        rt.subdivide_mesh(rt.SimpleMesh(v, i), 7)


def test_oracle_sdf_on_cube_is_box_distance():
    """Sanity of the definition: the cube.obj mesh is an axis-aligned box, so the
    signed distance is the analytic box SDF (to f32 rounding)."""
    v, i = mesh("cube.obj")
    p = v[:, :3] / v[:, 3:4]
    lo, hi = p.min(0), p.max(0)
    rng = np.random.default_rng(5)
    q = rng.uniform(-1, 1, (2000, 3)).astype(np.float32)
    got = cpuref.sdf_points(v, i, q)
    c, h = (lo + hi) / 2, (hi - lo) / 2
    d = np.abs(q - c) - h
    exact = np.linalg.norm(np.maximum(d, 0), axis=1) + np.minimum(d.max(1), 0)
    np.testing.assert_allclose(got, exact, atol=2e-6)


def test_oracle_octree_structure():
    v, i = mesh("cube.obj")
    rec = cpuref.sdf_octree(v, i, 3).reshape(-1, 36)
    off = rec[:, 32:].copy().view(np.uint32).ravel()
    vals = rec[:, :32].copy().view(np.float32).reshape(-1, 8)
    inner = off != 0
    assert off[0] == 1 and np.all(off[inner] % 8 == 1)
    assert np.all(vals[inner] == 0)
    # children blocks tile the node array exactly once, in BFS order
    kids = np.sort(np.concatenate([np.arange(o, o + 8) for o in off[inner]]))
    assert np.array_equal(kids, np.arange(1, len(rec)))


# --------------------------------------------------------------- GPU parity --
def _points(name, n, seed):
    """Uniform points in [-1,1]^3 plus points jittered around surface vertices."""
    v, _ = mesh(name)
    rng = np.random.default_rng(seed)
    u = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    pv = (v[:, :3] / v[:, 3:4])[rng.integers(0, len(v), n)]
    near = (pv + rng.normal(0, 0.01, (n, 3))).astype(np.float32)
    return np.concatenate([u, near, pv.astype(np.float32)])


@pytest.mark.gpu
@pytest.mark.parametrize("name,n", [("cube.obj", 3000), ("spot.obj", 2000), ("stanford-bunny.obj", 700)])
def test_sdf_points_bit_exact(gpu, rt, name, n):
    v, i = mesh(name)
    p = _points(name, n, 11)
    with rt.SDFMesh(rt.SimpleMesh(v, i)) as m:
        got = m.points(p)
    ref = cpuref.sdf_points(v, i, p, 16)
    bad = np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert bad.size == 0, f"{bad.size} of {len(p)} differ, e.g. {p[bad[:3]]} {got[bad[:3]]} {ref[bad[:3]]}"


@pytest.mark.gpu
@pytest.mark.parametrize("name,size", [("cube.obj", (17, 17, 17)), ("spot.obj", (20, 23, 18)),
                                       ("stanford-bunny.obj", (16, 16, 16))])
def test_sdf_grid_bit_exact(gpu, rt, name, size):
    v, i = mesh(name)
    with rt.SDFMesh(rt.SimpleMesh(v, i)) as m:
        sz, got = m.grid(size)
    ref = cpuref.sdf_points(v, i, cpuref.lattice_points(size), 16)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("name,depth", [("cube.obj", 4), ("spot.obj", 3), ("stanford-bunny.obj", 3)])
def test_sdf_octree_bit_exact(gpu, rt, name, depth):
    v, i = mesh(name)
    with rt.SDFMesh(rt.SimpleMesh(v, i)) as m:
        got = m.octree(depth)
    ref = cpuref.sdf_octree(v, i, depth, 16)
    assert got.size == ref.size and np.array_equal(got, ref)


@pytest.mark.gpu
def test_config3_standin_grid_sampled(gpu, rt):
    """BASELINE configs[2] stand-in (example_grid_large.grid is missing): the
    stanford-bunny SDF on a 256^3 lattice (64 MiB). Full-size check: 3000
    random lattice samples equal the oracle's brute force bit for bit, and the
    grid is a plausible SDF (negative inside, |grad| <= 1 between samples)."""
    v, i = mesh("stanford-bunny.obj")
    with rt.SDFMesh(rt.SimpleMesh(v, i)) as m:
        size, vals = m.grid(256)
    assert vals.size == 256 ** 3
    rng = np.random.default_rng(3)
    idx = rng.integers(0, vals.size, 3000)
    ijk = np.stack(np.unravel_index(idx, (256, 256, 256)), 1).astype(np.float32)
    pts = np.float32(2.0) * ijk / np.float32(255) - np.float32(1.0)
    ref = cpuref.sdf_points(v, i, pts, 16)
    assert np.array_equal(vals[idx].view(np.uint32), ref.view(np.uint32))
    g = vals.reshape(256, 256, 256)
    h = np.float32(2.0 / 255)
    # distance is 1-Lipschitz; sign flips only across the surface (the bunny's
    # open bottom can flip a few off-surface samples)
    assert np.mean(np.abs(np.diff(g, axis=2)) <= h * 1.0001) > 0.9999
    assert (g < 0).sum() > 100000 and g[0, 0, 0] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["grid", "octree"])
def test_render_generated_standins_bit_exact(gpu, rt, kind):
    """Frames of the GENERATED bunny SDF (grid 96^3 / octree depth 6) on the GPU
    equal the oracle's frames of the same data (primary and default mode)."""
    v, i = mesh("stanford-bunny.obj")
    with rt.SDFMesh(rt.SimpleMesh(v, i)) as m:
        if kind == "grid":
            size, vals = m.grid(96)
            ref_s, gpu_s = cpuref.RefScene.grid(size, vals), rt.SDFGrid(size, vals)
        else:
            nodes = m.octree(6)
            ref_s, gpu_s = cpuref.RefScene.octree(nodes), rt.SDFOctree(nodes)
    W, H = 320, 240
    with gpu_s:
        for mode, pos in (("primary", (0.0, 0.0, 2.5)), ("default", (1.5, 0.8, 2.0))):
            plane = S.MODES[mode][1]
            ref_s.set_plane(plane, (0.0, 1.0, 0.0), -1.0)
            gpu_s.set_plane(rt.Plane((0.0, 1.0, 0.0), -1.0) if plane else None)
            rc, rtt, _, _ = ref_s.render(S.params("stanford-bunny.obj", W, H, mode, pos, "ref"), W, H)
            gc = np.zeros((H, W), np.uint32)
            gt = np.full((H, W), np.inf, np.float32)
            gpu_s.render(S.params("stanford-bunny.obj", W, H, mode, pos, "gpu"), gc, gt, clear=True)
            assert np.isfinite(rtt).sum() > 1000
            assert np.array_equal(rc, gc), f"{kind} {mode}: {(rc != gc).sum()} colour px differ"
            assert np.array_equal(rtt.view(np.uint32), gt.view(np.uint32))


@pytest.mark.gpu
def test_stale_hip_error_reported_as_such(gpu, rt):
    """A HIP error left pending by an earlier call (here librtamd's own
    hipSetDevice(-1), rtx_inject_stale_error) is not taken for the failure of
    the next query's copy: the query succeeds, bit-exact, and the stale error
    is reported separately, naming the call that raised it (the round-4
    'hipMemcpy H2D failed' could not tell the two apart)."""
    import ctypes as C
    L = rt.lib()
    L.rtx_sdf_last_stale.restype = C.c_char_p
    v, i = mesh("cube.obj")
    p = _points("cube.obj", 500, 5)
    ref = cpuref.sdf_points(v, i, p, 16)
    with rt.SDFMesh(rt.SimpleMesh(v, i)) as m:
        assert m.points(p).view(np.uint32).tolist() == ref.view(np.uint32).tolist()
        assert L.rtx_sdf_last_stale() == b""
        assert L.rtx_inject_stale_error() == 0
        got = m.points(p)  # succeeds: the pending error is not this call's
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        msg = L.rtx_sdf_last_stale().decode()
        assert "stale HIP error" in msg and "hipSetDevice(-1)" in msg, msg
        m.points(p)
        assert L.rtx_sdf_last_stale() == b""  # read and cleared once
