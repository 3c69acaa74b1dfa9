"""OBJ writer, host-only.

rt_save_obj (product, csrc/rt_host.cpp) against the oracle's restatement of
cmesh4::SaveMeshToObj (src/core/mesh.cpp:14-63) byte for byte, and round trips
through the product OBJ loader (LoadMeshFromObj, mesh.cpp:206-300).
"""
import numpy as np
import pytest

import cpuref


def rand_mesh(seed, nv, nt):
    rng = np.random.default_rng(seed)
    v = np.concatenate([rng.normal(scale=3.0, size=(nv, 3)), np.ones((nv, 1))], 1).astype(np.float32)
    v[0, :3] = [-0.0, 1e-9, -123456.75]
    i = rng.integers(0, nv, size=3 * nt).astype(np.uint32)
    return v, i


@pytest.mark.parametrize("seed,nv,nt", [(0, 3, 1), (1, 50, 80), (2, 1000, 2000)])
@pytest.mark.parametrize("attrs", [False, True])
def test_save_obj_matches_reference_writer(rt, tmp_path, seed, nv, nt, attrs):
    v, i = rand_mesh(seed, nv, nt)
    rng = np.random.default_rng(seed + 100)
    n = rng.normal(size=(nv, 4)).astype(np.float32) if attrs else None
    t = rng.uniform(size=(nv, 2)).astype(np.float32) if attrs else None
    p = tmp_path / "m.obj"
    rt.save_mesh_to_obj(str(p), rt.SimpleMesh(v, i), n, t)
    assert p.read_bytes() == cpuref.save_obj_text(v, i, n, t)


@pytest.mark.parametrize("name", ["stanford-bunny.obj", "spot.obj"])
def test_save_load_roundtrip(rt, tmp_path, name):
    """Load (unscaled), save, load again: indices identical, positions equal to
    their "%f" rounding (float32 of the 6-decimal text)."""
    m = rt.load_mesh_from_obj(rt.data.path(name), scale=False)
    v, i = m.vPos4f, m.indices
    p = tmp_path / "rt.obj"
    rt.save_mesh_to_obj(str(p), rt.SimpleMesh(v, i))
    m2 = rt.load_mesh_from_obj(str(p), scale=False)
    v2, i2 = m2.vPos4f, m2.indices
    assert np.array_equal(i, i2)
    want = np.array([[float("%f" % float(x)) for x in row[:3]] for row in v], np.float32)
    assert np.array_equal(v2[:, :3], want)


def test_save_obj_errors(rt, tmp_path):
    v, i = rand_mesh(0, 4, 2)
    with pytest.raises(rt.RtError):
        rt.save_mesh_to_obj(str(tmp_path / "no" / "such" / "dir.obj"), rt.SimpleMesh(v, i))
    with pytest.raises(rt.RtError):
        rt.save_mesh_to_obj(str(tmp_path / "x.obj"), rt.SimpleMesh(v, i[:4]))
