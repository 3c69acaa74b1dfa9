"""The oracle (oracle/cpuref.cpp) against the reference's golden vectors.

The reference ships no tests; its only pins are the frame hashes the survey
recorded from the reference's own unmodified translation units (SURVEY.md
8(c)) and the per-ray work statistics of the same runs.
"""
import json
import os

import numpy as np
import pytest

import scenes as S

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("key", sorted(S.GOLDEN))
def test_golden_hashes(ref, key):
    name, W, H, mode = key
    c, t = S.ref_frame(name, W, H, mode)
    assert ref.fnv1a64_words(c) == S.GOLDEN[key]
    if key in S.COVERAGE:
        assert int(np.isfinite(t).sum()) == S.COVERAGE[key]


@pytest.mark.parametrize("name,W,H,expect", [
    # SURVEY.md 8(a) a5/a9/a11 (1080p, camera (0,0,2.5), primary rays)
    ("stanford-bunny.obj", 1920, 1080, {"bvh_inner": 1.93, "bvh_leaf": 0.31, "bvh_tri": 2.44}),
    ("example_grid.grid", 1920, 1080, {"grid_sdf": 5.03 + 6 * 0.244}),
    ("sdf_6.octree", 1920, 1080, {"oct_node": 11.65, "oct_leaf": 5.52, "oct_step": 2.93,
                                   "oct_normal": 0.324}),
])
def test_work_statistics(ref, name, W, H, expect):
    ref.counters(True)
    S.ref_frame(name, W, H, "primary")
    c = ref.counters(True)
    for k, v in expect.items():
        assert abs(c[k] / (W * H) - v) < 0.006, (k, c[k] / (W * H), v)
    bpr = ref.algorithmic_bytes(c, W * H) / (W * H)
    survey = {"stanford-bunny.obj": 543, "example_grid.grid": 216, "sdf_6.octree": 335}[name]
    assert abs(bpr - survey) < 1.0


def test_golden_frames_fixture(ref):
    """The committed small frames (tests/golden/make_golden.py) still reproduce."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    data = np.load(os.path.join(HERE, "golden", "frames.npz"))
    index = json.load(open(os.path.join(HERE, "golden", "frames.json")))
    assert len(index) == len(mg.CASES)
    for case, ent in zip(mg.CASES, index):
        assert mg.key(case) == ent["case"]
        name, W, H, mode, pos = case
        c, t = S.ref_frame(name, W, H, mode, pos)
        assert np.array_equal(c, data[ent["color"]]), ent["case"]
        assert np.array_equal(t.view(np.uint32), data[ent["t"]].view(np.uint32)), ent["case"]
        assert ref.fnv1a64_words(c) == ent["fnv1a64"]


def test_sort8_network_sorts(ref):
    """sort8 (raytracing.hpp:188-213) is a full sorting network on distinct keys:
    the oracle's BVH traversal order therefore visits children by ascending t."""
    rng = np.random.default_rng(0)
    # exercise through intersect_rays on a scene: covered by parity; here check the
    # network itself with a pure-python restatement of the comparator list
    pairs = [(0, 1), (2, 3), (4, 5), (6, 7), (0, 2), (1, 3), (4, 6), (5, 7), (1, 2), (5, 6),
             (0, 4), (3, 7), (1, 5), (2, 6), (1, 4), (3, 6), (2, 4), (3, 5), (3, 4)]
    for _ in range(2000):
        t = list(rng.permutation(8).astype(float))
        for a, b in pairs:
            if t[a] > t[b]:
                t[a], t[b] = t[b], t[a]
        assert t == sorted(t)


def test_tprev_semantics(ref):
    """Renderer::draw writes only hit pixels and reads t as tPrev (raytracing.cpp:89-94)."""
    W, H = 96, 54
    s = S.ref_scene("stanford-bunny.obj")
    s.set_plane(False)
    P = S.params("stanford-bunny.obj", W, H, "primary")
    c = np.full((H, W), 0xDEADBEEF, np.uint32)
    t = np.full((H, W), np.inf, np.float32)
    t[:, : W // 2] = 0.5  # nearer than the model: those pixels must stay untouched
    c2, t2, _, _ = s.render(P, W, H, c.copy(), t.copy())
    assert np.all(c2[:, : W // 2] == 0xDEADBEEF)
    assert np.all(t2[:, : W // 2] == 0.5)
    assert np.all(c2[~np.isfinite(t2)] == 0xDEADBEEF)
