"""The viewer's orbit camera and image output, host-only.

rt_camera_* (product, csrc/rt_host.cpp) against the oracle's restatement of
Camera (src/camera.cpp:1-72, src/quaternion.hpp:8-70) over seeded random
interaction sequences -- drags (rotate(-dx, -dy), main.cpp:277-280), wheel
zooms (main.cpp:281-288), target/position resets and up-locks: state and view
matrix bit for bit after every step. LiteMath itself stays unpinned.
"""
import struct
import zlib

import numpy as np
import pytest

import cpuref


def state_words(cam):
    s = cam.state()
    return np.array(list(s.position) + list(s.target) + list(s.orientation) + [s.sensitivity],
                    np.float32), int(s.lock_up), np.array(list(s.locked_up), np.float32)


@pytest.mark.parametrize("seed", range(6))
def test_camera_interaction_matches_reference(rt, seed):
    rng = np.random.default_rng(seed)
    pos = rng.uniform(-3, 3, 3).astype(np.float32)
    up = (0.0, 1.0, 0.0) if seed % 2 == 0 else tuple(rng.normal(size=3).astype(np.float32).tolist())
    cam, ref = rt.Camera(pos, (0.0, 0.0, 0.0), up), cpuref.RefCamera(pos, (0.0, 0.0, 0.0), up)
    for step in range(200):
        op = rng.integers(0, 10)
        if op < 6:
            dx, dy = rng.normal(scale=20.0, size=2).astype(np.float32)
            cam.rotate(-dx, -dy)
            ref.rotate(-dx, -dy)
        elif op == 6:
            w = float(rng.choice([-1.0, 1.0, 2.0]))
            cam.zoom(w)
            ref.zoom(w)
        elif op == 7:
            t = rng.uniform(-0.5, 0.5, 3).astype(np.float32)
            cam.resetTarget(t)
            ref.resetTarget(t)
        elif op == 8:
            p = rng.uniform(-3, 3, 3).astype(np.float32)
            cam.resetPosition(p)
            ref.resetPosition(p)
        else:
            on = bool(rng.integers(0, 2))
            cam.setLockUp(on)
            ref.setLockUp(on)
        w, lk, lu = state_words(cam)
        rs = ref.st
        assert np.array_equal(w.view(np.uint32), rs[:11].view(np.uint32)), (seed, step)
        assert lk == int(rs[11:12].view(np.int32)[0]), (seed, step)
        if lk:
            assert np.array_equal(lu.view(np.uint32), rs[12:15].view(np.uint32)), (seed, step)
        assert np.array_equal(cam.view_inv().view(np.uint32), ref.view_inv.view(np.uint32)), (seed, step)


def test_camera_basis_and_defaults(rt):
    cam = rt.Camera((0.0, 0.0, 2.5))
    assert cam.sensetivity() == np.float32(0.01)
    np.testing.assert_allclose(cam.up(), [0, 1, 0], atol=1e-6)
    np.testing.assert_allclose(cam.forward(), [0, 0, -1], atol=1e-6)
    np.testing.assert_allclose(cam.right(), [1, 0, 0], atol=1e-6)
    d0 = np.linalg.norm(cam.position())
    cam.rotate(-30.0, 0.0)  # a drag orbits: the distance to the target is kept
    assert abs(np.linalg.norm(cam.position()) - d0) < 1e-5
    cam.zoom(1.0)  # one wheel notch moves 1/25 of the distance towards the target
    assert abs(np.linalg.norm(cam.position()) - d0 * 24 / 25) < 1e-5


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, {}
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body) & 0xFFFFFFFF
        chunks.setdefault(typ, b"")
        chunks[typ] += body
        pos += 12 + n
    W, H, depth, ctype = struct.unpack(">IIBB", chunks[b"IHDR"][:10])
    assert (depth, ctype) == (8, 6)
    raw = zlib.decompress(chunks[b"IDAT"])
    rows = np.frombuffer(raw, np.uint8).reshape(H, 1 + 4 * W)
    assert np.all(rows[:, 0] == 0)
    return rows[:, 1:].reshape(H, W, 4)


@pytest.mark.parametrize("W,H", [(1, 1), (3, 2), (300, 200)])
def test_png_roundtrip(rt, tmp_path, W, H):
    rng = np.random.default_rng(W * H)
    fb = rt.FrameBuffer(W, H)
    fb.color[:] = rng.integers(0, 2 ** 32, size=(H, W), dtype=np.uint64).astype(np.uint32)
    fb.save_png(tmp_path / "f.png")
    px = _read_png(tmp_path / "f.png")
    assert np.array_equal(px.view(np.uint32).reshape(H, W), fb.color)  # R in the low byte


def test_png_errors(rt, tmp_path):
    fb = rt.FrameBuffer(2, 2)
    with pytest.raises(rt.RtError):
        fb.save_png(tmp_path / "missing_dir" / "f.png")
