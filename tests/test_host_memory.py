"""Caller host memory at the drop-in boundary.

The reference's frame loop draws into host memory the app owns and reuses
(frameBuf.clear(); renderer.draw(...), src/main.cpp:196-207;
src/raytracing.cpp:89-94). Round 5's GPU suite stopped on an "illegal memory
access" returned by the HIP runtime's own DMA from a caller's pageable buffer
(profiles/r05/gpu_suite_stop_multi_upload.log). The library now never hands a
caller's pageable memory to the runtime's DMA (rtdma / the staging frames), and
rt_host_unpin drains every library stream before it unregisters a range.

These tests drive exactly the failing pattern: a caller buffer pinned,
rendered into, unpinned and freed (munmap), then a NEW buffer mapped over the
same pages (MAP_FIXED, same address) and used pageable, then pinned again --
tPrev and cleared frames through rt_render and rt_multi_render (0,) (the RCCL
one-rank gather) and (0, 0) (peer copies), each bitwise against the oracle's
Renderer::draw over the same buffers."""
import ctypes as C

import numpy as np
import pytest

import scenes as S

pytestmark = pytest.mark.gpu

_libc = C.CDLL(None, use_errno=True)
_libc.mmap.restype = C.c_void_p
_libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
_libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
PROT_RW, MAP_PRIVATE, MAP_ANON, MAP_FIXED = 0x3, 0x02, 0x20, 0x10
PAGE = 4096


def _map(nbytes, at=None):
    """Anonymous pages (at `at` exactly when given) -> address."""
    flags = MAP_PRIVATE | MAP_ANON | (MAP_FIXED if at else 0)
    p = _libc.mmap(C.c_void_p(at) if at else None, nbytes, PROT_RW, flags, -1, 0)
    assert p not in (None, C.c_void_p(-1).value), f"mmap failed (errno {C.get_errno()})"
    if at:
        assert p == at
    return p


def _unmap(p, nbytes):
    assert _libc.munmap(C.c_void_p(p), nbytes) == 0


def _view(p, H, W, dtype):
    buf = (C.c_uint8 * (H * W * 4)).from_address(p)
    return np.frombuffer(buf, dtype=dtype).reshape(H, W)


def _eq(got, want, what):
    assert np.array_equal(got[0], want[0]), f"{what}: {(got[0] != want[0]).sum()} colour px differ"
    assert np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32)), f"{what}: t differs"


def test_reused_pages_after_unpin_and_free(gpu):
    rt = gpu
    L = rt.lib()
    name, W, H = "stanford-bunny.obj", 333, 197
    nbytes = (H * W * 4 + PAGE - 1) // PAGE * PAGE
    sc = S.gpu_scene(name)
    rs = S.ref_scene(name)
    mode = "default"
    S.set_planes(name, mode, sc, rs)
    cams = [(0.0, 0.3, 2.5), (0.8, 0.2, 2.1), (-0.6, 0.4, 2.3)]
    Pg = [S.params(name, W, H, mode, c, "gpu") for c in cams]
    Pr = [S.params(name, W, H, mode, c, "ref") for c in cams]

    def oracle(k, init=None):
        if init is None:
            c, t, _, _ = rs.render(Pr[k], W, H)
            return c, t
        c, t = init[0].copy(), init[1].copy()
        rs.render(Pr[k], W, H, color=c, t=t)
        return c, t

    # the tPrev base frame: camera 0's frame with a sentinel region it never wrote
    base = oracle(0)
    base[0][:20, :30] = 0x11223344

    pc, pt = _map(nbytes), _map(nbytes)
    c, t = _view(pc, H, W, np.uint32), _view(pt, H, W, np.float32)
    rt._lib.check(L.rt_host_pin(C.c_void_p(pc), nbytes))
    rt._lib.check(L.rt_host_pin(C.c_void_p(pt), nbytes))
    try:
        # the range is pinned: pinning an overlapping range is refused
        assert L.rt_host_pin(C.c_void_p(pc + PAGE), PAGE) < 0
        assert b"not unpinned" in L.rt_last_error()
        # 1) pinned: cleared frames stored straight into the caller's pages
        c[:] = 0
        t[:] = np.inf
        sc.render(Pg[0], c, t, cleared=True)
        _eq((c, t), oracle(0), "rt_render cleared, pinned")
        with rt.MultiRenderer(sc, (0, 0)) as mr:
            c[:] = 0
            t[:] = np.inf
            mr.render(Pg[1], c, t, cleared=True)
            _eq((c, t), oracle(1), "rt_multi (0, 0) cleared, pinned")
            c[:], t[:] = base
            mr.render(Pg[1], c, t)
            _eq((c, t), oracle(1, base), "rt_multi (0, 0) tPrev, pinned")
    finally:
        rt._lib.check(L.rt_host_unpin(C.c_void_p(pc)))
        rt._lib.check(L.rt_host_unpin(C.c_void_p(pt)))
    # 2) freed, and new pages mapped at the same addresses: pageable now
    _unmap(pc, nbytes)
    _unmap(pt, nbytes)
    pc, pt = _map(nbytes, pc), _map(nbytes, pt)
    c, t = _view(pc, H, W, np.uint32), _view(pt, H, W, np.float32)
    try:
        c[:], t[:] = base
        sc.render(Pg[1], c, t)
        _eq((c, t), oracle(1, base), "rt_render tPrev, pageable at reused pages")
        for devices in ((0,), (0, 0)):
            with rt.MultiRenderer(sc, devices) as mr:
                c[:], t[:] = base
                mr.render(Pg[2], c, t)
                _eq((c, t), oracle(2, base), f"rt_multi {devices} tPrev, pageable at reused pages")
                c[:] = 0
                t[:] = np.inf
                mr.render(Pg[0], c, t, cleared=True)
                _eq((c, t), oracle(0), f"rt_multi {devices} cleared, pageable at reused pages")
                mr.render(Pg[1], c, t, clear=True)
                _eq((c, t), oracle(1), f"rt_multi {devices} clear, pageable at reused pages")
        # 3) the same pages pinned again
        rt._lib.check(L.rt_host_pin(C.c_void_p(pc), nbytes))
        rt._lib.check(L.rt_host_pin(C.c_void_p(pt), nbytes))
        try:
            c[:], t[:] = base
            sc.render(Pg[2], c, t)
            _eq((c, t), oracle(2, base), "rt_render tPrev, re-pinned")
            with rt.MultiRenderer(sc, (0,)) as mr:
                c[:], t[:] = base
                mr.render(Pg[1], c, t)
                _eq((c, t), oracle(1, base), "rt_multi (0,) tPrev, re-pinned")
                c[:] = 0
                t[:] = np.inf
                mr.render(Pg[2], c, t, cleared=True)
                _eq((c, t), oracle(2), "rt_multi (0,) cleared, re-pinned")
        finally:
            rt._lib.check(L.rt_host_unpin(C.c_void_p(pc)))
            rt._lib.check(L.rt_host_unpin(C.c_void_p(pt)))
    finally:
        _unmap(pc, nbytes)
        _unmap(pt, nbytes)


def test_unpin_of_unknown_range_is_refused(gpu):
    rt = gpu
    L = rt.lib()
    a = np.zeros(4096, np.uint8)
    assert L.rt_host_unpin(C.c_void_p(a.ctypes.data)) < 0
    assert b"not a range pinned" in L.rt_last_error()


def test_rccl_version_reported(gpu):
    """rt_multi's gather runs on whichever librccl the process resolved first
    (torch loads its own); the library reports which."""
    rt = gpu
    v = C.c_int32(0)
    rt._lib.check(rt.lib().rt_multi_rccl_version(C.byref(v)))
    assert v.value >= 20000, v.value  # 2.x
