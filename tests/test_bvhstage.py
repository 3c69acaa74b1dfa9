"""The device BVH builder's host half on the CPU (no GPU): rt_bvhstage.cpp's
parallel stage loop (table build, first minimum over SAH chunks, createNode's
FIFO, triangles_raytracing.cpp:155-225) driven with its device steps emulated
on the host (rtx_bvh_stage_emulate: stage copies, std::sort of each segment,
chunked SAH sweeps, apply, child boxes) must give the host builder's tree,
node for node. The GPU half is compared with the host builder in
test_bvhgpu.py; this pins the stage logic where the GPU is absent and runs
under the sanitizer builds (make sanitize)."""
import ctypes as C

import numpy as np
import pytest

import scenes as S


def canon_emulated(v, i):
    import rtamd
    L = rtamd.lib()
    L.rtx_bvh_stage_emulate.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p,
                                        C.POINTER(C.c_int64)]
    v = np.ascontiguousarray(v, np.float32)
    i = np.ascontiguousarray(i, np.uint32)
    nn = C.c_int64(0)
    rtamd._lib.check(L.rtx_bvh_stage_emulate(v.ctypes.data, len(v), i.ctypes.data, len(i), None, C.byref(nn)))
    canon = np.zeros((nn.value, 52), np.uint32)
    rtamd._lib.check(L.rtx_bvh_stage_emulate(v.ctypes.data, len(v), i.ctypes.data, len(i), canon.ctypes.data,
                                             C.byref(nn)))
    return canon


def canon_host(v, i):
    import rtamd
    L = rtamd.lib()
    rtamd._lib.check(L.rt_set_bvh_builder(1))
    try:
        v = np.ascontiguousarray(v, np.float32)
        i = np.ascontiguousarray(i, np.uint32)
        nn = C.c_int64(0)
        rtamd._lib.check(L.rt_bvh_export(v.ctypes.data, len(v), i.ctypes.data, len(i), None, C.byref(nn), None,
                                         None))
        canon = np.zeros((nn.value, 52), np.uint32)
        rtamd._lib.check(L.rt_bvh_export(v.ctypes.data, len(v), i.ctypes.data, len(i), canon.ctypes.data,
                                         C.byref(nn), None, None))
        return canon
    finally:
        rtamd._lib.check(L.rt_set_bvh_builder(0))


def same_tree(v, i):
    ch, ce = canon_host(v, i), canon_emulated(v, i)
    assert ch.shape == ce.shape, f"{len(ce)} nodes emulated vs {len(ch)} on the host"
    bad = np.flatnonzero((ch != ce).any(1))
    assert bad.size == 0, f"{bad.size} nodes differ, first {bad[:5]}"


@pytest.mark.parametrize("name", ["cube.obj", "spot.obj", "stanford-bunny.obj"])
def test_stage_loop_shipped_meshes(name):
    _, (v, i), _ = S.inputs(name)
    same_tree(v, i)


@pytest.mark.parametrize("seed,ntri,mode", [(1, 1, "rand"), (3, 9, "rand"), (4, 300, "rand"), (6, 64, "same"),
                                            (7, 500, "grid"), (8, 100, "flat"), (9, 30000, "grid"),
                                            (10, 12000, "same"), (11, 40000, "rand"), (13, 3000, "signed0"),
                                            (14, 40000, "signed0")])
def test_stage_loop_edge_meshes(seed, ntri, mode):
    """Tie-heavy meshes, with enough open nodes per stage (> 2048) for the
    stage passes to run in parallel."""
    v4 = S.edge_mesh(seed, ntri, mode)
    same_tree(v4, np.arange(len(v4), dtype=np.uint32))
