"""ctypes binding of the oracle (oracle/cpuref.cpp) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the parity checker / CPU baseline. The product path
(triangles-sdf-cpu-raytracing_amd/) never imports it.

Everything here is host memory + numpy. The C functions restate the reference
hot path; see the header of cpuref.cpp for the file:line map.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CPUREF_LIB: a variant build of the same source (the sanitizer build of `make sanitize`)
_LIB_PATH = os.environ.get("CPUREF_LIB") or os.path.join(_HERE, "_build", "libcpuref.so")
_lib = None


def build(force: bool = False) -> str:
    if os.environ.get("CPUREF_LIB"):
        return _LIB_PATH
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        vp, i64, i32, f32, f64 = C.c_void_p, C.c_int64, C.c_int32, C.c_float, C.c_double
        P = C.POINTER
        L.cpuref_load_obj.restype = vp
        L.cpuref_load_obj.argtypes = [C.c_char_p, C.c_int, P(i64), P(i64)]
        L.cpuref_mesh_copy.argtypes = [vp, vp, vp]
        L.cpuref_mesh_free.argtypes = [vp]
        L.cpuref_scene_mesh.restype = vp
        L.cpuref_scene_mesh.argtypes = [vp, i64, vp, i64]
        L.cpuref_scene_grid.restype = vp
        L.cpuref_scene_grid.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, vp]
        L.cpuref_scene_octree.restype = vp
        L.cpuref_scene_octree.argtypes = [vp, i64]
        L.cpuref_scene_set_plane.argtypes = [vp, C.c_int, vp, f32]
        L.cpuref_scene_free.argtypes = [vp]
        L.cpuref_bvh_node_count.restype = i64
        L.cpuref_bvh_node_count.argtypes = [vp]
        L.cpuref_bvh_export.restype = i64
        L.cpuref_bvh_export.argtypes = [vp, vp, i64]
        L.cpuref_bvh_indices.argtypes = [vp, vp, vp]
        L.cpuref_camera.argtypes = [vp, vp, vp, f32, f32, f32, f32, vp, vp]
        L.cpuref_render.restype = f64
        L.cpuref_render.argtypes = [vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp]
        L.cpuref_intersect_rays.argtypes = [vp, vp, vp, i64, f32, f32, vp, vp, vp, vp]
        L.cpuref_counters.argtypes = [C.c_int, vp]
        L.cpuref_pixel_cost.argtypes = [vp, vp, C.c_int, C.c_int, vp]
        L.cpuref_primary_rays.argtypes = [vp, C.c_int, C.c_int, vp]
        L.cpuref_fnv1a64.restype = C.c_uint64
        L.cpuref_sdf_points.argtypes = [vp, i64, vp, i64, vp, i64, vp, C.c_int]
        L.cpuref_cam_op.argtypes = [vp, C.c_int, vp, vp, vp, f32, f32, vp]
        L.cpuref_fnv1a64.argtypes = [vp, i64]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class RefParams(C.Structure):
    """Same layout as rt_render_params (include/rtamd.h)."""
    _fields_ = [
        ("camera_pos", C.c_float * 3),
        ("view_inv", C.c_float * 16),
        ("proj_inv", C.c_float * 16),
        ("light_pos", C.c_float * 3),
        ("shading_mode", C.c_int32),
        ("enable_shadows", C.c_int32),
        ("enable_reflections", C.c_int32),
        ("reserved", C.c_int32),
    ]


def load_obj(path: str, scale: bool = True):
    """cmesh4::LoadMeshFromObj + loadAndScale (main.cpp:326-343) -> (vpos4 [N,4] f32, idx [M] u32)."""
    L = lib()
    nv, ni = C.c_int64(), C.c_int64()
    h = L.cpuref_load_obj(path.encode(), int(scale), C.byref(nv), C.byref(ni))
    if not h:
        raise IOError(f"cannot load {path}")
    v = np.empty((nv.value, 4), np.float32)
    i = np.empty(ni.value, np.uint32)
    L.cpuref_mesh_copy(h, _p(v), _p(i))
    L.cpuref_mesh_free(h)
    return v, i


def camera_matrices(pos, target=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0), fovy=45.0, aspect=16 / 9,
                    znear=0.01, zfar=100.0):
    """(view_inv, proj_inv) as column-major float32[16] (main.cpp:198-201, raytracing.cpp:73-75)."""
    vi = np.zeros(16, np.float32)
    pi = np.zeros(16, np.float32)
    a = lambda x: np.asarray(x, np.float32)
    p, t, u = a(pos), a(target), a(up)
    lib().cpuref_camera(_p(p), _p(t), _p(u), fovy, aspect, znear, zfar, _p(vi), _p(pi))
    return vi, pi


def make_params(cam_pos, view_inv, proj_inv, light=(2.0, 2.0, 2.0), mode=0, shadows=True,
                reflections=True) -> RefParams:
    P = RefParams()
    P.camera_pos[:] = [float(x) for x in cam_pos]
    P.view_inv[:] = [float(x) for x in view_inv]
    P.proj_inv[:] = [float(x) for x in proj_inv]
    P.light_pos[:] = [float(x) for x in light]
    P.shading_mode = int(mode)
    P.enable_shadows = int(bool(shadows))
    P.enable_reflections = int(bool(reflections))
    return P


class RefScene:
    def __init__(self, handle):
        self.h = handle

    @staticmethod
    def mesh(vpos4, idx):
        vpos4 = np.ascontiguousarray(vpos4, np.float32)
        idx = np.ascontiguousarray(idx, np.uint32)
        return RefScene(lib().cpuref_scene_mesh(_p(vpos4), len(vpos4), _p(idx), len(idx)))

    @staticmethod
    def grid(size, values):
        values = np.ascontiguousarray(values, np.float32)
        return RefScene(lib().cpuref_scene_grid(int(size[0]), int(size[1]), int(size[2]), _p(values)))

    @staticmethod
    def octree(nodes_bytes: np.ndarray):
        nb = np.ascontiguousarray(nodes_bytes)
        return RefScene(lib().cpuref_scene_octree(_p(nb), nb.nbytes // 36))

    def set_plane(self, enabled=True, normal=(0.0, 1.0, 0.0), offset=-1.0):
        n = np.asarray(normal, np.float32)
        lib().cpuref_scene_set_plane(self.h, int(enabled), _p(n), float(offset))

    def bvh_export(self):
        L = lib()
        n = L.cpuref_bvh_node_count(self.h)
        out = np.zeros((n, 52), np.uint32)
        m = L.cpuref_bvh_export(self.h, _p(out), n)
        return out[:m]

    def bvh_indices(self, n_idx):
        idx = np.zeros(n_idx, np.uint32)
        tri = np.zeros(n_idx // 3, np.uint32)
        lib().cpuref_bvh_indices(self.h, _p(idx), _p(tri))
        return idx, tri

    def render(self, params: RefParams, W: int, H: int, color=None, t=None, prim=False, rows=None,
               threads: int = 0):
        """Renderer::draw into (color u32[H,W], t f32[H,W]); returns (color, t, prim|None, ms)."""
        if color is None:
            color = np.zeros((H, W), np.uint32)
        if t is None:
            t = np.full((H, W), np.inf, np.float32)
        pr = np.full((H, W), -1, np.int64) if prim else None
        r0, r1 = (0, H) if rows is None else rows
        ms = lib().cpuref_render(self.h, C.byref(params), _p(color), _p(t), _p(pr), W, H, r0, r1,
                                 threads, None)
        return color, t, pr, ms

    def pixel_cost(self, params: RefParams, W: int, H: int):
        """Per-pixel primary-ray work (node visits + leaf visits + tests/steps)."""
        cost = np.zeros((H, W), np.int32)
        lib().cpuref_pixel_cost(self.h, C.byref(params), W, H, _p(cost))
        return cost

    def intersect_rays(self, o, d, tnear=0.01, tfar=100.0):
        o = np.ascontiguousarray(o, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        n = len(o)
        hit = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        nrm = np.zeros((n, 3), np.float32)
        prim = np.zeros(n, np.int64)
        lib().cpuref_intersect_rays(self.h, _p(o), _p(d), n, tnear, tfar, _p(hit), _p(t), _p(nrm),
                                    _p(prim))
        return hit, t, nrm, prim

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.cpuref_scene_free(self.h)
            self.h = None


def primary_rays(params: RefParams, W: int, H: int) -> np.ndarray:
    """World-space primary ray directions [H, W, 3] (Renderer::draw ray generation)."""
    d = np.zeros((H, W, 3), np.float32)
    lib().cpuref_primary_rays(C.byref(params), W, H, _p(d))
    return d


def fnv1a64_words(color: np.ndarray) -> str:
    """Word-wise FNV-1a-64 over the colour buffer in y*W+x order."""
    c = np.ascontiguousarray(color, np.uint32).ravel()
    return f"{lib().cpuref_fnv1a64(_p(c), c.size):016x}"


COUNTER_NAMES = ("bvh_inner", "bvh_leaf", "bvh_tri", "grid_sdf", "oct_node", "oct_leaf", "oct_step",
                 "oct_normal", "rays")


def counters(reset: bool = True) -> dict:
    """Work counters of cpuref_render calls since the last reset (SURVEY 8(d) byte model)."""
    out = np.zeros(len(COUNTER_NAMES), np.int64)
    lib().cpuref_counters(int(reset), _p(out))
    return dict(zip(COUNTER_NAMES, out.tolist()))


def algorithmic_bytes(c: dict, pixels: int) -> int:
    """Bytes the reference's data layout makes one frame touch:
    BVH: 200 B / inner node visit, 8 B / leaf visit, 60 B / triangle test;
    grid: 32 B / sdf evaluation; octree: 4 B / node visit, 32 B / leaf visit,
    32 B / nodeSDF step, 32 B / nodeNormal; + 8 B / pixel framebuffer (colour + t)."""
    return int(200 * c["bvh_inner"] + 8 * c["bvh_leaf"] + 60 * c["bvh_tri"] + 32 * c["grid_sdf"]
               + 4 * c["oct_node"] + 32 * c["oct_leaf"] + 32 * c["oct_step"] + 32 * c["oct_normal"]
               + 8 * pixels)


# ------------------------------------------------------------ mesh -> SDF --
# Definition of the SDF construction the GPU generator (rt_sdf_mesh_*) must
# reproduce; the reference has none, so this is
# "parity unpinned" against the reference and pins the GPU path only.

def sdf_points(vpos4, idx, p3, threads: int = 8) -> np.ndarray:
    """Signed distance at points p3 [n,3], brute force over all triangles."""
    v = np.ascontiguousarray(vpos4, np.float32)
    i = np.ascontiguousarray(idx, np.uint32)
    p = np.ascontiguousarray(p3, np.float32).reshape(-1, 3)
    out = np.empty(len(p), np.float32)
    rc = lib().cpuref_sdf_points(_p(v), len(v), _p(i), len(i), _p(p), len(p), _p(out), int(threads))
    if rc != 0:
        raise ValueError("cpuref_sdf_points failed")
    return out


def lattice_points(size) -> np.ndarray:
    """Sample (i,j,k) of a size[0] x size[1] x size[2] lattice at 2*i/(n-1) - 1
    per axis (f32 ops: mul, div, sub), in the SDFGrid index order
    (x*sy+y)*sz+z (grid_raytracing.hpp:13-15)."""
    axes = [np.float32(2.0) * np.arange(n, dtype=np.float32) / np.float32(n - 1) - np.float32(1.0)
            for n in (int(size[0]), int(size[1]), int(size[2]))]
    X, Y, Z = np.meshgrid(*axes, indexing="ij")
    return np.stack([X.ravel(), Y.ravel(), Z.ravel()], 1)


def sdf_octree(vpos4, idx, depth: int, threads: int = 8) -> np.ndarray:
    """Sparse SDF octree in the reference's 36-byte node format (octree_raytracing.hpp:8-18):
    top-down from the root [-1,1]^3; a node at depth d < depth is refined iff
    |sdf(centre)| <= sqrt(3) * 2^-d (f32 1.7320508 * 2^-d); refined nodes hold
    zeros and childrenOffset; unrefined nodes are empty leaves (values 1000);
    depth-`depth` nodes are leaves with the SDF at their 8 corners,
    values[(x<<2)+(y<<1)+z] (octree_raytracing.hpp:35-37). BFS order, the 8
    children of a node contiguous, child id (x<<2)|(y<<1)|z (divide_box_8)."""
    levels = [[(0, 0, 0)]]
    refine = []
    for d in range(depth):
        cur = levels[d]
        half = np.float32(2.0 ** -d)
        c = np.array(cur, np.int64)
        centres = (2 * c + 1).astype(np.float32) * half - np.float32(1.0)
        s = sdf_points(vpos4, idx, centres, threads)
        r = np.abs(s) <= np.float32(1.7320508) * half
        refine.append(r)
        nxt = []
        for (x, y, z), rr in zip(cur, r):
            if rr:
                for k in range(8):
                    nxt.append((2 * x + (k >> 2), 2 * y + ((k >> 1) & 1), 2 * z + (k & 1)))
        levels.append(nxt)
    leaves = np.array(levels[depth], np.int64).reshape(-1, 3)
    size = np.float32(2.0 ** (1 - depth))
    corners = np.array([(k >> 2, (k >> 1) & 1, k & 1) for k in range(8)], np.int64)
    pts = ((leaves[:, None, :] + corners[None]).astype(np.float32) * size - np.float32(1.0)).reshape(-1, 3)
    cv = sdf_points(vpos4, idx, pts, threads).reshape(-1, 8) if len(pts) else np.zeros((0, 8), np.float32)
    total = sum(len(L) for L in levels)
    vals = np.zeros((total, 8), np.float32)
    off = np.zeros(total, np.uint32)
    base = 0
    for d in range(depth + 1):
        n = len(levels[d])
        child = base + n
        for j in range(n):
            if d == depth:
                vals[base + j] = cv[j]
            elif refine[d][j]:
                off[base + j] = child
                child += 8
            else:
                vals[base + j] = 1000.0
        base += n
    rec = np.zeros((total, 36), np.uint8)
    rec[:, :32] = vals.view(np.uint8).reshape(total, 32)
    rec[:, 32:] = off.view(np.uint8).reshape(total, 4)
    return rec.ravel()


def subdivide(vpos4, idx, levels: int):
    """Midpoint subdivision: per triangle (a,b,c) with edge midpoints ab, bc, ca
    (created in that order on first use, value (u+v)*0.5 on all 4 components)
    -> (a,ab,ca), (ab,b,bc), (ca,bc,c), (ab,bc,ca)."""
    V = [tuple(r) for r in np.asarray(vpos4, np.float32)]
    I = np.asarray(idx, np.uint32).tolist()
    half = np.float32(0.5)
    for _ in range(levels):
        mid = {}
        J = []

        def m(a, b):
            k = (a, b) if a < b else (b, a)
            r = mid.get(k)
            if r is None:
                r = len(V)
                V.append(tuple((np.float32(V[a][c]) + np.float32(V[b][c])) * half for c in range(4)))
                mid[k] = r
            return r
        for t in range(len(I) // 3):
            a, b, c = I[3 * t:3 * t + 3]
            ab, bc, ca = m(a, b), m(b, c), m(c, a)
            J += [a, ab, ca, ab, b, bc, ca, bc, c, ab, bc, ca]
        I = J
    return np.array(V, np.float32).reshape(-1, 4), np.array(I, np.uint32)


# ------------------------------------------------------------ orbit camera --
class RefCamera:
    """The reference Camera (camera.cpp:1-72) over an rt_camera_state-shaped
    array of 15 words; every op returns inverse4x4(lookAtMatrix())."""

    def __init__(self, pos, target=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0)):
        self.st = np.zeros(15, np.float32)
        self.view_inv = self._op(0, pos, target, up)

    def _op(self, op, a=None, b=None, c=None, x=0.0, y=0.0):
        arr = [None if v is None else np.ascontiguousarray(v, np.float32) for v in (a, b, c)]
        vi = np.zeros(16, np.float32)
        lib().cpuref_cam_op(_p(self.st), op, *[_p(v) for v in arr], float(x), float(y), _p(vi))
        return vi

    def rotate(self, dx, dy):
        self.view_inv = self._op(1, x=dx, y=dy)

    def resetPosition(self, p):
        self.view_inv = self._op(2, a=p)

    def resetTarget(self, t):
        self.view_inv = self._op(3, a=t)

    def setLockUp(self, on):
        self.view_inv = self._op(4, x=1.0 if on else 0.0)

    def zoom(self, wheel):
        self.view_inv = self._op(5, x=wheel)


def save_obj_text(vpos4, idx, vnorm4=None, vtex2=None) -> bytes:
    """cmesh4::SaveMeshToObj (src/core/mesh.cpp:14-63) restated: std::to_string
    is printf "%f" of the float promoted to double; section order v, vt, vn,
    "s off", faces "f i/i/i" (1-based). Missing normals / texture coordinates
    take fix_missing's defaults (mesh.cpp:143-160)."""
    v = np.asarray(vpos4, np.float32).reshape(-1, 4)
    n = np.tile(np.float32([0, 0, 1, 0]), (len(v), 1)) if vnorm4 is None else np.asarray(vnorm4, np.float32)
    t = np.zeros((len(v), 2), np.float32) if vtex2 is None else np.asarray(vtex2, np.float32)
    f = lambda x: "%f" % float(x)
    out = ["# obj file created by custom obj loader\n", "o MainModel\n"]
    out += ["v %s %s %s\n" % (f(p[0]), f(p[1]), f(p[2])) for p in v]
    out += ["vt %s %s\n" % (f(p[0]), f(p[1])) for p in t.reshape(-1, 2)]
    out += ["vn %s %s %s\n" % (f(p[0]), f(p[1]), f(p[2])) for p in n.reshape(-1, 4)]
    out.append("s off\n")
    ii = np.asarray(idx, np.uint32).reshape(-1, 3).astype(np.int64) + 1
    out += ["f %d/%d/%d %d/%d/%d %d/%d/%d\n" % (a, a, a, b, b, b, c, c, c) for a, b, c in ii]
    return "".join(out).encode()
