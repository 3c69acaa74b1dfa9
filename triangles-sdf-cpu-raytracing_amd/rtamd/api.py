"""Python mirror of the reference's render surface, over the C ABI.

Reference interface (iMacsimus/Triangles-SDF-CPU-RayTracing @ 2025-07-04):
  FrameBuffer {color, t}; clear()             src/raytracing.hpp:9-20
  ShadingMode {Normal, Lambert, Color}         src/raytracing.hpp:99
  Renderer {lightPos, enableShadows, enableReflections, shadingMode};
      float draw(scene, frameBuffer, camera, projInv)  src/raytracing.hpp:101-117
  IScene::intersect(rayPos, rayDir, tNear, tFar) -> HitInfo  src/raytracing.hpp:75-81
  BVHBuilder::perform(SimpleMesh)               src/triangles_raytracing.hpp:38-67
  SDFGrid / loadSDFGrid                         src/grid_raytracing.hpp:10-22
  SDFOctree / loadSDFOctree                     src/octree_raytracing.hpp:20-49
  Plane(normal, offset), SceneUnion(a, b)       src/raytracing.hpp:83-97, 119-186
  Camera(position, target, up)                  src/camera.hpp:7-61
  cmesh4::LoadMeshFromObj + loadAndScale        src/core/mesh.cpp:178, src/main.cpp:326-343

Every call goes to the HIP implementation in librtamd.so; errors raise RtError.
"""
from __future__ import annotations

import ctypes as C
import enum
from dataclasses import dataclass

import numpy as np

from ._lib import (RT_FLAG_CLEAR, RT_FLAG_HITS_ONLY, CameraState, RenderParams, RtError, Tile, check, lib)

__all__ = [
    "ShadingMode", "SimpleMesh", "FrameBuffer", "Camera", "Renderer", "HitInfo", "IScene",
    "BVHBuilder", "SDFGrid", "SDFOctree", "Plane", "SceneUnion", "load_mesh_from_obj",
    "load_sdf_grid", "load_sdf_octree", "camera_matrices", "render_params", "RtError",
    "RT_FLAG_CLEAR", "Tile", "device_count", "SDFMesh", "subdivide_mesh", "save_mesh_to_obj",
    "MultiRenderer",
]


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def device_count() -> int:
    return lib().rt_device_count()


class ShadingMode(enum.IntEnum):
    Normal = 0
    Lambert = 1
    Color = 2


@dataclass
class SimpleMesh:
    """cmesh4::SimpleMesh positions + indices (src/core/mesh.h:15-55)."""
    vPos4f: np.ndarray      # float32 [N, 4]
    indices: np.ndarray     # uint32 [3*T]

    def TrianglesNum(self) -> int:
        return len(self.indices) // 3


def load_mesh_from_obj(path: str, scale: bool = True) -> SimpleMesh:
    """LoadMeshFromObj (+ loadAndScale when scale=True, as main.cpp does for every .obj)."""
    L = lib()
    nv, ni = C.c_int64(0), C.c_int64(0)
    check(L.rt_load_obj(path.encode(), int(scale), None, C.byref(nv), None, C.byref(ni)))
    v = np.empty((nv.value, 4), np.float32)
    i = np.empty(ni.value, np.uint32)
    check(L.rt_load_obj(path.encode(), int(scale), _p(v), C.byref(nv), _p(i), C.byref(ni)))
    return SimpleMesh(v, i)


def save_mesh_to_obj(path: str, mesh: SimpleMesh, normals=None, texcoords=None):
    """cmesh4::SaveMeshToObj (src/core/mesh.cpp:14-63), byte for byte."""
    v = np.ascontiguousarray(mesh.vPos4f, np.float32)
    i = np.ascontiguousarray(mesh.indices, np.uint32)
    n = None if normals is None else np.ascontiguousarray(normals, np.float32)
    t = None if texcoords is None else np.ascontiguousarray(texcoords, np.float32)
    check(lib().rt_save_obj(str(path).encode(), _p(v), len(v), _p(i), len(i), _p(n), _p(t)))


def load_sdf_grid(path: str):
    """loadSDFGrid -> (size uint32[3], values float32[sx*sy*sz])."""
    L = lib()
    size = np.zeros(3, np.uint32)
    check(L.rt_load_grid(path.encode(), _p(size), None))
    vals = np.empty(int(size[0]) * int(size[1]) * int(size[2]), np.float32)
    check(L.rt_load_grid(path.encode(), _p(size), _p(vals)))
    return size, vals


def load_sdf_octree(path: str) -> np.ndarray:
    """loadSDFOctree -> raw nodes, uint8 [count*36] (SDFOctreeNode, 36 B each)."""
    L = lib()
    n = C.c_int64(0)
    check(L.rt_load_octree(path.encode(), C.byref(n), None))
    buf = np.empty(n.value * 36, np.uint8)
    check(L.rt_load_octree(path.encode(), C.byref(n), _p(buf)))
    return buf


def camera_matrices(position, target=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0), fovy=45.0,
                    aspect=16.0 / 9.0, znear=0.01, zfar=100.0):
    """(view_inv, proj_inv) column-major float32[16]:
    inverse4x4(Camera(position, target, up).lookAtMatrix()) and
    inverse4x4(perspectiveMatrix(fovy, aspect, znear, zfar)) (main.cpp:198-201)."""
    # keep the argument arrays alive across the call (a temporary's buffer may be freed)
    pos = np.array(position, np.float32)
    tgt = np.array(target, np.float32)
    upv = np.array(up, np.float32)
    vi = np.zeros(16, np.float32)
    pi = np.zeros(16, np.float32)
    check(lib().rt_camera(_p(pos), _p(tgt), _p(upv), fovy, aspect, znear, zfar, _p(vi), _p(pi)))
    return vi, pi


def render_params(cam_pos, view_inv, proj_inv, light=(2.0, 2.0, 2.0), mode=ShadingMode.Lambert,
                  shadows=True, reflections=True) -> RenderParams:
    P = RenderParams()
    P.camera_pos[:] = [float(x) for x in cam_pos]
    P.view_inv[:] = [float(x) for x in view_inv]
    P.proj_inv[:] = [float(x) for x in proj_inv]
    P.light_pos[:] = [float(x) for x in light]
    P.shading_mode = int(mode)
    P.enable_shadows = int(bool(shadows))
    P.enable_reflections = int(bool(reflections))
    P.reserved = 0
    return P


class Camera:
    """Camera (src/camera.hpp:7-61, src/camera.cpp:1-72): the viewer's orbit
    camera -- position, target and an orientation quaternion -- through the
    host-side C ABI (rt_camera_*), bit-identical to the reference's float math."""

    def __init__(self, position=(0.0, 0.0, 2.5), target=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0)):
        self._s = CameraState()
        p, t, u = (np.ascontiguousarray(x, np.float32) for x in (position, target, up))
        check(lib().rt_camera_init(_p(p), _p(t), _p(u), C.byref(self._s)))

    def position(self):
        return np.array(self._s.position, np.float32)

    def target(self):
        return np.array(self._s.target, np.float32)

    def _basis(self):
        u, r, f = (np.zeros(3, np.float32) for _ in range(3))
        check(lib().rt_camera_basis(C.byref(self._s), _p(u), _p(r), _p(f)))
        return u, r, f

    def up(self):
        return self._basis()[0]

    def right(self):
        return self._basis()[1]

    def forward(self):
        return self._basis()[2]

    def sensetivity(self) -> float:  # (sic) camera.hpp:38
        return float(self._s.sensitivity)

    def rotate(self, dx: float, dy: float):
        """Camera::rotate (camera.cpp:5-20); the viewer calls rotate(-dx, -dy) on a drag."""
        check(lib().rt_camera_rotate(C.byref(self._s), float(dx), float(dy)))

    def resetPosition(self, position):
        p = np.ascontiguousarray(position, np.float32)
        check(lib().rt_camera_reset_position(C.byref(self._s), _p(p)))

    def resetTarget(self, target):
        t = np.ascontiguousarray(target, np.float32)
        check(lib().rt_camera_reset_target(C.byref(self._s), _p(t)))

    def setLockUp(self, on: bool):
        check(lib().rt_camera_set_lock_up(C.byref(self._s), int(bool(on))))

    def isLockedUp(self) -> bool:
        return bool(self._s.lock_up)

    def zoom(self, wheel: float):
        """The viewer's mouse wheel (main.cpp:281-288)."""
        check(lib().rt_camera_zoom(C.byref(self._s), float(wheel)))

    def view_inv(self):
        """inverse4x4(lookAtMatrix()), column-major float32[16]."""
        vi = np.zeros(16, np.float32)
        check(lib().rt_camera_view_inverse(C.byref(self._s), _p(vi)))
        return vi

    def state(self) -> CameraState:
        return self._s


class FrameBuffer:
    """FrameBuffer {Image2D<uint32_t> color; Image2D<float> t;} (raytracing.hpp:9-20)."""

    def __init__(self, width: int, height: int):
        self.resize(width, height)

    def resize(self, width: int, height: int):
        self.color = np.zeros((height, width), np.uint32)
        self.t = np.full((height, width), np.inf, np.float32)

    def clear(self):
        self.color.fill(0)
        self.t.fill(np.inf)

    @property
    def width(self):
        return self.color.shape[1]

    @property
    def height(self):
        return self.color.shape[0]

    def save_png(self, path: str):
        """The colour buffer as an 8-bit RGBA PNG (rt_write_png)."""
        c = np.ascontiguousarray(self.color, np.uint32)
        check(lib().rt_write_png(str(path).encode(), _p(c), self.width, self.height))


@dataclass
class HitInfo:
    """HitInfo (raytracing.hpp:67-73) for a batch; prim is this build's primitive id."""
    hitten: np.ndarray
    t: np.ndarray
    normal: np.ndarray
    prim: np.ndarray


class IScene:
    """A scene resident on the current HIP device (one rt_scene handle)."""

    _h = None
    _plane = None

    def _handle(self):
        if self._h is None:
            raise RtError("scene not built")
        return self._h

    def set_plane(self, plane: "Plane | None"):
        self._plane = plane
        if plane is None:
            check(lib().rt_scene_set_plane(self._handle(), 0, None, 0.0))
        else:
            n = np.asarray(plane.normal, np.float32)
            check(lib().rt_scene_set_plane(self._handle(), 1, _p(n), float(plane.offset)))

    def intersect(self, ray_pos, ray_dir, tNear=0.01, tFar=100.0) -> HitInfo:
        """IScene::intersect for a batch of rays ([N,3] origins and directions)."""
        o = np.ascontiguousarray(np.asarray(ray_pos, np.float32).reshape(-1, 3))
        d = np.ascontiguousarray(np.asarray(ray_dir, np.float32).reshape(-1, 3))
        n = len(o)
        hit = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        nrm = np.zeros((n, 3), np.float32)
        prim = np.zeros(n, np.int64)
        check(lib().rt_intersect_rays(self._handle(), _p(o), _p(d), n, tNear, tFar, _p(hit), _p(t),
                                      _p(nrm), _p(prim)))
        return HitInfo(hit.astype(bool), t, nrm, prim)

    def render(self, params: RenderParams, color: np.ndarray, t: np.ndarray, clear: bool = False,
               cleared: bool = False):
        """Renderer::draw on host buffers; returns the kernel time in ms.
        clear: FrameBuffer::clear() + draw fused (every pixel written);
        cleared: the buffers already hold a cleared frame (only the hits'
        bounding box is copied back); neither: t is read as tPrev."""
        H, W = color.shape
        assert color.dtype == np.uint32 and t.dtype == np.float32 and t.shape == color.shape
        assert color.flags.c_contiguous and t.flags.c_contiguous
        ms = C.c_float(0.0)
        flags = (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY) if cleared else RT_FLAG_CLEAR if clear else 0
        check(lib().rt_render(self._handle(), C.byref(params), _p(color), _p(t), W, H, flags, C.byref(ms)))
        return ms.value

    def render_device(self, params: RenderParams, color_ptr: int, t_ptr: int, W: int, H: int,
                      clear: bool = True, tile: Tile | None = None, stream: int | None = None,
                      flags: int = 0):
        """Renderer::draw into device buffers (e.g. torch tensors' data_ptr()).
        `flags` adds RT_FLAG_TILE_NATURAL / RT_FLAG_HITS_ONLY (include/rtamd.h)."""
        check(lib().rt_render_device(self._handle(), C.byref(params), C.c_void_p(color_ptr),
                                     C.c_void_p(t_ptr), W, H, (RT_FLAG_CLEAR if clear else 0) | flags,
                                     C.byref(tile) if tile is not None else None,
                                     C.c_void_p(stream) if stream else None))

    def render_device_frames(self, params_list, color_ptrs, t_ptrs, W: int, H: int, flags: int,
                             tile: Tile | None = None, stream: int | None = None):
        """rt_render_device_frames: up to 16 frames per launch, one host call."""
        n = len(params_list)
        arr = (RenderParams * n)(*params_list)
        cp = (C.c_void_p * n)(*color_ptrs)
        tp = (C.c_void_p * n)(*t_ptrs)
        check(lib().rt_render_device_frames(self._handle(), arr, n, cp, tp, W, H, flags,
                                            C.byref(tile) if tile is not None else None,
                                            C.c_void_p(stream) if stream else None))

    def bench_frames(self, params_list, W: int, H: int, clear: bool = True):
        arr = (RenderParams * len(params_list))(*params_list)
        mean, total = C.c_float(0.0), C.c_float(0.0)
        check(lib().rt_bench_frames(self._handle(), arr, len(params_list), W, H,
                                    RT_FLAG_CLEAR if clear else 0, C.byref(mean), C.byref(total)))
        return mean.value, total.value

    COUNTER_NAMES = ("bvh_inner", "bvh_leaf", "bvh_tri", "grid_sdf", "oct_node", "oct_leaf",
                     "oct_step", "oct_normal", "rays")

    def count_work(self, params_list, W: int, H: int, clear: bool = True,
                   tile: Tile | None = None) -> dict:
        """Reference-traversal work counters over the given frames (rt_count_work)."""
        arr = (RenderParams * len(params_list))(*params_list)
        out = np.zeros(9, np.int64)
        check(lib().rt_count_work(self._handle(), arr, len(params_list), W, H,
                                  RT_FLAG_CLEAR if clear else 0,
                                  C.byref(tile) if tile is not None else None, _p(out)))
        return dict(zip(self.COUNTER_NAMES, out.tolist()))

    @staticmethod
    def algorithmic_bytes(c: dict, pixels: int) -> int:
        """Bytes the reference's data layout touches for this work:
        BVH 200 B / inner-node visit (Box8 + realCount + offset), 8 B / leaf visit,
        60 B / triangle test (3 indices + 3 float4 vertices); grid 32 B / sdf
        evaluation (8 taps); octree 4 B / node visit, 32 B / leaf visit, 32 B /
        march step, 32 B / normal; + 8 B / pixel of framebuffer (colour + t)."""
        return int(200 * c["bvh_inner"] + 8 * c["bvh_leaf"] + 60 * c["bvh_tri"] + 32 * c["grid_sdf"]
                   + 4 * c["oct_node"] + 32 * c["oct_leaf"] + 32 * c["oct_step"]
                   + 32 * c["oct_normal"] + 8 * pixels)

    def device_bytes(self) -> int:
        return int(lib().rt_scene_device_bytes(self._handle()))

    def tree_stats(self):
        n, i, d = C.c_int64(0), C.c_int64(0), C.c_int32(0)
        check(lib().rt_scene_bvh_stats(self._handle(), C.byref(n), C.byref(i), C.byref(d)))
        return n.value, i.value, d.value

    def close(self):
        if self._h is not None:
            check(lib().rt_scene_destroy(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BVHBuilder(IScene):
    """BVHBuilder::perform(mesh): host SAH BVH8 build + device upload."""

    def __init__(self, mesh: SimpleMesh | None = None):
        if mesh is not None:
            self.perform(mesh)

    def perform(self, mesh: SimpleMesh):
        self.close()
        v = np.ascontiguousarray(mesh.vPos4f, np.float32)
        i = np.ascontiguousarray(mesh.indices, np.uint32)
        h = C.c_void_p()
        check(lib().rt_scene_create_mesh(_p(v), len(v), _p(i), len(i), C.byref(h)))
        self._h = h
        return self


class SDFGrid(IScene):
    def __init__(self, size, values):
        size = np.ascontiguousarray(size, np.uint32)
        values = np.ascontiguousarray(values, np.float32)
        h = C.c_void_p()
        check(lib().rt_scene_create_grid(_p(size), _p(values), C.byref(h)))
        self._h = h
        self.size = size


class SDFOctree(IScene):
    def __init__(self, nodes36: np.ndarray):
        nodes36 = np.ascontiguousarray(nodes36).view(np.uint8)
        h = C.c_void_p()
        check(lib().rt_scene_create_octree(_p(nodes36), nodes36.nbytes // 36, C.byref(h)))
        self._h = h


@dataclass
class Plane:
    """Plane(normal, offset): the plane dot(p, normal) = offset (raytracing.hpp:121-124)."""
    normal: tuple = (0.0, 1.0, 0.0)
    offset: float = 0.0


class SceneUnion:
    """SceneUnion(scene, plane) (raytracing.hpp:83-97). The second operand must be a Plane."""

    def __init__(self, first: IScene, second: Plane):
        if not isinstance(second, Plane):
            raise RtError("SceneUnion supports (scene, Plane) as in the reference application")
        self.first, self.second = first, second


class Renderer:
    """Renderer (raytracing.hpp:101-117)."""

    def __init__(self):
        self.lightPos = (2.0, 2.0, 2.0)  # main.cpp:60
        self.enableShadows = True
        self.enableReflections = True
        self.shadingMode = ShadingMode.Lambert

    def draw(self, scene, frame_buffer: FrameBuffer, camera: Camera, proj_inv) -> float:
        """Renderer::draw: renders into frame_buffer (t read as tPrev, written on hit)."""
        if isinstance(scene, SceneUnion):
            base = scene.first
            base.set_plane(scene.second)
        else:
            base = scene
            base.set_plane(None)
        P = render_params(camera.position(), camera.view_inv(), proj_inv, self.lightPos,
                          self.shadingMode, self.enableShadows, self.enableReflections)
        return base.render(P, frame_buffer.color, frame_buffer.t, clear=False)


# ------------------------------------ one process, several GPUs (rt_multi) --
class MultiRenderer:
    """Renderer::draw over several GPUs of one process (rt_multi_*): the
    scene (on devices[0]) is replicated on the other devices, the frame is cut
    into row bands (band b -> slot b mod n, as the reference's draw splits rows
    over OpenMP threads, raytracing.cpp:77-96), each slot renders its bands on
    its own stream and one gather per frame (RCCL ncclGather for distinct
    devices, peer copies when a device repeats) assembles it on devices[0]."""

    RCCL, PEER_COPY = 1, 2

    def __init__(self, scene: IScene, devices, band_rows: int = 8):
        devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        h = C.c_void_p()
        check(lib().rt_multi_create(scene._handle(), devs, len(devices), int(band_rows), C.byref(h)))
        self._h = h
        self.scene = scene  # the root scene must outlive the handle

    def info(self):
        """-> (slots, exchange (MultiRenderer.RCCL / PEER_COPY), band_rows)."""
        n, x, b = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        check(lib().rt_multi_info(self._h, C.byref(n), C.byref(x), C.byref(b)))
        return n.value, x.value, b.value

    def render(self, params: RenderParams, color: np.ndarray, t: np.ndarray, clear: bool = False,
               cleared: bool = False) -> float:
        """The same contract as IScene.render (host buffers); returns the device
        time from the first launch to the assembled frame, in ms."""
        H, W = color.shape
        assert color.dtype == np.uint32 and t.dtype == np.float32 and t.shape == color.shape
        assert color.flags.c_contiguous and t.flags.c_contiguous
        ms = C.c_float(0.0)
        flags = (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY) if cleared else RT_FLAG_CLEAR if clear else 0
        check(lib().rt_multi_render(self._h, C.byref(params), _p(color), _p(t), W, H, flags, C.byref(ms)))
        return ms.value

    def render_device_frames(self, params_list, color_ptrs, t_ptrs, W: int, H: int,
                             stream: int | None = None):
        """Frames into device buffers on devices[0], stream-ordered on `stream`."""
        n = len(params_list)
        arr = (RenderParams * n)(*params_list)
        cp = (C.c_void_p * n)(*color_ptrs)
        tp = (C.c_void_p * n)(*t_ptrs)
        check(lib().rt_multi_render_device_frames(self._h, arr, n, cp, tp, W, H, RT_FLAG_CLEAR,
                                                  C.c_void_p(stream) if stream else None))

    def close(self):
        if getattr(self, "_h", None):
            check(lib().rt_multi_destroy(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --------------------------------------------- mesh -> SDF --
class SDFMesh:
    """A triangle mesh prepared on the GPU for signed-distance queries
    (rt_sdf_mesh_*): point queries, SDFGrid lattices and sparse SDFOctrees in
    the reference's file formats (grid_raytracing.cpp:127-134,
    octree_raytracing.cpp:8-16). Generates the config-3/4 stand-ins."""

    def __init__(self, mesh: SimpleMesh):
        v = np.ascontiguousarray(mesh.vPos4f, np.float32)
        i = np.ascontiguousarray(mesh.indices, np.uint32)
        h = C.c_void_p()
        check(lib().rt_sdf_mesh_create(_p(v), len(v), _p(i), len(i), C.byref(h)))
        self._h = h

    def points(self, p3) -> np.ndarray:
        p3 = np.ascontiguousarray(p3, np.float32).reshape(-1, 3)
        out = np.empty(len(p3), np.float32)
        check(lib().rt_sdf_mesh_points(self._h, _p(p3), len(p3), _p(out)))
        return out

    def grid(self, size):
        """-> (size uint32[3], values float32[sx*sy*sz]) as SDFGrid holds them."""
        size = np.ascontiguousarray(np.broadcast_to(np.asarray(size, np.uint32), (3,)))
        vals = np.empty(int(size[0]) * int(size[1]) * int(size[2]), np.float32)
        check(lib().rt_sdf_mesh_grid(self._h, _p(size), _p(vals)))
        return size, vals

    def octree(self, depth: int) -> np.ndarray:
        """-> raw nodes, uint8 [count*36] (SDFOctreeNode records, BFS)."""
        n = C.c_int64(0)
        check(lib().rt_sdf_mesh_octree(self._h, int(depth), C.byref(n), None))
        buf = np.empty(n.value * 36, np.uint8)
        check(lib().rt_sdf_mesh_octree(self._h, int(depth), C.byref(n), _p(buf)))
        return buf

    def close(self):
        if getattr(self, "_h", None):
            check(lib().rt_sdf_mesh_destroy(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def subdivide_mesh(mesh: SimpleMesh, levels: int) -> SimpleMesh:
    """Midpoint subdivision (rt_mesh_subdivide): the config-5 stand-in mesh."""
    L = lib()
    v = np.ascontiguousarray(mesh.vPos4f, np.float32)
    i = np.ascontiguousarray(mesh.indices, np.uint32)
    nv, ni = C.c_int64(0), C.c_int64(0)
    check(L.rt_mesh_subdivide(_p(v), len(v), _p(i), len(i), int(levels), None, C.byref(nv), None,
                              C.byref(ni)))
    ov = np.empty((nv.value, 4), np.float32)
    oi = np.empty(ni.value, np.uint32)
    check(L.rt_mesh_subdivide(_p(v), len(v), _p(i), len(i), int(levels), _p(ov), C.byref(nv), _p(oi),
                              C.byref(ni)))
    return SimpleMesh(ov, oi)
