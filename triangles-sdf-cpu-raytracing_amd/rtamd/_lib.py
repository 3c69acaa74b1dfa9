"""ctypes binding of librtamd.so (C ABI declared in include/rtamd.h).

The shared library is built in-tree (``make -C triangles-sdf-cpu-raytracing_amd``)
and loaded from ``triangles-sdf-cpu-raytracing_amd/lib/librtamd.so``. There is
no fallback: if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RTAMD_LIB") or os.path.join(PKG_ROOT, "lib", "librtamd.so")

RT_OK = 0
RT_FLAG_CLEAR = 1
RT_FLAG_TILE_NATURAL = 2
RT_FLAG_HITS_ONLY = 4
RT_IPC_HANDLE_BYTES = 64
RT_SCENE_MESH, RT_SCENE_GRID, RT_SCENE_OCTREE = 1, 2, 3

_lib = None


class RtError(RuntimeError):
    pass


class RenderParams(C.Structure):
    """rt_render_params (include/rtamd.h)."""
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


class Tile(C.Structure):
    """rt_tile (include/rtamd.h)."""
    _fields_ = [("band_rows", C.c_int32), ("rank", C.c_int32), ("num_ranks", C.c_int32),
                ("reserved", C.c_int32)]


class CameraState(C.Structure):
    """rt_camera_state (include/rtamd.h)."""
    _fields_ = [("position", C.c_float * 3), ("target", C.c_float * 3), ("orientation", C.c_float * 4),
                ("sensitivity", C.c_float), ("lock_up", C.c_int32), ("locked_up", C.c_float * 3)]


# name -> (restype, argtypes)
_SIGS = {
    "rt_last_error": (C.c_char_p, []),
    "rt_abi_version": (C.c_int, []),
    "rt_build_id": (C.c_char_p, []),
    "rt_device_count": (C.c_int, []),
    "rt_set_device": (C.c_int, [C.c_int]),
    "rt_load_obj": (C.c_int, [C.c_char_p, C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_void_p,
                              C.POINTER(C.c_int64)]),
    "rt_load_grid": (C.c_int, [C.c_char_p, C.c_void_p, C.c_void_p]),
    "rt_load_octree": (C.c_int, [C.c_char_p, C.POINTER(C.c_int64), C.c_void_p]),
    "rt_camera": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_float, C.c_float,
                            C.c_float, C.c_void_p, C.c_void_p]),
    "rt_bvh_export": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p,
                                C.POINTER(C.c_int64), C.c_void_p, C.POINTER(C.c_int32)]),
    "rt_set_bvh_builder": (C.c_int, [C.c_int]),
    "rt_scene_create_mesh": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                       C.POINTER(C.c_void_p)]),
    "rt_scene_create_grid": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    "rt_scene_create_octree": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(C.c_void_p)]),
    "rt_scene_set_plane": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_float]),
    "rt_scene_kind": (C.c_int, [C.c_void_p]),
    "rt_scene_device_bytes": (C.c_int64, [C.c_void_p]),
    "rt_scene_bvh_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                     C.POINTER(C.c_int32)]),
    "rt_scene_destroy": (C.c_int, [C.c_void_p]),
    "rt_scene_replicate": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "rt_scene_device": (C.c_int, [C.c_void_p]),
    "rt_scene_get_plane": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.c_void_p, C.POINTER(C.c_float)]),
    "rt_multi_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "rt_multi_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rt_multi_render": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                  C.c_uint32, C.POINTER(C.c_float)]),
    "rt_multi_render_device_frames": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                                C.c_int32, C.c_int32, C.c_uint32, C.c_void_p]),
    "rt_multi_rccl_version": (C.c_int, [C.POINTER(C.c_int32)]),
    "rt_multi_destroy": (C.c_int, [C.c_void_p]),
    "rt_render": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                            C.c_uint32, C.POINTER(C.c_float)]),
    "rt_host_pin": (C.c_int, [C.c_void_p, C.c_int64]),
    "rt_host_unpin": (C.c_int, [C.c_void_p]),
    "rt_render_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                   C.c_int32, C.c_uint32, C.c_void_p, C.c_void_p]),
    "rt_untile_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                   C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "rt_tile_pixels": (C.c_int64, [C.c_int32, C.c_int32, C.c_void_p]),
    "rt_render_device_frames": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                          C.c_int32, C.c_int32, C.c_uint32, C.c_void_p, C.c_void_p]),
    "rt_clear_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]),
    "rt_stream_prepare": (C.c_int, [C.c_void_p]),
    "rt_stream_release": (C.c_int, [C.c_void_p]),
    "rt_exchange_alloc": (C.c_int, [C.c_int64, C.POINTER(C.c_void_p)]),
    "rt_exchange_free": (C.c_int, [C.c_void_p]),
    "rt_ipc_get_handle": (C.c_int, [C.c_void_p, C.c_void_p]),
    "rt_ipc_open": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "rt_ipc_close": (C.c_int, [C.c_void_p]),
    "rt_intersect_rays": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_float,
                                    C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_count_work": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                C.c_uint32, C.c_void_p, C.c_void_p]),
    "rt_bench_frames": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                  C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "rt_sdf_mesh_create": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                     C.POINTER(C.c_void_p)]),
    "rt_sdf_mesh_points": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]),
    "rt_sdf_mesh_grid": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_sdf_mesh_octree": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64), C.c_void_p]),
    "rt_sdf_mesh_destroy": (C.c_int, [C.c_void_p]),
    "rt_mesh_subdivide": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p,
                                    C.POINTER(C.c_int64), C.c_void_p, C.POINTER(C.c_int64)]),
    "rt_camera_init": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(CameraState)]),
    "rt_camera_rotate": (C.c_int, [C.POINTER(CameraState), C.c_float, C.c_float]),
    "rt_camera_reset_position": (C.c_int, [C.POINTER(CameraState), C.c_void_p]),
    "rt_camera_reset_target": (C.c_int, [C.POINTER(CameraState), C.c_void_p]),
    "rt_camera_set_lock_up": (C.c_int, [C.POINTER(CameraState), C.c_int]),
    "rt_camera_zoom": (C.c_int, [C.POINTER(CameraState), C.c_float]),
    "rt_camera_basis": (C.c_int, [C.POINTER(CameraState), C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_camera_view_inverse": (C.c_int, [C.POINTER(CameraState), C.c_void_p]),
    "rt_write_png": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int32, C.c_int32]),
    "rt_save_obj": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p,
                              C.c_void_p]),
}

EXPORTED = tuple(_SIGS)


def source_build_id() -> str:
    """rt_build_id() of a library built from this tree (the Makefile's ID_SRCS
    rule): sha256 of csrc/{*.cpp,*.h,*.hip} in sorted order, then
    include/rtamd.h, then the Makefile (its compile flags); first 16 hex
    digits. Variant builds (tools/build_variant.sh) append "+<name>:<flags
    hash>", so they never pass for the shipping library."""
    import glob
    import hashlib
    srcs = sorted(os.path.relpath(p, PKG_ROOT) for ext in ("cpp", "h", "hip")
                  for p in glob.glob(os.path.join(PKG_ROOT, "csrc", f"*.{ext}")))
    h = hashlib.sha256()
    for rel in srcs + [os.path.join("..", "include", "rtamd.h"), "Makefile"]:
        with open(os.path.join(PKG_ROOT, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build(force: bool = False) -> str:
    """Compile librtamd.so in-tree (hipcc, gfx950). Always runs make: it skips
    up-to-date targets, and the objects list their headers, so a source edit
    never leaves a stale library behind the tests. A library injected through
    RTAMD_LIB is taken as is."""
    if os.environ.get("RTAMD_LIB"):
        return LIB_PATH
    subprocess.run(["make", "-C", PKG_ROOT, "-s"] + (["-B"] if force else []), check=True)
    return LIB_PATH


def _share_torch_runtime() -> None:
    """One HIP runtime per process. torch bundles its own libamdhip64 /
    libhsa-runtime64 with the same SONAME (libamdhip64.so.7) as /opt/rocm's;
    if torch is loaded first, the dynamic loader binds librtamd.so to that
    already-loaded runtime, so torch tensors, RCCL and our kernels share one
    device context. Loading librtamd.so first would instead bring up a second
    runtime that torch cannot see the GPU through."""
    if os.environ.get("RTAMD_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    global _lib
    if _lib is None:
        _share_torch_runtime()
        if not os.path.exists(LIB_PATH):
            raise RtError(f"librtamd.so not built ({LIB_PATH}); run build() / make -C {PKG_ROOT}")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != RT_OK:
        msg = lib().rt_last_error()
        raise RtError(f"rtamd error {rc}: {msg.decode() if msg else ''}")
