"""rtamd -- MI355X-native primary-ray renderer (Python binding over include/rtamd.h).

The hot path (per-pixel BVH8 / SDF-grid / SDF-octree intersection and the
reference's shading) runs in hand-written HIP kernels in librtamd.so; this
package only marshals arguments.
"""
from ._lib import EXPORTED, LIB_PATH, RT_FLAG_CLEAR, RenderParams, RtError, Tile, build, lib
from .api import (BVHBuilder, Camera, FrameBuffer, HitInfo, IScene, MultiRenderer, Plane, Renderer, SceneUnion,
                  SDFGrid, SDFMesh, SDFOctree, ShadingMode, SimpleMesh, camera_matrices, device_count,
                  load_mesh_from_obj, load_sdf_grid, load_sdf_octree, render_params, save_mesh_to_obj,
                  subdivide_mesh)
from . import data, tiles, workloads

__all__ = [
    "EXPORTED", "LIB_PATH", "RT_FLAG_CLEAR", "RenderParams", "RtError", "Tile", "build", "lib",
    "BVHBuilder", "Camera", "FrameBuffer", "HitInfo", "IScene", "MultiRenderer", "Plane", "Renderer", "SceneUnion",
    "SDFGrid", "SDFMesh", "SDFOctree", "ShadingMode", "SimpleMesh", "camera_matrices", "device_count",
    "load_mesh_from_obj", "load_sdf_grid", "load_sdf_octree", "render_params", "save_mesh_to_obj",
    "subdivide_mesh",
    "data",
    "tiles", "workloads",
]
