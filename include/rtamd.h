/* rtamd.h -- C ABI of the MI355X-native primary-ray renderer.
 *
 * Drop-in boundary for the per-pixel intersection hot path of
 * iMacsimus/Triangles-SDF-CPU-RayTracing (reference @ 2025-07-04). The reference
 * has no FFI for this path other than the per-node ISPC exports
 * (src/ray_pack.ispc:220,242,290); a per-node call across a device boundary is
 * infeasible, so the boundary sits at FRAME granularity, mirroring
 *     float Renderer::draw(const IScene&, FrameBuffer&, const Camera&,
 *                          const float4x4 projInv) const       (src/raytracing.hpp:109-110)
 * and, for ray-level checks,
 *     virtual HitInfo IScene::intersect(rayPos, rayDir, tNear, tFar) const
 *                                                           (src/raytracing.hpp:77-79)
 *
 * Plain C types only: pointers + sizes, no torch, no HIP types in signatures
 * (streams are passed as void*). Every entry point returns 0 on success or a
 * negative RT_E* code; rt_last_error() gives a message (thread-local).
 * Nothing throws across the ABI.
 */
#ifndef RTAMD_H
#define RTAMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTAMD_ABI_VERSION 8

enum rt_status {
  RT_OK = 0,
  RT_E_INVALID = -1,   /* bad argument */
  RT_E_IO = -2,        /* file missing / truncated */
  RT_E_DEVICE = -3,    /* HIP runtime error (no GPU, OOM, launch failure) */
  RT_E_STATE = -4      /* wrong scene kind for the call */
};

/* ShadingMode, same order as the reference enum (src/raytracing.hpp:99). */
enum rt_shading_mode { RT_SHADING_NORMAL = 0, RT_SHADING_LAMBERT = 1, RT_SHADING_COLOR = 2 };

enum rt_scene_kind { RT_SCENE_MESH = 1, RT_SCENE_GRID = 2, RT_SCENE_OCTREE = 3 };

/* rt_render flags */
#define RT_FLAG_CLEAR 1u /* treat the framebuffer as FrameBuffer::clear()ed (color=0, t=+inf;
                            src/raytracing.hpp:16-19) and write every pixel: clear+draw fused.
                            Without it, t is read as tPrev and color/t are written only on hit
                            (src/raytracing.cpp:89-94). */
#define RT_FLAG_TILE_NATURAL 2u /* with a tile: write this rank's bands at their own rows of a
                                   full W*H frame (e.g. rank 0's frame mapped over xGMI by
                                   rt_ipc_open) instead of packed */
#define RT_FLAG_HITS_ONLY 4u /* with RT_FLAG_CLEAR: the frame is already cleared (rt_clear_device,
                                or FrameBuffer::clear() for rt_render's host buffers), so only hit
                                pixels are stored -- the same image as CLEAR alone, with misses
                                costing no stores (no xGMI traffic for background; for rt_render,
                                only the hits' bounding box is copied back) */

typedef struct rt_scene rt_scene; /* opaque: owns the device copy of one scene on one GPU */
typedef struct rt_sdf_mesh rt_sdf_mesh; /* opaque: a triangle mesh prepared for SDF queries */

/* Per-frame parameters. Matrices are column-major float[16] (LiteMath float4x4
 * m_col[4] layout: element (r,c) at [c*4 + r]).
 *   view_inv = inverse4x4(camera.lookAtMatrix())           (src/raytracing.cpp:73-75)
 *   proj_inv = inverse4x4(perspectiveMatrix(45, W/H, 0.01, 100)) (src/main.cpp:198-201)
 * rtamd_camera() computes both exactly as the reference does. */
typedef struct rt_render_params {
  float camera_pos[3];       /* Camera::position()                          */
  float view_inv[16];
  float proj_inv[16];
  float light_pos[3];        /* Renderer::lightPos  (src/raytracing.hpp:103) */
  int32_t shading_mode;      /* rt_shading_mode     (src/raytracing.hpp:106) */
  int32_t enable_shadows;    /* Renderer::enableShadows      (:104)          */
  int32_t enable_reflections;/* Renderer::enableReflections  (:105)          */
  int32_t reserved;          /* must be 0 */
} rt_render_params;

/* Row-band tiling for multi-GPU rendering: image rows are cut into bands of
 * band_rows rows; band b belongs to rank (b % num_ranks). A rank renders only
 * its bands and writes them PACKED (its bands in increasing order, each band
 * W*band_rows pixels, the last band possibly shorter). rank=0,num_ranks=1
 * renders the full frame in natural layout. */
typedef struct rt_tile {
  int32_t band_rows;
  int32_t rank;
  int32_t num_ranks;
  int32_t reserved;
} rt_tile;

/* ---- errors / device ---------------------------------------------------- */
const char *rt_last_error(void);
int rt_abi_version(void);
/* First 16 hex digits of the sha256 of the sources this library was built
 * from (triangles-sdf-cpu-raytracing_amd/csrc/{*.cpp,*.h,*.hip} sorted, then
 * include/rtamd.h): ties a shipped binary to a source tree. */
const char *rt_build_id(void);
/* Number of visible HIP devices (0 if none); never fails. */
int rt_device_count(void);
/* Select the HIP device used by subsequent scene creation on this thread. */
int rt_set_device(int device);

/* ---- host-side inputs (loaders; mirror the reference loaders) ----------- */
/* cmesh4::LoadMeshFromObj (src/core/mesh.cpp:178-287) [+ loadAndScale,
 * src/main.cpp:326-343, when scale != 0]. Two-call protocol: call with
 * vpos4 = idx = NULL to get the counts, then with buffers of that size.
 * vpos4: float[4*nverts] (x,y,z,w), idx: uint32[nidx]. */
int rt_load_obj(const char *path, int scale, float *vpos4, int64_t *nverts, uint32_t *idx,
                int64_t *nidx);
/* loadSDFGrid (src/grid_raytracing.cpp:127-134): 12-byte header uint32 size[3],
 * then float values[size.x*size.y*size.z], index (x*sy+y)*sz+z. Two-call protocol. */
int rt_load_grid(const char *path, uint32_t size[3], float *values);
/* loadSDFOctree (src/octree_raytracing.cpp:8-16): uint32 count, then count x
 * 36-byte SDFOctreeNode {float values[8]; uint32 childrenOffset}. Two-call protocol. */
int rt_load_octree(const char *path, int64_t *count, void *nodes36);

/* Camera(pos, target, up).lookAtMatrix() inverse and perspective inverse,
 * following src/camera.cpp:36-62 + LiteMath ("unpinned"). */
int rt_camera(const float pos[3], const float target[3], const float up[3], float fovy_deg,
              float aspect, float znear, float zfar, float view_inv[16], float proj_inv[16]);

/* Host-only: build the BVH8 exactly as rt_scene_create_mesh does and export it
 * in canonical pre-order (52 x uint32 per node: isLeaf, realCount|count,
 * startIndex, 0, then the reference Box8 SoA as float bits, +inf in unused
 * slots, zeros for leaves) plus the triangle permutation (original triangle id
 * per triangle slot, i.e. BVHBuilder's reordered mesh.indices / 3). Two-call
 * protocol on *nnodes. Used to check the tree against the reference's. */
int rt_bvh_export(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                  uint32_t *canon, int64_t *nnodes, uint32_t *perm_tri, int32_t *max_depth);
/* Which builder rt_scene_create_mesh / rt_bvh_export use for BVHBuilder::perform
 * (src/triangles_raytracing.cpp:12-258): RT_BVH_HOST (OpenMP on the host),
 * RT_BVH_DEVICE (on the current HIP device: libstdc++'s introsort replicated
 * with parallel partitions, SAH sweeps as device scans) or RT_BVH_AUTO (the
 * device from 32,768 triangles when a device is visible). Both give the
 * identical tree. Process-wide. */
enum rt_bvh_builder { RT_BVH_AUTO = 0, RT_BVH_HOST = 1, RT_BVH_DEVICE = 2 };
int rt_set_bvh_builder(int mode);

/* ---- scenes ------------------------------------------------------------- */
/* BVHBuilder::perform (src/triangles_raytracing.cpp:227-258): builds the same
 * 8-wide SAH BVH on the host, then uploads a GPU layout of it. */
int rt_scene_create_mesh(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                         rt_scene **out);
/* SDFGrid (src/grid_raytracing.hpp:10-21). values: x-major, float[sx*sy*sz]. */
int rt_scene_create_grid(const uint32_t size[3], const float *values, rt_scene **out);
/* SDFOctree (src/octree_raytracing.hpp:20-47). nodes36: count x 36 bytes. */
int rt_scene_create_octree(const void *nodes36, int64_t count, rt_scene **out);
/* SceneUnion(scene, Plane(normal, offset)) (src/raytracing.hpp:83-97,119-186;
 * src/main.cpp:189-190). enabled=0 renders the scene alone. */
int rt_scene_set_plane(rt_scene *s, int enabled, const float normal[3], float offset);
int rt_scene_kind(const rt_scene *s);
/* Device bytes held by the scene (nodes/triangles/voxels). */
int64_t rt_scene_device_bytes(const rt_scene *s);
/* Statistics of the host BVH (mesh scenes): node count, inner count, max depth. */
int rt_scene_bvh_stats(const rt_scene *s, int64_t *nodes, int64_t *inner, int32_t *max_depth);
int rt_scene_destroy(rt_scene *s);
/* A copy of scene s on another HIP device (device arrays copied device to
 * device, over xGMI between GPUs; no rebuild): the same tree, plane and kernel
 * instantiation, so every frame it renders is bitwise s's. For replicating one
 * scene on the GPUs of a single-process multi-GPU render (rt_multi_create). */
int rt_scene_replicate(const rt_scene *s, int device, rt_scene **out);
/* HIP device the scene lives on. */
int rt_scene_device(const rt_scene *s);
/* The plane last given to rt_scene_set_plane (enabled, normal, offset). */
int rt_scene_get_plane(const rt_scene *s, int *enabled, float normal[3], float *offset);

/* ---- frames ------------------------------------------------------------- */
/* Renderer::draw on HOST buffers color[W*H] (RGBA8 packed, R in the low byte)
 * and t[W*H] (row-major y*W+x). Uploads, renders, downloads, synchronises.
 * flags: 0 (t read as tPrev, write on hit), RT_FLAG_CLEAR (clear + draw, every
 * pixel written) or RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY (the caller's buffers
 * already hold a cleared frame, src/main.cpp:197). Without RT_FLAG_CLEAR, or
 * with both, only the bounding box of the stored hits is copied back: the
 * other pixels keep the caller's values, as Renderer::draw leaves them. Once a
 * copy is queued every return, an error included, waits for it first, so the
 * buffers may be unpinned / freed when the call returns.
 * *ms (optional) receives the kernel time in milliseconds (HIP events). */
int rt_render(rt_scene *s, const rt_render_params *p, uint32_t *color, float *t, int32_t W,
              int32_t H, uint32_t flags, float *ms);
/* Pin (page-lock) a host framebuffer range, mapped on every device: rt_render
 * and rt_multi_render then store a cleared frame's hits straight into it and
 * DMA the other frames' copies directly. The caller keeps it pinned while it
 * reuses the buffer (the reference app keeps one FrameBuffer across frames,
 * src/main.cpp:88) and MUST unpin it before freeing it: a range freed while
 * pinned stays mapped to its old pages, and a later buffer at the same address
 * would be written through that stale mapping (rt_host_pin refuses a range
 * that overlaps one still pinned). rt_host_unpin first drains every stream the
 * library created. Optional: on pageable memory the library copies through its
 * own pinned staging frames on the host, so the HIP runtime never DMAs from or
 * to a caller's pageable memory. The range is
 * registered coarse-grained: it is coherent with the host at stream
 * synchronisation points only, which every rt_render / rt_multi_render call
 * reaches before it returns; a caller that hands the same range to its own
 * HIP work must synchronise that work before reading the range on the host. */
int rt_host_pin(void *ptr, int64_t bytes);
int rt_host_unpin(void *ptr);
/* Same on DEVICE buffers, asynchronously on `stream` (hipStream_t or NULL).
 * With tile != NULL only this rank's bands are rendered, packed (rt_tile). */
int rt_render_device(rt_scene *s, const rt_render_params *p, uint32_t *d_color, float *d_t,
                     int32_t W, int32_t H, uint32_t flags, const rt_tile *tile, void *stream);
/* Scatter gathered packed bands of all ranks (ranks x per-rank capacity, as
 * produced by rt_render_device with a tile) into a natural-layout frame, on
 * the device. per_rank_pixels = capacity of one rank's packed slot. */
int rt_untile_device(const uint32_t *d_packed_color, const float *d_packed_t, int64_t per_rank_pixels,
                     uint32_t *d_color, float *d_t, int32_t W, int32_t H, const rt_tile *tile,
                     void *stream);
/* Pixels a rank owns under `tile` (its packed buffer length). */
int64_t rt_tile_pixels(int32_t W, int32_t H, const rt_tile *tile);
/* rt_render_device for `frames` frames of one size/tile/shading path, on
 * `stream`: frame f uses params[f], d_color[f], d_t[f]. Up to 16 frames share
 * ONE launch (blockIdx.z = frame), so each frame's silhouette tail is covered
 * by the next frames' tiles; the image of every frame is identical to
 * rt_render_device's. */
int rt_render_device_frames(rt_scene *s, const rt_render_params *params, int32_t frames,
                            uint32_t *const *d_color, float *const *d_t, int32_t W, int32_t H,
                            uint32_t flags, const rt_tile *tile, void *stream);
/* FrameBuffer::clear() (src/raytracing.hpp:16-19) on device buffers: color = 0,
 * t = +inf over n pixels, on `stream`. */
int rt_clear_device(uint32_t *d_color, float *d_t, int64_t n, void *stream);
/* Per-stream render state (the multi-frame launches' work-queue heads),
 * allocated and zeroed in stream order on the current device. Optional:
 * rt_render_device_frames creates it on a stream's first use, also in stream
 * order (no device-wide synchronisation); calling this first keeps that
 * allocation out of a timed region. rt_stream_release frees it (stream
 * ordered); a later launch on the stream re-creates it. No reference
 * counterpart: the reference renders on the host (src/raytracing.cpp:67-102). */
int rt_stream_prepare(void *stream);
int rt_stream_release(void *stream);

/* ---- multi-GPU rendering in ONE process (Renderer::draw over n devices) --
 * The reference renders a frame with one call, Renderer::draw (src/main.cpp:
 * 196-207), which splits it by image rows across OpenMP threads
 * (src/raytracing.cpp:77-96). rt_multi does the same across GPUs of one
 * process: the scene (on devices[0], the root) is replicated on every other
 * device (rt_scene_replicate), the frame is cut into bands of band_rows rows,
 * band b -> slot b mod n (rt_tile), every slot renders its bands packed on its
 * own stream, and the bands come to the root in one gather per frame and
 * buffer: RCCL ncclGather over a communicator from ncclCommInitAll when the
 * devices are distinct, device-to-device (peer) copies when a device is
 * listed more than once (RCCL refuses a device twice in one communicator; the
 * one-GPU test box runs {0, 0}). The root de-interleaves them
 * (rt_untile_device). Frames are bitwise the single-device frames. */
typedef struct rt_multi rt_multi;
enum rt_multi_exchange { RT_MULTI_RCCL = 1, RT_MULTI_PEER_COPY = 2 };
/* scene must live on devices[0]; it is not owned and must outlive the handle
 * (its plane is re-read at every render). band_rows <= 0 selects 8. */
int rt_multi_create(rt_scene *scene, const int32_t *devices, int32_t n, int32_t band_rows, rt_multi **out);
/* Slots, the exchange in use (rt_multi_exchange) and the band height. */
int rt_multi_info(const rt_multi *m, int32_t *n, int32_t *exchange, int32_t *band_rows);
/* Renderer::draw on HOST buffers, the same contract as rt_render (flags 0 =
 * tPrev frame, RT_FLAG_CLEAR, RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY). Blocks until
 * the frame is in color / t. The cleared frame (RT_FLAG_CLEAR |
 * RT_FLAG_HITS_ONLY, the app's clear() + draw) takes no gather: every slot
 * stores its bands' hits at their own rows straight into host memory (the
 * caller's buffers when rt_host_pin pinned them, else a pinned staging frame
 * whose stored spans the host copies). The other flags gather on the root.
 * *ms (optional): device time from the first launch to the assembled frame
 * (HIP events). */
int rt_multi_render(rt_multi *m, const rt_render_params *p, uint32_t *color, float *t, int32_t W, int32_t H,
                    uint32_t flags, float *ms);
/* Version code of the RCCL library rt_multi's gather runs on (ncclGetVersion:
 * major * 10000 + minor * 100 + patch), i.e. whichever librccl the process
 * resolved first (torch loads its own). */
int rt_multi_rccl_version(int32_t *version);
/* `frames` frames into DEVICE buffers on the root (d_color[f], d_t[f]),
 * flags must contain RT_FLAG_CLEAR. Stream-ordered on `stream` (a stream of
 * the root device, or NULL): the slots start after the work queued on it so
 * far, and it waits for the assembled frames; the host does not block. Each
 * slot renders up to 16 frames per launch (rt_render_device_frames). */
int rt_multi_render_device_frames(rt_multi *m, const rt_render_params *params, int32_t frames,
                                  uint32_t *const *d_color, float *const *d_t, int32_t W, int32_t H,
                                  uint32_t flags, void *stream);
int rt_multi_destroy(rt_multi *m);

/* ---- frame exchange over xGMI (multi-GPU, one process per GPU) -----------
 * Rank 0 allocates its frame slots with rt_exchange_alloc, exports them with
 * rt_ipc_get_handle, and every other rank maps them with rt_ipc_open; the ranks
 * then render their bands straight into rank 0's frame (RT_FLAG_TILE_NATURAL |
 * RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY). Slots are uncached device memory, so
 * peer stores land where rank 0's kernels read them. Replaces the reference's
 * framebuffer (src/raytracing.hpp:9-20) for the row-split render. */
#define RT_IPC_HANDLE_BYTES 64
int rt_exchange_alloc(int64_t bytes, void **d_ptr);
int rt_exchange_free(void *d_ptr);
int rt_ipc_get_handle(void *d_ptr, uint8_t handle[RT_IPC_HANDLE_BYTES]);
/* Map a peer's exported allocation on the current device; *d_ptr is usable by
 * kernels of this device (peer access over xGMI). */
int rt_ipc_open(const uint8_t handle[RT_IPC_HANDLE_BYTES], void **d_ptr);
int rt_ipc_close(void *d_ptr);

/* ---- rays (IScene::intersect) ------------------------------------------- */
/* Batch of n rays, host buffers. hit[i] (0/1), t[i], normal[3i..3i+2] exactly
 * as HitInfo (src/raytracing.hpp:67-73; normal NOT flipped toward the ray),
 * prim[i] = primitive id (mesh: original triangle index in OBJ face order;
 * grid: linear index of the c0 cell of the hit sample; octree: leaf node
 * index; plane: -2; miss: -1). */
int rt_intersect_rays(rt_scene *s, const float *o, const float *d, int64_t n, float tnear,
                      float tfar, int32_t *hit, float *t, float *normal, int64_t *prim);

/* Timing helper for benchmarks: renders `frames` frames back to back on the
 * device (buffers owned by the library), returns the mean kernel ms per frame
 * and the total in *total_ms. params[frames] gives one camera per frame. */
int rt_bench_frames(rt_scene *s, const rt_render_params *params, int32_t frames, int32_t W,
                    int32_t H, uint32_t flags, float *mean_ms, float *total_ms);

/* Work counters of the reference traversal for `frames` frames (diagnostic
 * kernel variant; same traversal as the timed kernels): counters[0..8] =
 * BVH inner-node visits, BVH leaf visits, triangle tests, grid sdf
 * evaluations, octree node visits, octree leaf visits, octree march steps,
 * octree normal evaluations, rays (scene intersections). Shadow rays stop at
 * their first hit here, so with shadows on the counts are lower than the
 * reference's full traversal; primary-ray counts are identical. */
int rt_count_work(rt_scene *s, const rt_render_params *params, int32_t frames, int32_t W, int32_t H,
                  uint32_t flags, const rt_tile *tile, int64_t counters[9]);

/* ---- mesh -> SDF construction -------------------
 * The reference renders SDF grids/octrees it does not generate (course data in
 * the formats read by loadSDFGrid, src/grid_raytracing.cpp:127-134, and
 * loadSDFOctree, src/octree_raytracing.cpp:8-16 / octree_raytracing.hpp:8-18);
 * BASELINE configs 3-4 name large inputs absent from the reference
 * (.MISSING_LARGE_BLOBS). These entry points build them deterministically on
 * the GPU: signed distance = distance to the closest triangle (ties: lowest
 * triangle id), sign from the angle-weighted pseudonormal of the closest
 * feature, positions after v /= v.w. See DESIGN.md 9. */
int rt_sdf_mesh_create(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                       rt_sdf_mesh **out);
/* Signed distance at n points p3[3n] (host buffers). */
int rt_sdf_mesh_points(rt_sdf_mesh *m, const float *p3, int64_t n, float *dist);
/* SDFGrid values for a size[0] x size[1] x size[2] lattice over [-1,1]^3
 * (sample i at 2i/(size-1)-1, index (x*sy+y)*sz+z), host buffer. */
int rt_sdf_mesh_grid(rt_sdf_mesh *m, const uint32_t size[3], float *values);
/* Sparse SDFOctree of max depth `depth` (36-byte nodes, BFS, 8 children
 * contiguous): a node is refined when |sdf(centre)| <= its half-diagonal;
 * unrefined nodes are empty leaves (values 1000); depth-`depth` nodes are
 * leaves holding the SDF at their corners. Two-call protocol on *count (the
 * result is cached in the handle). */
int rt_sdf_mesh_octree(rt_sdf_mesh *m, int32_t depth, int64_t *count, void *nodes36);
int rt_sdf_mesh_destroy(rt_sdf_mesh *m);
/* Host-only: midpoint subdivision `levels` times (each triangle -> 4, edge
 * midpoints shared, (a+b)*0.5 on the 4 components): the config-5 stand-in
 * for MotorcycleCylinderHead.obj. Two-call protocol on the counts. */
int rt_mesh_subdivide(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, int32_t levels,
                      float *out_vpos4, int64_t *out_nverts, uint32_t *out_idx, int64_t *out_nidx);

/* ---- the viewer's orbit camera and image output --
 * Camera (src/camera.hpp:7-61, src/camera.cpp:1-72, src/quaternion.hpp:8-70):
 * position/target plus an orientation quaternion; rotate(dx, dy) is the
 * viewer's mouse drag (main.cpp:277-280: rotate(-dx, -dy)), zoom(wheel) its
 * mouse wheel (main.cpp:281-288). Host-only; the state is a plain struct. */
typedef struct rt_camera_state {
  float position[3];
  float target[3];
  float orientation[4]; /* x, y, z, w (un-normalised after construction, as the reference) */
  float sensitivity;    /* 0.01 (camera.hpp:55) */
  int32_t lock_up;
  float locked_up[3];
} rt_camera_state;
int rt_camera_init(const float pos[3], const float target[3], const float up[3], rt_camera_state *c);
int rt_camera_rotate(rt_camera_state *c, float dx, float dy);
int rt_camera_reset_position(rt_camera_state *c, const float pos[3]);
int rt_camera_reset_target(rt_camera_state *c, const float target[3]);
int rt_camera_set_lock_up(rt_camera_state *c, int on);
int rt_camera_zoom(rt_camera_state *c, float wheel);
/* up(), right(), forward() (camera.hpp:29-37); any pointer may be NULL. */
int rt_camera_basis(const rt_camera_state *c, float up[3], float right[3], float forward[3]);
/* inverse4x4(lookAtMatrix()) -- the view_inv of rt_render_params. */
int rt_camera_view_inverse(const rt_camera_state *c, float view_inv[16]);
/* Write a colour buffer (W*H packed RGBA8, R in the low byte, row 0 = top) as
 * an 8-bit RGBA PNG (what the viewer shows, main.cpp:239-242). */
int rt_write_png(const char *path, const uint32_t *color, int32_t W, int32_t H);
/* cmesh4::SaveMeshToObj (src/core/mesh.cpp:14-63), byte for byte: v / vt / vn
 * per vertex with std::to_string, faces "f i/i/i". vnorm4 (4 per vertex) and
 * vtex2 (2 per vertex) may be NULL: fix_missing's defaults (0,0,1) / (0,0). */
int rt_save_obj(const char *path, const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                const float *vnorm4, const float *vtex2);

#ifdef __cplusplus
}
#endif
#endif /* RTAMD_H */
