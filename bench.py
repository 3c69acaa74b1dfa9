#!/usr/bin/env python3
"""bench.py -- primary-ray throughput of the MI355X renderer (BASELINE.json metric).

Metric: "Mrays/sec + ms/frame at 1920x1080, bunny tris & SDF grid, 1/2/4/8 MI355X".
Workload (N=1 and N>1): BASELINE configs[1], stanford-bunny.obj triangles at
1920x1080, primary rays (Normal shading, no ground plane: one ray per pixel,
the pure intersection hot path), over a deterministic 64-frame camera orbit
(SURVEY.md 8(d)). A "step" is one frame. The orbit's frames are independent:
--group (default 8) of them go out in ONE launch (blockIdx.z = frame), so a
frame's last tiles (grazing rays at the silhouette, the per-frame tail) are
covered by the next frames' tiles, and launches alternate over --streams
(default 2) HIP streams with their own framebuffers, so one launch's tail
overlaps the next launch. value = rays of all K frames / wall time of the K
frames; the one-frame-at-a-time latency is reported beside it
("frame_latency"). At N=1 the other BASELINE configs are measured the same way
and reported under "extra" (rank 0): the SDF grid (configs[2]) on a 256^3 SDF
of stanford-bunny generated on the GPU (stand-in: example_grid_large.grid is
missing from the reference) and on the shipped 65^3 example_grid.grid; the
octree (configs[3]) at 3840x2160 on a depth-8 generated octree (stand-in for
example_octree_large.octree) and on the shipped sdf_6.octree; and the config-5
mesh stand-in (stanford-bunny subdivided twice, 1,111,216 triangles) at
3840x2160.

Multi-GPU (torch.distributed.run, one process per GPU; rtamd.rowsplit): every
frame is split into --band-rows (8) row bands dealt round-robin to the ranks
(load balance: the model covers the middle rows), with the same launches
(--group frames, --streams streams). Exchange p2p (default): each rank's
kernel stores its HIT pixels straight into rank 0's frame slots over xGMI
(IPC-mapped), and one 4-byte RCCL all-reduce per group signals completion;
exchange gather: one RCCL gather per group of the packed bands (8 B/pixel) and
a de-interleave on rank 0. Total work per step is fixed (one 1080p frame), so
scaling is "strong"; value = pixels of all frames / max-over-ranks wall time.
rank 0 checks that its last assembled frame equals a whole-frame render.

Timing: W untimed warm-up frames, then exactly K frames between barrier +
torch.cuda.synchronize() on both sides; max over ranks. Inputs are resident
in HBM before the timed region. Roofline: algorithmic bytes per launch
(SURVEY.md 8(d) byte model, counted exactly by a diagnostic variant of the
same kernel over the same frames) / the render kernel's average launch
duration (HIP events around each launch on its own stream; what rocprofv3's
kernel stats report); the amortized rate (wall / K, launches overlap) is
reported beside it. Peak 8.0 TB/s HBM.
cpu_baseline: the oracle (C++ restatement of the reference's CPU path, with
the ISPC kernels in scalar C++) on the host cores, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))

import torch  # noqa: E402  (load torch's HIP runtime first: one runtime per process)
import torch.distributed as dist  # noqa: E402

import rtamd  # noqa: E402
from rtamd import workloads as WL  # noqa: E402

METRIC = "Mrays/sec + ms/frame at 1920x1080, bunny tris & SDF grid, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
W_IMG, H_IMG = 1920, 1080


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--workload", default="stanford-bunny.obj")
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--exchange", choices=("p2p", "gather"), default="p2p",
                    help="N>1 frame assembly: peer stores over xGMI, or one RCCL gather per group")
    ap.add_argument("--group", type=int, default=8,
                    help="frames per launch (blockIdx.z = frame); N>1: also per completion signal / gather")
    ap.add_argument("--depth", type=int, default=3, help="N>1: groups whose slots are in flight")
    ap.add_argument("--streams", type=int, default=2, help="HIP streams the launches alternate over")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="wall budget of the CPU sample")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 HBM-traffic passes")
    ap.add_argument("--dist", action="store_true",
                    help="use the banded + gather path even at WORLD_SIZE 1 (protocol test)")
    return ap.parse_args()


def host_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def frame_params(n_frames):
    orbit = WL.orbit_positions(64)
    return [WL.params_for(orbit[k % 64], W_IMG, H_IMG, rtamd.ShadingMode.Normal)
            for k in range(n_frames)]


def run_single(scene, params, warmup, steps, W=W_IMG, H=H_IMG, inflight=2, tile=None, batch=1):
    """N=1: full frames, render kernel only. Frames go out in launches of
    `batch` frames (rt_render_device_frames: blockIdx.z = frame, so a frame's
    silhouette tail is covered by the next frames' tiles); launch j is issued
    on stream j % inflight with its own framebuffers, so up to `inflight`
    launches are in flight. batch=1, inflight=1 is one frame at a time. HIP
    events bracket each launch on its own stream.
    Returns (wall_s, kernel_ms_avg per launch, buffers of the last frame)."""
    dev = torch.device("cuda")
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(inflight - 1)]
    bufs = [[(torch.empty((H, W), dtype=torch.int32, device=dev),
              torch.empty((H, W), dtype=torch.float32, device=dev)) for _ in range(batch)]
            for _ in range(inflight)]

    def issue(j, k0, n, ev=None):
        st = streams[j % inflight]
        fb = bufs[j % inflight][:n]
        with torch.cuda.stream(st):
            if ev:
                ev[0].record(st)
            if n == 1:
                scene.render_device(params[k0], fb[0][0].data_ptr(), fb[0][1].data_ptr(), W, H, clear=True,
                                    tile=tile, stream=st.cuda_stream)
            else:
                scene.render_device_frames(params[k0:k0 + n], [c.data_ptr() for c, _ in fb],
                                           [t.data_ptr() for _, t in fb], W, H, rtamd.RT_FLAG_CLEAR,
                                           tile=tile, stream=st.cuda_stream)
            if ev:
                ev[1].record(st)

    def launches(k0, nframes):
        return [(k0 + i, min(batch, nframes - i)) for i in range(0, nframes, batch)]

    for j, (k, n) in enumerate(launches(0, warmup)):
        issue(j, k, n)
    timed = launches(warmup, steps)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in timed]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j, (k, n) in enumerate(timed):
        issue(j, k, n, evs[j])
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    jl, (kl, nl) = len(timed) - 1, timed[-1]
    return wall, kms, bufs[jl % inflight][nl - 1]


def run_distributed(scene, params, warmup, steps, a):
    """N>1: row bands per rank, assembled on rank 0 (rtamd.rowsplit). With the
    p2p exchange every rank stores its hit pixels straight into rank 0's frame
    over xGMI and one 4-byte RCCL all-reduce per group of frames signals
    completion; with the gather exchange one RCCL gather per group moves the
    packed bands (8 B/pixel). With the gloo backend (RTAMD_DIST_BACKEND=gloo:
    several ranks sharing one GPU, a protocol test on a 1-GPU box) signals and
    gathers are host-synchronous."""
    from rtamd.rowsplit import RowSplitRenderer

    def make(exchange):
        r = RowSplitRenderer(scene, W_IMG, H_IMG, band_rows=a.band_rows, group=a.group, depth=a.depth,
                             streams=a.streams, exchange=exchange)
        r.render(params[:max(warmup, 1)])
        r.drain()
        return r

    rs = make(a.exchange)
    # the warm-up's last assembled frame must equal a whole-frame render on rank 0;
    # a p2p exchange that fails this (IPC mapping, peer-store visibility) is replaced
    # by the RCCL gather before anything is timed
    ok = 1
    if dist.get_rank() == 0:
        _, _, (c1, t1) = run_single(scene, params[max(warmup, 1) - 1:max(warmup, 1)], 0, 1, inflight=1)
        fc, ft = rs.last()
        ok = int(torch.equal(c1, fc) and torch.equal(t1.view(torch.int32), ft.view(torch.int32)))
    if not rs._all_ok(ok):
        if rs.exchange == "p2p":
            rs.close()
            rs = make("gather")
            rs.fallback = "p2p warm-up frame differed from a whole-frame render"
        else:
            raise SystemExit("row-split gather: assembled warm-up frame differs from a whole-frame render")
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rs.render(params[warmup:warmup + steps])
    rs.host_issue_s = time.perf_counter() - t0  # host time to issue every launch and signal
    rs.drain()
    dist.barrier()
    wall = time.perf_counter() - t0
    # render-launch duration of this rank's bands: the same launches (a.group frames each,
    # a.streams streams) rendered locally, HIP events on each launch's stream
    n = min(steps, 64)
    _, kms, _ = run_single(scene, params[warmup:warmup + n], 0, n, inflight=a.streams, tile=rs.tile,
                           batch=a.group)
    return wall, kms, rs


def roofline(scene, params, tile, kms, W=W_IMG, H=H_IMG, amortized_ms=None, frames_per_launch=1):
    """Algorithmic bytes per launch (SURVEY.md 8(d) byte model, counted exactly
    by the counting variant of the kernel over the same frames) / the kernel's
    event-timed average launch duration over the timed region (kernel_ms, what
    rocprofv3's kernel stats report). With frames in flight the launches
    overlap; the amortized rate (wall / launches) is reported beside it."""
    c = scene.count_work(params, W, H, clear=True, tile=tile)
    npx = (rtamd.lib().rt_tile_pixels(W, H, ctypes.byref(tile)) if tile is not None else W * H)
    algo = scene.algorithmic_bytes(c, npx * len(params)) / len(params) * frames_per_launch
    if amortized_ms is not None:
        amortized_ms *= frames_per_launch
    achieved = algo / (kms * 1e-3) / 1e9
    per_ray = {k: round(v / (npx * len(params)), 4) for k, v in c.items() if v}
    out = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
           "algorithmic_bytes_per_launch": int(algo), "kernel_ms": round(kms, 5),
           "work_per_ray": per_ray, "frames_per_launch": frames_per_launch}
    if amortized_ms is not None:
        # launches overlap (frames in flight): algorithmic bytes per amortized launch.
        # The byte model counts cache-served bytes, so this can exceed the HBM peak.
        out["amortized_ms_per_launch"] = round(amortized_ms, 5)
        out["amortized_achieved"] = round(algo / (amortized_ms * 1e-3) / 1e9, 1)
    return out


def one_stream(scene, params, warmup, steps, W, H, group, rl):
    """The same launches (group frames each) issued on ONE stream: launches do
    not overlap, so the event-timed launch duration is the launch's own time
    and bytes / duration is the kernel's rate without a second launch beside
    it. Reported beside the default two-stream roofline."""
    wall, kms, _ = run_single(scene, params, warmup, steps, W, H, inflight=1, batch=group)
    achieved = rl["algorithmic_bytes_per_launch"] / (kms * 1e-3) / 1e9
    return {"streams": 1, "ms_per_step": round(wall * 1e3 / steps, 4), "kernel_ms": round(kms, 5),
            "achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4)}


def pmc_traffic(workload, W, H, group, frames=32):
    """HBM bytes per launch of the headline render kernel (launches of `group`
    frames, the timed region's launch shape) from rocprofv3 PMC counters,
    collected in two separate --pmc passes (FETCH_SIZE, WRITE_SIZE cannot
    share a pass) over tools/prof_frames.py, as MI355X_MICROARCH.md's
    HBM section prescribes: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
    FETCH_SIZE reports half the bytes of coalesced reads, so it is doubled.
    Runs as child processes BEFORE this process touches the GPU. Returns
    (bytes_per_launch | None, detail dict)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, {"error": "rocprofv3 not found"}
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    # the batch path's kernel: render_persist_kernel (work queue) or, with
    # RTAMD_PERSIST=0, render_batch_kernel; one frame per launch: render_kernel
    knames = ("render_persist_kernel", "render_batch_kernel") if group > 1 else ("render_kernel",)
    tmp = tempfile.mkdtemp(prefix="rtamd_pmc_", dir="/tmp")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = ["timeout", "-k", "10", "180", prof, "--pmc", ctr, "--output-format", "csv", "-d", d,
                   "-o", "p", "--", sys.executable, os.path.join(ROOT, "tools", "prof_frames.py"),
                   "--workload", workload, "--frames", str(frames), "--W", str(W), "--H", str(H),
                   "--group", str(group)]
            r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True)
            if r.returncode != 0:
                return None, {"error": f"{ctr} pass rc={r.returncode}: {r.stderr[-300:]}"}
            per = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if any(k in row["Kernel_Name"] for k in knames) and row["Counter_Name"] == ctr:
                            per.append(float(row["Counter_Value"]))
            if not per:
                return None, {"error": f"no {ctr} rows for {knames}"}
            vals[ctr] = sum(per) / len(per)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch = 2.0 * vals["FETCH_SIZE"] * 1024.0
    write = vals["WRITE_SIZE"] * 1024.0
    return fetch + write, {"fetch_bytes": round(fetch), "write_bytes": round(write),
                           "raw_kib": {k: round(v, 1) for k, v in vals.items()},
                           "launches": frames // group, "frames_per_launch": group,
                           "correction": "FETCH_SIZE x2 (gfx950), KiB -> B"}


def standin_scenes(which):
    """BASELINE configs 3-5 stand-ins, generated deterministically on the GPU
    from the shipped stanford-bunny.obj (rt_sdf_mesh_* / rt_mesh_subdivide)."""
    from rtamd import data
    bunny = rtamd.load_mesh_from_obj(data.path("stanford-bunny.obj"))
    if which == "mesh_large":
        return rtamd.BVHBuilder(rtamd.subdivide_mesh(bunny, 2))
    sm = rtamd.SDFMesh(bunny)
    if which == "grid":
        return rtamd.SDFGrid(*sm.grid(256))
    return rtamd.SDFOctree(sm.octree(8))


EXTRAS = [
    # key, scene source, W, H, description
    ("grid", "grid", 1920, 1080,
     "stanford-bunny SDF 256^3 grid generated on the GPU (stand-in for the missing "
     "example_grid_large.grid, BASELINE configs[2])"),
    ("grid_shipped", "example_grid.grid", 1920, 1080, "shipped example_grid.grid (65^3)"),
    ("octree", "octree", 3840, 2160,
     "stanford-bunny SDF octree of depth 8 generated on the GPU (stand-in for the missing "
     "example_octree_large.octree, BASELINE configs[3])"),
    ("octree_shipped", "sdf_6.octree", 3840, 2160, "shipped sdf_6.octree"),
    ("mesh_large", "mesh_large", 3840, 2160,
     "stanford-bunny midpoint-subdivided twice, 1,111,216 triangles (stand-in for the missing "
     "MotorcycleCylinderHead.obj, BASELINE configs[4]), 1 GPU"),
]


def run_extras(warmup, steps, streams, group):
    out = {}
    for key, src, W, H, desc in EXTRAS:
        if "." in src:
            kind, payload, _ = WL.load_input(src)
            sc = WL.make_scene(kind, payload)
        else:
            sc = standin_scenes(src)
        sc.set_plane(None)
        orbit = WL.orbit_positions(64)
        prm = [WL.params_for(orbit[k % 64], W, H, rtamd.ShadingMode.Normal) for k in range(warmup + steps)]
        wall, kms, _ = run_single(sc, prm, warmup, steps, W, H, inflight=streams, batch=group)
        rl = roofline(sc, prm[warmup:], None, kms, W, H, wall * 1e3 / steps, group)
        out[key] = {"workload": f"{desc}, {W}x{H} primary rays, same orbit",
                    "value": round(W * H * steps / wall / 1e6, 1), "unit": "Mrays/s",
                    "ms_per_step": round(wall * 1e3 / steps, 4), "steps": steps, "roofline": rl}
        if streams > 1:
            out[key]["roofline_one_stream"] = one_stream(sc, prm, warmup, steps, W, H, group, rl)
        sc.close()
        torch.cuda.synchronize()
    return out


def cpu_baseline(name, budget_s):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpuref  # the oracle: test infrastructure, used here only as the CPU baseline
    from rtamd import data
    p = data.path(name)
    threads = host_threads()
    if name.endswith(".obj"):
        v, i = cpuref.load_obj(p)
        sc = cpuref.RefScene.mesh(v, i)
    else:
        import numpy as np
        size = np.fromfile(p, np.uint32, 3)
        vals = np.fromfile(p, np.float32, offset=12)
        sc = cpuref.RefScene.grid(size, vals)
    sc.set_plane(False)
    orbit = WL.orbit_positions(64)
    frames, ms_total = 0, 0.0
    t0 = time.perf_counter()
    while frames < 64 and (time.perf_counter() - t0) < budget_s:
        vi, pi = cpuref.camera_matrices(orbit[frames], aspect=W_IMG / H_IMG)
        P = cpuref.make_params(orbit[frames], vi, pi, mode=0)
        _, _, _, ms = sc.render(P, W_IMG, H_IMG, threads=threads)
        ms_total += ms
        frames += 1
    mrays = W_IMG * H_IMG * frames / (ms_total * 1e-3) / 1e6
    return {"value": round(mrays, 2), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "ms_per_frame": round(ms_total / frames, 2),
            "sample": f"{frames} frames of the 64-frame orbit, {name} {W_IMG}x{H_IMG} primary rays, "
                      f"OpenMP schedule(dynamic) over rows, {threads} threads, ISPC kernels as scalar "
                      f"C++ (oracle/cpuref.cpp)"}


def main():
    # libraries (RCCL, gloo) print banners to stdout: send fd 1 to stderr and
    # keep the real stdout for the one JSON line
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    use_dist = world > 1 or a.dist
    pmc, pmc_extra = None, {}
    if not use_dist and not a.no_pmc:
        pmc = pmc_traffic(a.workload, W_IMG, H_IMG, a.group)  # child processes, before this one inits the GPU
        if not a.no_extra:  # the SDF-grid sphere march (north star: >= 60 % of HBM peak)
            pmc_extra["grid"] = pmc_traffic("grid", W_IMG, H_IMG, a.group)
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a HIP device (the renderer has no CPU path)")
    device = local % ndev  # ranks > devices only for the gloo protocol test
    torch.cuda.set_device(device)
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        backend = os.environ.get("RTAMD_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    rtamd._lib.check(rtamd.lib().rt_set_device(device))

    kind, payload, _ = WL.load_input(a.workload)
    scene = WL.make_scene(kind, payload)
    scene.set_plane(None)
    params = frame_params(a.warmup + a.steps)

    latency = None
    if not use_dist:
        wall, kms, _ = run_single(scene, params, a.warmup, a.steps, inflight=a.streams, batch=a.group)
        tile = None
        if a.streams * a.group > 1:  # single-frame latency (one frame at a time), reported beside
            lwall, lkms, _ = run_single(scene, params, min(a.warmup, 8), min(a.steps, 64), inflight=1)
            latency = {"ms_per_frame": round(lwall * 1e3 / min(a.steps, 64), 4),
                       "kernel_ms": round(lkms, 5)}
    else:
        wall, kms, rs = run_distributed(scene, params, a.warmup, a.steps, a)
        tile = rs.tile
        t = torch.tensor([wall], dtype=torch.float64,
                         device="cpu" if dist.get_backend() == "gloo" else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        if rank == 0:  # the assembled last frame must equal a whole-frame render of it
            _, _, (c1, t1) = run_single(scene, params[-1:], 0, 1, inflight=1)
            fc, ft = rs.last()
            check_equal = bool(torch.equal(c1, fc) and torch.equal(t1.view(torch.int32), ft.view(torch.int32)))
        dist.barrier()
        rs.close()

    rl = roofline(scene, params[a.warmup:], tile, kms, amortized_ms=wall * 1e3 / a.steps,
                  frames_per_launch=a.group)
    if pmc is not None:
        rl["traffic"] = None if pmc[0] is None else round(pmc[0])
        rl["traffic_detail"] = pmc[1]
    total_rays = W_IMG * H_IMG * a.steps
    value = total_rays / wall / 1e6
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "Mrays/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(wall * 1e3 / a.steps, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic deterministic 64-frame camera orbit over the shipped {a.workload}",
        "config": {"workload": f"{a.workload} triangles {W_IMG}x{H_IMG} primary rays "
                               "(BASELINE configs[1]); Normal shading, no plane",
                   "resolution": [W_IMG, H_IMG], "camera": "orbit r=2.5 h=0.5 fovy 45",
                   "parallelism": (f"row bands of {a.band_rows} rows x {world} GPUs, exchange "
                                   f"{rs.exchange}, {a.group} frames per launch and signal, {a.streams} streams")
                   if use_dist else "1 GPU, 1 thread per pixel",
                   "frames_per_launch": a.group, "streams": a.streams},
        "roofline": rl,
    }
    if latency is not None:
        out["frame_latency"] = latency
    if not use_dist and a.streams > 1:
        out["roofline_one_stream"] = one_stream(scene, params, a.warmup, a.steps, W_IMG, H_IMG, a.group, rl)
    if use_dist and rank == 0:
        out["frame_check"] = {"assembled_equals_single_render": check_equal,
                              "backend": dist.get_backend(), "exchange": rs.exchange,
                              "fallback": getattr(rs, "fallback", None)}
        out["host_issue_ms_per_frame"] = round(rs.host_issue_s * 1e3 / a.steps, 4)
    if rank == 0 and not use_dist and not a.no_extra:
        out["extra"] = run_extras(min(a.warmup, 16), min(a.steps, 64), a.streams, a.group)
        for key, (tb, detail) in pmc_extra.items():
            out["extra"][key]["roofline"]["traffic"] = None if tb is None else round(tb)
            out["extra"][key]["roofline"]["traffic_detail"] = detail
    if rank == 0 and not use_dist and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.workload, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
