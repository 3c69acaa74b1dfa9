#!/usr/bin/env python3
"""bench.py -- primary-ray throughput of the MI355X renderer (BASELINE.json metric).

Metric: "Mrays/sec + ms/frame at 1920x1080, bunny tris & SDF grid, 1/2/4/8 MI355X".
A "step" is one frame of a deterministic 64-frame camera orbit.
`--workload` picks the headline (default `bunny`: BASELINE configs[1],
stanford-bunny.obj at 1920x1080, primary rays = Normal shading, no ground plane,
one ray per pixel, the pure intersection hot path); every key of WORKLOADS
works at every N, e.g. `--workload mesh_large` is configs[4] (the 1.1 M-triangle
stand-in at 3840x2160) and `--workload grid` configs[2] (the 256^3 stand-in).
Orbit frames are independent: up to --group of them (8 on one GPU, 16 per
rank at N > 1, where a rank's share of a frame is 1/N) go out in ONE launch
(the persistent kernel pulls 8x8 pixel tiles of all of them from one work
queue) and launches alternate over --streams (2) HIP streams with their own
framebuffers. value = rays of all K frames / wall time of the K frames.

Warm-up: every stream gets its work-queue state (rt_stream_prepare) and at
least one full launch before t0, whatever --warmup is. The K timed frames are
ceil(K / group) launches of near-equal size, bracketed by synchronize().

At N=1 the other BASELINE configs are measured the same way under "extra"
(rank 0): the grid (configs[2]: 256^3 stand-in and the shipped 65^3), the
octree (configs[3]: depth-8 stand-in and the shipped sdf_6, both 3840x2160),
configs[4]'s mesh on one GPU, and the bunny in the reference's DEFAULT shading
mode (plane + Lambert + shadows + reflections; also reported as traced rays/s).

Measured cache traffic (every workload): L1->L2 read requests
(TCP_TCC_READ_REQ_sum) and L1 accesses (TCP_TOTAL_CACHE_ACCESSES_sum) in bytes,
by the bytes per request / access of a calibration dispatch in the same
rocprofv3 pass (calib_read_kernel: 256 MiB read once at 16 B per lane), over
the same wall time -> roofline.measured; binding_roof / binding_frac = the
largest MEASURED roof (DRAM, VALU issue, L2 reads).

Roofline (every workload): achieved = ALGORITHMIC bytes per frame (the SURVEY
8(d) byte model on the reference's data layout, counted exactly by the
diagnostic variant of the same kernel over the same frames) / ms_per_step (the
wall time per frame of the timed region, the same clock as `value`). The bytes
are cache-served (every scene is cache-resident): when they arrive faster than
the 8 TB/s HBM peak they are held against the aggregate L2 peak instead
(peak_kind). Measured DRAM bytes per frame (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE,
separate --pmc passes, MI355X_MICROARCH.md's gfx950 correction) over the same
wall time give dram.frac; SQ_INSTS_VALU x 2 cycles over 1024 SIMDs x 2.4 GHz
give valu_frac; SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU) the lane
utilisation. `one_stream` repeats the launches on ONE stream, where a launch's
HIP-event duration is its own (rocprofv3's average for the kernel must agree).
Raw counters go to the --detail file, not the JSON line.

Multi-GPU (one process per GPU; rtamd.rowsplit): `--gpus N` under
torch.distributed.run, or run directly: without WORLD_SIZE in the environment
this process spawns the N rank processes itself (spawn_ranks, before anything
touches the GPU), relays rank 0's line and exits with the worst rank's code; a
GPU count it cannot run is an error, never a 1-GPU line. Every frame is split
into --band-rows (8) row bands dealt round-robin to the ranks. Exchange p2p
(default): each rank's kernel stores its HIT pixels straight into rank 0's
frame slots over xGMI (IPC-mapped), each wave ending with a system-scope
release, and one 4-byte RCCL all-reduce per group signals completion; exchange
gather: one RCCL gather per group of packed bands + a de-interleave on rank 0.
The frame is fixed as N grows ("strong"); value = pixels of all frames /
max-over-ranks wall time. Every rank reports its render-kernel time
(rank_kernel_ms). The warm-up is a verification pass: every slot group is
reused at least twice and EVERY assembled frame of it is compared bitwise
with a whole-frame render on rank 0 (frame_check.verify_pass), and so is the
last timed frame.

drop_in (N=1): rt_render, the Renderer::draw surface INTEGRATION.md binds, on
HOST buffers (upload when not cleared, render, download), ms per frame with the
copies, on pageable and on pinned (rt_host_pin) buffers; multi_rehearsal: the
same for rt_multi_render with two slots on the one GPU. --single-process (and
the N>1 run's single_process leg) reports rt_multi_render's host-buffer
figures over its devices.

cpu_baseline: the oracle (C++ restatement of the reference's CPU path, ISPC
kernels as scalar C++) on every CPU this process is granted (see
host_threads), OpenMP schedule(dynamic) over rows, rank 0 at N=1 only: the
headline workload, its default shading mode, the shipped 65^3 grid (1080p) and
sdf_6 (4K), each a time-bounded sample of the same orbit.
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))

import torch  # noqa: E402  (load torch's HIP runtime first: one runtime per process)
import torch.distributed as dist  # noqa: E402

import rtamd  # noqa: E402
from rtamd import workloads as WL  # noqa: E402

METRIC = "Mrays/sec + ms/frame at 1920x1080, bunny tris & SDF grid, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
L2_PEAK_GBS = 34500.0  # aggregate L2, 8 XCDs x 4 MiB (MI355X_MICROARCH.md, L2)
SIMDS, CLOCK_HZ = 1024, 2.4e9  # 256 CUs x 4 SIMDs, max clock

# key -> (input, W, H, mode, BASELINE config, description)
WORKLOADS = {
    "bunny": ("stanford-bunny.obj", 1920, 1080, "primary", "configs[1]",
              "shipped stanford-bunny.obj (69,451 triangles)"),
    "grid": ("grid", 1920, 1080, "primary", "configs[2]", WL.STANDINS["grid"]),
    "grid_shipped": ("example_grid.grid", 1920, 1080, "primary", "configs[2] (shipped file)",
                     "shipped example_grid.grid (65^3)"),
    "octree": ("octree", 3840, 2160, "primary", "configs[3]", WL.STANDINS["octree"]),
    "octree_shipped": ("sdf_6.octree", 3840, 2160, "primary", "configs[3] (shipped file)",
                       "shipped sdf_6.octree (depth 6)"),
    "mesh_large": ("mesh_large", 3840, 2160, "primary", "configs[4]", WL.STANDINS["mesh_large"]),
    "default_mode": ("stanford-bunny.obj", 1920, 1080, "default", "configs[1], default shading",
                     "stanford-bunny.obj, the reference's default shading: ground plane + Lambert + shadows + "
                     "one reflection (raytracing.cpp:13-65)"),
}
EXTRAS = ["grid", "grid_shipped", "octree", "octree_shipped", "mesh_large", "default_mode"]
# CPU baselines beside the GPU figures: (workload key, share of --cpu-seconds, max frames)
CPU_SAMPLES = [("default_mode", 0.25, 16), ("grid_shipped", 0.25, 16), ("octree_shipped", 0.25, 8)]


def workload_entry(name):
    """A WORKLOADS key, or a shipped input file name (1920x1080 primary rays)."""
    if name in WORKLOADS:
        return name, WORKLOADS[name]
    for k, v in WORKLOADS.items():
        if v[0] == name and v[3] == "primary":
            return k, v
    if name.endswith((".obj", ".grid", ".octree")):
        return name, (name, 1920, 1080, "primary", "shipped input", f"shipped {name}")
    raise SystemExit(f"unknown --workload {name!r}; keys: {', '.join(WORKLOADS)} or a shipped input file")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--workload", default="bunny", help="a WORKLOADS key or a shipped input file")
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--exchange", choices=("p2p", "gather"), default="p2p",
                    help="N>1 frame assembly: peer stores over xGMI, or one RCCL gather per group")
    ap.add_argument("--group", type=int, default=None,
                    help="frames per launch (at most 16; default: --steps split evenly over --streams, "
                         "at most 16); "
                         "N>1: also per completion signal / gather")
    ap.add_argument("--depth", type=int, default=3, help="N>1: groups whose slots are in flight")
    ap.add_argument("--streams", type=int, default=2, help="HIP streams the launches alternate over")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--no-drop-in", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=24.0, help="wall budget of all CPU samples")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 counter passes")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="file for the raw counters and per-launch times (not the JSON line)")
    ap.add_argument("--single-process", action="store_true",
                    help="N GPUs from ONE process (rt_multi: scene replicas, row bands, RCCL ncclGather)")
    ap.add_argument("--devices", default=None,
                    help="--single-process: comma-separated device list (default 0..N-1; a device may repeat)")
    ap.add_argument("--no-single-process-leg", action="store_true",
                    help="N>1: skip rank 0's single-process measurement over all N devices")
    ap.add_argument("--dist", action="store_true",
                    help="use the banded + gather path even at WORLD_SIZE 1 (protocol test)")
    return ap.parse_args()


def host_threads():
    """CPU threads this process may actually run on -> (threads, how it was decided).
    The affinity set can list the whole machine while a cgroup quota (cpu.max) or
    the job's OMP_NUM_THREADS grants a share of it (the GPU box: 256 CPUs listed,
    16 granted); oversubscribing that share makes OpenMP far slower, so the
    smallest of the three is used."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    n, why = aff, f"affinity set {aff}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max" and int(q) // int(per) < n:
            n, why = max(1, int(q) // int(per)), f"cgroup cpu.max quota {q}/{per} (affinity set {aff})"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < n:
        n, why = int(omp), f"OMP_NUM_THREADS={omp} (affinity set {aff})"
    return max(1, n), why


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def orbit_params(n, W, H, mode="primary"):
    orbit = WL.orbit_positions(64)
    sm = rtamd.ShadingMode.Normal if mode == "primary" else rtamd.ShadingMode.Lambert
    return [WL.params_for(orbit[k % 64], W, H, sm) for k in range(n)]


def split_launches(k0, n, batch):
    """n frames from k0 as ceil(n / batch) launches of near-equal size."""
    if n <= 0:
        return []
    nl = -(-n // batch)
    base, extra = divmod(n, nl)
    out, k = [], k0
    for j in range(nl):
        m = base + (1 if j < extra else 0)
        out.append((k, m))
        k += m
    return out


_POOL = []


def stream_pool(k):
    """k HIP streams for the render launches, created ONCE per process and
    reused by every measurement. Streams share the device's hardware queues
    (GPU_MAX_HW_QUEUES, 4 here) round-robin in creation order; a stream created
    per measurement would sooner or later share a queue with the other one and
    serialise the 'overlapping' launches. Four consecutive pool streams, never
    the null stream."""
    while len(_POOL) < max(k, 4):
        _POOL.append(torch.cuda.Stream())
    return _POOL[:k]


LAST_RUN = {}


class NoGC:
    """No garbage-collector pass inside a timed region: a full collection of
    this process's heap (torch, numpy, ctypes) stalls the host thread that
    issues the launches for milliseconds, longer than the 20-frame run itself.
    The collection runs on entry, before the region's warm-up: run right
    before t0 it left the first timed launch's issue ~120 us slower (bunny
    bands, tools/issue_probe2.py), 0.13 ms of the 20-frame wall. Nested uses
    leave the collector off."""

    def __enter__(self):
        self.was = gc.isenabled()
        if self.was:
            gc.collect()
            gc.disable()
        return self

    def __exit__(self, *exc):
        if self.was:
            gc.enable()


def run_single(scene, params, warmup, steps, W, H, inflight=2, tile=None, batch=1):
    """Full frames (or one rank's row bands with `tile`), render kernel only.
    Frames go out in launches of up to `batch` frames (rt_render_device_frames);
    launch j is issued on stream j % inflight with its own framebuffers. Before
    t0 every stream is prepared (rt_stream_prepare) and warmed with at least one
    full launch; params[i] is used for frame i (warm-up frames cycle through
    params). HIP events bracket each timed launch on its own stream.
    Returns (wall_s, per-launch kernel ms [(ms, frames)], buffers of the last frame)."""
    dev = torch.device("cuda")
    streams = stream_pool(inflight)
    for st in streams:
        rtamd._lib.check(rtamd.lib().rt_stream_prepare(ctypes.c_void_p(st.cuda_stream)))
    bufs = [[(torch.empty((H, W), dtype=torch.int32, device=dev),
              torch.empty((H, W), dtype=torch.float32, device=dev)) for _ in range(batch)]
            for _ in range(inflight)]

    def issue(j, prm, ev=None):
        st = streams[j % inflight]
        fb = bufs[j % inflight][:len(prm)]
        with torch.cuda.stream(st):
            if ev:
                ev[0].record(st)
            if len(prm) == 1:
                scene.render_device(prm[0], fb[0][0].data_ptr(), fb[0][1].data_ptr(), W, H, clear=True,
                                    tile=tile, stream=st.cuda_stream)
            else:
                scene.render_device_frames(prm, [c.data_ptr() for c, _ in fb], [t.data_ptr() for _, t in fb],
                                           W, H, rtamd.RT_FLAG_CLEAR, tile=tile, stream=st.cuda_stream)
            if ev:
                ev[1].record(st)

    nwarm = max(warmup, inflight * batch)
    with NoGC():
        for j, (k, n) in enumerate(split_launches(0, nwarm, batch)):
            issue(j, [params[(k + i) % len(params)] for i in range(n)])
        timed = split_launches(warmup, steps, batch)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in timed]
        for j, (a, b) in enumerate(evs):  # a torch event creates its HIP event at its first record: here, untimed
            a.record(streams[j % inflight])
            b.record(streams[j % inflight])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t_each = []
        for j, (k, n) in enumerate(timed):
            issue(j, params[k:k + n], evs[j])
            t_each.append(time.perf_counter())
        t_issued = time.perf_counter()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    LAST_RUN["issue_s"] = t_issued - t0  # host time to issue the timed launches (tools/ab.py)
    LAST_RUN["issue_each_us"] = [round((b - a) * 1e6) for a, b in zip([t0] + t_each[:-1], t_each)]
    launches = [(a.elapsed_time(b), n) for (a, b), (_, n) in zip(evs, timed)]
    jl, (kl, nl) = len(timed) - 1, timed[-1]
    return wall, launches, bufs[jl % inflight][nl - 1]


def verify_frames(a, warmup):
    """N>1 warm-up = verification pass: enough frames to reuse every slot group
    at least twice and end on a partial group."""
    return max(warmup, 2 * a.group * a.depth + a.group // 2 + 1, a.group * a.streams * a.depth)


def per_frame_ms(launches):
    """Frame-weighted kernel time per frame over the timed launches."""
    return sum(ms for ms, _ in launches) / sum(n for _, n in launches)


def run_distributed(scene, params, warmup, steps, a, W, H):
    """N>1: row bands per rank, assembled on rank 0 (rtamd.rowsplit). With the
    p2p exchange every rank stores its hit pixels straight into rank 0's frame
    over xGMI and one 4-byte RCCL all-reduce per group of frames signals
    completion; with the gather exchange one RCCL gather per group moves the
    packed bands (8 B/pixel). With the gloo backend (RTAMD_DIST_BACKEND=gloo:
    several ranks sharing one GPU, a protocol test on a 1-GPU box) signals and
    gathers are host-synchronous."""
    from rtamd.rowsplit import RowSplitRenderer

    nverify = verify_frames(a, warmup)

    def make(exchange):
        """A renderer whose warm-up is a verification pass: nverify frames (every
        slot group reused at least twice, ending on a partial group) go through
        the slot / signal protocol and rank 0 keeps a copy of EVERY assembled
        frame (on_frame, in stream order before the slot is cleared), each then
        compared bitwise with the same frame rendered whole by the one-frame
        kernel. -> (renderer, ok on every rank, frames that differed on rank 0)"""
        got = {}

        def keep(k, c, t):
            got[k] = (c.clone(), t.clone())
        r = RowSplitRenderer(scene, W, H, band_rows=a.band_rows, group=a.group, depth=a.depth,
                             streams=a.streams, exchange=exchange, on_frame=keep)
        r.render(params[:nverify])
        r.drain()
        r.on_frame = None
        bad = []
        if dist.get_rank() == 0:
            for k in range(nverify):
                _, _, (c1, t1) = run_single(scene, params[k:k + 1], 0, 1, W, H, inflight=1)
                fc, ft = got.get(k, (None, None))
                if fc is None or not (torch.equal(c1, fc) and torch.equal(t1.view(torch.int32),
                                                                          ft.view(torch.int32))):
                    bad.append(k)
        got.clear()
        return r, r._all_ok(int(not bad)), bad

    # a p2p exchange that fails the check (IPC mapping, peer-store visibility) is
    # replaced by the RCCL gather before anything is timed
    nogc = NoGC().__enter__()  # (collects before the verification pass; see NoGC)
    try:
        return _timed_distributed(make, nverify, params, warmup, steps, a, W, H, scene)
    finally:
        nogc.__exit__()


def _timed_distributed(make, nverify, params, warmup, steps, a, W, H, scene):
    rs, ok, bad = make(a.exchange)
    rs.verified = {"frames": nverify, "exchange": rs.exchange, "differing": bad}
    if not ok:
        if rs.exchange == "p2p":
            rs.close()
            rs, ok, bad2 = make("gather")
            rs.verified = {"frames": nverify, "exchange": rs.exchange, "differing": bad2,
                           "p2p_differing": bad}
            rs.fallback = f"p2p: {len(bad)} of {nverify} assembled frames differed from whole-frame renders"
        if not ok:
            raise SystemExit("row-split gather: assembled frames differ from whole-frame renders")
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
    _, launches, _ = run_single(scene, params[warmup:warmup + n], 0, n, W, H, inflight=a.streams, tile=rs.tile,
                                batch=a.group)
    return wall, per_frame_ms(launches), rs


# ------------------------------------------------------------ roofline --
L2_TOTAL_BYTES = 8 * 4 << 20  # 8 XCDs x 4 MiB


def peak_for(achieved, scene_bytes):
    """The roof the algorithmic bytes are held against. Residency decides
    first: a scene that fits the aggregate L2 (32 MiB) is served from the
    caches by construction, so it is held against the L2 roof whatever its
    rate (the 65^3 grid sits near 8 TB/s and would otherwise switch roofs, and
    its fraction by ~4x, on a few percent of run-to-run noise). A larger scene
    (the 64 MiB 256^3 grid, the ~60 MB 1.1 M-triangle mesh) is held against
    HBM, except when its algorithmic bytes arrive faster than HBM can deliver
    at all (the 1.1 M-triangle mesh at ~12 TB/s): those bytes are cache-served
    too, and an HBM fraction above 1 would name no roof. Such a workload could
    change roofs if its rate drifted across 8 TB/s, so the line carries both
    fractions (hbm_frac_of_algorithmic, l2_frac_of_algorithmic)."""
    if scene_bytes <= L2_TOTAL_BYTES or achieved > HBM_PEAK_GBS:
        return L2_PEAK_GBS, "l2"
    return HBM_PEAK_GBS, "hbm"


def work_model(scene, params, tile, W, H):
    """algorithmic bytes per frame, from the diagnostic kernel's
    exact work counts over the same frames. -> (bytes per frame, work per ray)."""
    c = scene.count_work(params, W, H, clear=True, tile=tile)
    npx = (rtamd.lib().rt_tile_pixels(W, H, ctypes.byref(tile)) if tile is not None else W * H)
    per_frame = scene.algorithmic_bytes(c, npx * len(params)) / len(params)
    per_ray = {k: round(v / (npx * len(params)), 4) for k, v in c.items() if v}
    return per_frame, per_ray


def calib_bytes(calib):
    """Bytes per L1->L2 read request and per L1 access on gfx950, from the
    calibration dispatches (CALIB_MIB read once at 16 B/lane, every line missing
    L1 exactly once): -> (bytes per TCP_TCC_READ_REQ, bytes per
    TCP_TOTAL_CACHE_ACCESSES), or (None, None). MI355X_MICROARCH.md calibrates
    only FETCH_SIZE / WRITE_SIZE ("other access widths are uncalibrated:
    calibrate on a known byte count"), so these are measured in the same run."""
    c = (calib or {}).get(16, {})
    req, acc = c.get("TCP_TCC_READ_REQ_sum"), c.get("TCP_TOTAL_CACHE_ACCESSES_sum")
    nbytes = CALIB_MIB << 20
    return (nbytes / req if req else None), (nbytes / acc if acc else None)


def roofline(algo_frame, ms_step, scene_bytes, ctr=None, pmc_err=None, group=8, calib=None):
    """The contract's roofline object for one workload, on the wall clock:
    achieved = algorithmic bytes per frame / ms_per_step; frac x peak x
    ms_per_step reproduces the bytes per frame. PMC counters (per launch of
    `group` frames, one stream) give the measured DRAM traffic and issue
    fractions over the same wall time."""
    dur = ms_step * 1e-3
    achieved = algo_frame / dur / 1e9
    peak, kind = peak_for(achieved, scene_bytes)
    rl = {"bound": kind, "achieved": round(achieved, 1), "peak": peak, "peak_kind": kind, "unit": "GB/s",
          "frac": round(achieved / peak, 4), "traffic": None, "per": "frame (step); time = ms_per_step",
          "algorithmic_bytes_per_frame": int(algo_frame), "ms_per_step": round(ms_step, 5),
          "scene_device_bytes": int(scene_bytes),
          "hbm_frac_of_algorithmic": round(achieved / HBM_PEAK_GBS, 4),
          "l2_frac_of_algorithmic": round(achieved / L2_PEAK_GBS, 4)}
    if pmc_err or not ctr or "FETCH_SIZE" not in ctr or "SQ_INSTS_VALU" not in ctr:
        rl["pmc_error"] = (pmc_err or "no counters")[:160]
        return rl
    fetch = 2.0 * ctr["FETCH_SIZE"] * 1024.0 / group  # gfx950: FETCH_SIZE reports half; KiB -> B; per frame
    write = ctr["WRITE_SIZE"] * 1024.0 / group
    rl["traffic"] = round(fetch + write)
    dram = (fetch + write) / dur / 1e9
    valu = ctr["SQ_INSTS_VALU"] / group
    issue = valu * 2.0 / (SIMDS * CLOCK_HZ * dur)
    lane = (ctr["SQ_THREAD_CYCLES_VALU"] / (64.0 * ctr["SQ_ACTIVE_INST_VALU"])
            if ctr.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in ctr else None)
    hits, miss = ctr.get("TCC_HIT_sum", 0.0), ctr.get("TCC_MISS_sum", 0.0)
    rl["dram"] = {"achieved": round(dram, 1), "frac": round(dram / HBM_PEAK_GBS, 4),
                  "write_bytes_per_frame": round(write)}
    rl["valu_frac"] = round(issue, 4)
    rl["lane_util"] = round(lane, 4) if lane is not None else None
    rl["l2_hit"] = round(hits / (hits + miss), 4) if hits + miss else None
    roofs = {"dram": dram / HBM_PEAK_GBS, "valu_issue": issue}
    # measured cache traffic: L1->L2 read requests and L1 accesses, in bytes by
    # the calibration dispatch's bytes per request / access, over the same time
    bpr, bpa = calib_bytes(calib)
    if bpr and "TCP_TCC_READ_REQ_sum" in ctr:
        l2_read = ctr["TCP_TCC_READ_REQ_sum"] * bpr / group
        l2_rate = l2_read / dur / 1e9
        l1_acc = ctr.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0) / group
        m = {"l2_read_bytes_per_frame": round(l2_read), "l2_read_GBs": round(l2_rate, 1),
             "l2_read_frac": round(l2_rate / L2_PEAK_GBS, 4),
             "l1_accesses_per_frame": round(l1_acc),
             "l1_access_bytes_per_frame": round(l1_acc * bpa) if bpa else None,
             "l1_access_GBs": round(l1_acc * bpa / dur / 1e9, 1) if bpa else None,
             "algorithmic_over_l2_read": round(algo_frame / l2_read, 2) if l2_read else None,
             "bytes_per_l2_read_req": round(bpr, 2), "bytes_per_l1_access": round(bpa, 2) if bpa else None,
             "calibration": f"calib_read_kernel: {CALIB_MIB} MiB read once, 16 B per lane, same rocprofv3 pass"}
        rl["measured"] = m
        roofs["l2_read"] = l2_rate / L2_PEAK_GBS
        if achieved > HBM_PEAK_GBS:
            rl["algorithmic_note"] = (
                f"algorithmic bytes arrive at {achieved / HBM_PEAK_GBS:.2f}x the HBM peak: they are cache hits "
                f"(measured L2 read bytes are 1/{algo_frame / l2_read:.1f} of them, DRAM bytes "
                f"{(fetch + write) / algo_frame * 100:.1f} %), so no byte roof binds this kernel")
    top = max(roofs, key=roofs.get)
    rl["binding_roof"] = top
    rl["binding_frac"] = round(roofs[top], 4)
    rl["binding"] = top if roofs[top] >= 0.5 else f"latency (largest roof {top} {roofs[top]:.2f})"
    return rl


def one_stream_leg(scene, params, warmup, steps, W, H, group, algo_frame, peak, kind):
    """The same launches on ONE stream: a launch's HIP-event duration is its own
    (the figure rocprofv3's kernel trace must reproduce)."""
    w1, l1, _ = run_single(scene, params, warmup, steps, W, H, inflight=1, batch=group)
    kl = statistics.mean(ms for ms, n in l1 if n == group) if any(n == group for _, n in l1) else \
        per_frame_ms(l1) * group
    kf = per_frame_ms(l1)
    a = algo_frame / (kf * 1e-3) / 1e9  # held against the workload's own roof (peak, kind)
    return {"ms_per_step": round(w1 * 1e3 / steps, 4), "kernel_ms_per_frame": round(kf, 5),
            "kernel_ms_per_launch": round(kl, 5), "frames_per_launch": group, "achieved": round(a, 1),
            "peak_kind": kind, "frac": round(a / peak, 4)}


# ------------------------------------------------------------ PMC passes --
PMC_PASSES = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"],
    ["SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU",
     "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_VMEM_RD", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum",
     "GRBM_GUI_ACTIVE"],
]
PMC_LAUNCHES = 2
CALIB_MIB, CALIB_WIDTHS = 256, (16, 4)  # L1/L2 counter calibration: MiB read once, bytes per lane


def pmc_counters(keys, group):
    """rocprofv3 --pmc passes (one counter set per run, as MI355X_MICROARCH.md
    prescribes) over tools/prof_frames.py, which renders PMC_LAUNCHES launches
    of `group` frames of every workload in `keys`, in order, on one stream.
    Runs as child processes BEFORE this process touches the GPU.
    Returns ({key: {counter: mean per launch}}, error | None)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return {}, "rocprofv3 not found"
    env = dict(os.environ, TMPDIR="/tmp")
    plan = ",".join(f"{k}:{WORKLOADS[k][0]}:{WORKLOADS[k][1]}:{WORKLOADS[k][2]}:{WORKLOADS[k][3]}" for k in keys)
    # the byte calibration of the L1 / L2 counters: one read pass of CALIB_MIB at
    # 16 and at 4 bytes per lane (calib_read_kernel), in every pass
    plan += "".join(f",calib:{w}:{CALIB_MIB}:0:-" for w in CALIB_WIDTHS)
    out = {k: {} for k in keys}
    out["_calib"] = {w: {} for w in CALIB_WIDTHS}
    tmp = tempfile.mkdtemp(prefix="rtamd_pmc_", dir="/tmp")
    try:
        for i, ctrs in enumerate(PMC_PASSES):
            d = os.path.join(tmp, f"p{i}")
            cmd = ["timeout", "-k", "10", "240", prof, "--pmc", *ctrs, "--output-format", "csv", "-d", d,
                   "-o", "p", "--", sys.executable, os.path.join(ROOT, "tools", "prof_frames.py"),
                   "--plan", plan, "--group", str(group), "--launches", str(PMC_LAUNCHES)]
            r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True)
            if r.returncode != 0:
                return out, f"pass {ctrs[0]} rc={r.returncode}: {r.stderr[-200:]}"
            rows, cal = {}, {}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        dst = rows if "render_" in row["Kernel_Name"] else \
                            cal if "calib_read_kernel" in row["Kernel_Name"] else None
                        if dst is None:
                            continue
                        dst.setdefault(int(row["Dispatch_Id"]), {})[row["Counter_Name"]] = \
                            float(row["Counter_Value"])
            cdisp = [cal[k] for k in sorted(cal)]
            if len(cdisp) == len(CALIB_WIDTHS):
                for w, m in zip(CALIB_WIDTHS, cdisp):
                    out["_calib"][w].update(m)
            disp = [rows[k] for k in sorted(rows)]
            if len(disp) != PMC_LAUNCHES * len(keys):
                return out, f"pass {ctrs[0]}: {len(disp)} render dispatches, expected {PMC_LAUNCHES * len(keys)}"
            for j, k in enumerate(keys):
                mine = disp[j * PMC_LAUNCHES:(j + 1) * PMC_LAUNCHES]
                for c in ctrs:
                    out[k][c] = sum(m.get(c, 0.0) for m in mine) / len(mine)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return out, None


# ------------------------------------------------------------ workloads --
def measure(key, entry, warmup, steps, streams, group, pmc, pmc_err, detail):
    """One extra workload at N=1: compact figures for the JSON line, the rest in `detail`."""
    src, W, H, mode, cfg, desc = entry
    scene, off = WL.scene_for(src)
    scene.set_plane(rtamd.Plane((0.0, 1.0, 0.0), off) if mode == "default" else None)
    prm = orbit_params(warmup + steps, W, H, mode)
    wall, launches, (lc, lt) = run_single(scene, prm, warmup, steps, W, H, inflight=streams, batch=group)
    issue_us = list(LAST_RUN["issue_each_us"])
    ms_step = wall * 1e3 / steps
    _, _, (c1, t1) = run_single(scene, prm[warmup + steps - 1:], 0, 1, W, H, inflight=1)  # as the headline's check
    frame_ok = bool(torch.equal(c1, lc) and torch.equal(t1.view(torch.int32), lt.view(torch.int32)))
    algo, per_ray = work_model(scene, prm[warmup:], None, W, H)
    rl = roofline(algo, ms_step, scene.device_bytes(), pmc.get(key), pmc_err, group, pmc.get("_calib"))
    one = one_stream_leg(scene, prm, warmup, steps, W, H, group, algo, rl["peak"], rl["peak_kind"]) \
        if streams > 1 else None
    out = {"config": cfg, "res": f"{W}x{H}", "mode": mode,
           "value": round(W * H * steps / wall / 1e6, 1), "ms_per_step": round(ms_step, 4),
           "frac": rl["frac"], "peak_kind": rl["peak_kind"],
           "dram_frac": rl.get("dram", {}).get("frac"), "valu_frac": rl.get("valu_frac"),
           "lane_util": rl.get("lane_util"),
           "l2_read_bytes_per_frame": rl.get("measured", {}).get("l2_read_bytes_per_frame"),
           "l2_read_frac": rl.get("measured", {}).get("l2_read_frac"),
           "binding": rl.get("binding"), "binding_frac": rl.get("binding_frac"),
           "1stream_launch_ms": one["kernel_ms_per_launch"] if one else None,
           "frame_check": frame_ok}
    if mode == "default":
        rays = per_ray.get("rays", 1.0)
        out["traced_rays_per_px"] = rays
        out["traced_value"] = round(W * H * rays * steps / wall / 1e6, 1)
    detail[key] = {"workload": desc, "roofline": rl, "one_stream": one, "work_per_ray": per_ray,
                   "launch_ms": [round(ms, 5) for ms, _ in launches], "issue_us": issue_us,
                   "wall_ms": round(wall * 1e3, 4), "pmc_per_launch": pmc.get(key)}
    scene.close()
    torch.cuda.synchronize()
    return out


def drop_in(scene, params, W, H, frames=16):
    """rt_render on HOST buffers (Renderer::draw's surface):
    ms per frame including the copies, on pageable and pinned buffers, for
    three ways of calling it: `clear` (RT_FLAG_CLEAR: clear + draw fused, no
    upload, the whole frame copied back), `cleared` (RT_FLAG_CLEAR |
    RT_FLAG_HITS_ONLY: the app's frameBuf.clear() + draw, main.cpp:197-203; the
    kernel stores its hits into host memory: the pinned buffers themselves, or
    a staging frame whose stored row spans the host copies) and `tprev` (no
    flag: upload of color and t, write-on-hit, the hits' box copied back)."""
    import numpy as np
    L = rtamd.lib()
    out = {}
    with NoGC():  # as the timed regions: no collection lands inside one of the 16 calls
        _drop_in_legs(scene, params, W, H, frames, L, out, np)
    out["note"] = f"rt_render on host buffers, {W}x{H}, ms/frame incl. copies, {frames} frames each"
    return out


def _drop_in_legs(scene, params, W, H, frames, L, out, np):
    for pinned in (False, True):
        c = np.zeros((H, W), np.uint32)
        t = np.full((H, W), np.inf, np.float32)
        if pinned:
            rtamd._lib.check(L.rt_host_pin(c.ctypes.data, c.nbytes))
            rtamd._lib.check(L.rt_host_pin(t.ctypes.data, t.nbytes))
        try:
            for how in ("clear", "cleared", "tprev"):
                kw = {"clear": how == "clear", "cleared": how == "cleared"}
                scene.render(params[0], c, t, **kw)  # warm
                wall, ks = 0.0, []
                for k in range(frames):
                    if how == "cleared":  # the app's frameBuf.clear(), outside the timed call
                        c.fill(0)
                        t.fill(np.inf)
                    t0 = time.perf_counter()
                    ks.append(scene.render(params[k % len(params)], c, t, **kw))
                    wall += time.perf_counter() - t0
                out[f"{'pinned' if pinned else 'pageable'}_{how}_ms"] = round(wall * 1e3 / frames, 4)
                out.setdefault("kernel_ms", round(statistics.median(ks), 4))
                if how == "cleared":  # the zero-copy kernel stores into host memory: its own time
                    out[f"{'pinned' if pinned else 'pageable'}_cleared_kernel_ms"] = round(statistics.median(ks), 4)
        finally:
            if pinned:
                L.rt_host_unpin(c.ctypes.data)
                L.rt_host_unpin(t.ctypes.data)


def drop_in_multi(scene, params, W, H, devices, frames=16):
    """rt_multi_render (Renderer::draw over several GPUs of one process) on HOST
    buffers, ms per frame including the copies, pageable and pinned: `cleared`
    (the app's clear() + draw: every slot stores its hits at their own rows
    straight into host memory, no gather), `clear` and `tprev` (the gather on
    the root). At N = 1 the rehearsal runs two slots on the one GPU."""
    import numpy as np
    L = rtamd.lib()
    out = {"devices": list(devices)}
    with NoGC(), rtamd.MultiRenderer(scene, devices) as mr:
        for pinned in (False, True):
            c = np.zeros((H, W), np.uint32)
            t = np.full((H, W), np.inf, np.float32)
            if pinned:
                rtamd._lib.check(L.rt_host_pin(c.ctypes.data, c.nbytes))
                rtamd._lib.check(L.rt_host_pin(t.ctypes.data, t.nbytes))
            try:
                for how in ("cleared", "clear", "tprev"):
                    kw = {"clear": how == "clear", "cleared": how == "cleared"}
                    mr.render(params[0], c, t, **kw)  # warm
                    wall, ks = 0.0, []
                    for k in range(frames):
                        if how == "cleared":  # the app's frameBuf.clear(), outside the timed call
                            c.fill(0)
                            t.fill(np.inf)
                        t0 = time.perf_counter()
                        ks.append(mr.render(params[k % len(params)], c, t, **kw))
                        wall += time.perf_counter() - t0
                    tag = "pinned" if pinned else "pageable"
                    out[f"{tag}_{how}_ms"] = round(wall * 1e3 / frames, 4)
                    if how == "cleared":
                        out[f"{tag}_cleared_device_ms"] = round(statistics.median(ks), 4)
            finally:
                if pinned:
                    L.rt_host_unpin(c.ctypes.data)
                    L.rt_host_unpin(t.ctypes.data)
    out["note"] = (f"rt_multi_render on host buffers, {W}x{H}, slots on devices {list(devices)}, ms/frame incl. "
                   f"copies, {frames} frames each; *_device_ms: first launch to last slot done (HIP events)")
    return out


def cpu_scene(src):
    """The oracle's scene of a workload input (the same arrays the GPU renders)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import cpuref  # the oracle: test infrastructure, used here only as the CPU baseline
    from rtamd import data
    if src.endswith(".obj"):
        v, i = cpuref.load_obj(data.path(src))
        return cpuref.RefScene.mesh(v, i), float((v[:, 1] / v[:, 3]).min())
    if src.endswith(".grid"):
        p = data.path(src)
        return cpuref.RefScene.grid(np.fromfile(p, np.uint32, 3), np.fromfile(p, np.float32, offset=12)), -1.0
    if src.endswith(".octree"):
        return cpuref.RefScene.octree(np.fromfile(data.path(src), np.uint8, offset=4)), -1.0
    # a stand-in: the arrays the GPU scene is built from
    bunny = rtamd.load_mesh_from_obj(data.path("stanford-bunny.obj"))
    if src == "mesh_large":
        m = rtamd.subdivide_mesh(bunny, 2)
        return cpuref.RefScene.mesh(m.vPos4f, m.indices), float(bunny.vPos4f[:, 1].min())
    sm = rtamd.SDFMesh(bunny)
    try:
        if src == "grid":
            return cpuref.RefScene.grid(*sm.grid(256)), -1.0
        return cpuref.RefScene.octree(sm.octree(8)), -1.0
    finally:
        sm.close()


def cpu_baseline(entry, budget_s, max_frames):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpuref
    src, W, H, mode, cfg, desc = entry
    threads, why = host_threads()
    sc, off = cpu_scene(src)
    sc.set_plane(mode == "default", (0.0, 1.0, 0.0), off)
    orbit = WL.orbit_positions(64)
    frames, ms_total = 0, 0.0
    t0 = time.perf_counter()
    while frames < max_frames and (frames == 0 or (time.perf_counter() - t0) < budget_s):
        vi, pi = cpuref.camera_matrices(orbit[frames % 64], aspect=W / H)
        P = cpuref.make_params(orbit[frames % 64], vi, pi, mode=0 if mode == "primary" else 1)
        _, _, _, ms = sc.render(P, W, H, threads=threads)
        ms_total += ms
        frames += 1
    return {"value": round(W * H * frames / (ms_total * 1e-3) / 1e6, 2), "unit": "Mrays/s", "cores": threads,
            "kind": "port", "ms_per_frame": round(ms_total / frames, 2),
            "sample": f"{frames} orbit frames, {src} {W}x{H} {mode}"}, why


def run_multi(scene, params, warmup, steps, W, H, devices, band_rows):
    """One process, len(devices) slots (rt_multi): every frame split into row
    bands over the devices and gathered on devices[0] (RCCL ncclGather, or peer
    copies when a device repeats). The K timed frames go out as ONE
    rt_multi_render_device_frames call (16 frames per slot launch, chunks
    pipelined inside the library) into K resident frames on devices[0].
    Returns (wall_s, exchange name, buffers of the last frame)."""
    dev = torch.device("cuda", devices[0])
    mr = rtamd.MultiRenderer(scene, devices, band_rows)
    try:
        return _timed_multi(mr, params, warmup, steps, W, H, devices, dev)
    finally:
        mr.close()


def _timed_multi(mr, params, warmup, steps, W, H, devices, dev):
    with NoGC():  # (collects before the warm-up; see NoGC)
        n, exch, _ = mr.info()
        st = stream_pool(1)[0]
        nwarm = max(warmup, 16)
        wb = [(torch.empty((H, W), dtype=torch.int32, device=dev), torch.empty((H, W), dtype=torch.float32, device=dev))
              for _ in range(min(nwarm, 16))]
        ob = [(torch.empty((H, W), dtype=torch.int32, device=dev), torch.empty((H, W), dtype=torch.float32, device=dev))
              for _ in range(steps)]
        for k0 in range(0, nwarm, len(wb)):
            m = min(len(wb), nwarm - k0)
            mr.render_device_frames([params[(k0 + i) % len(params)] for i in range(m)],
                                    [c.data_ptr() for c, _ in wb[:m]], [t.data_ptr() for _, t in wb[:m]], W, H,
                                    stream=st.cuda_stream)

        def sync_all():
            for d in sorted(set(devices)):
                torch.cuda.synchronize(d)
        sync_all()
        t0 = time.perf_counter()
        mr.render_device_frames(params[warmup:warmup + steps], [c.data_ptr() for c, _ in ob],
                                [t.data_ptr() for _, t in ob], W, H, stream=st.cuda_stream)
        sync_all()
        wall = time.perf_counter() - t0
    return wall, ("rccl_gather" if exch == mr.RCCL else "peer_copy"), ob[-1]


def single_process_main(a, json_out):
    """bench.py --gpus N --single-process: the headline over N GPUs of ONE
    process (the C ABI a C++ Renderer::draw binds, rt_multi_*)."""
    key, entry = workload_entry(a.workload)
    src, W, H, mode, cfg, desc = entry
    devices = [int(x) for x in a.devices.split(",")] if a.devices else list(range(a.gpus))
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a HIP device (the renderer has no CPU path)")
    if max(devices) >= ndev:
        raise SystemExit(f"bench.py --single-process: devices {devices} but {ndev} visible")
    torch.cuda.set_device(devices[0])
    rtamd._lib.check(rtamd.lib().rt_set_device(devices[0]))
    scene, off = WL.scene_for(src)
    scene.set_plane(rtamd.Plane((0.0, 1.0, 0.0), off) if mode == "default" else None)
    params = orbit_params(max(a.warmup + a.steps, 16), W, H, mode)
    wall, exch, (lc, lt) = run_multi(scene, params, a.warmup, a.steps, W, H, devices, a.band_rows)
    k = a.warmup + a.steps - 1
    _, _, (c1, t1) = run_single(scene, params[k:k + 1], 0, 1, W, H, inflight=1)
    ok = bool(torch.equal(c1, lc) and torch.equal(t1.view(torch.int32), lt.view(torch.int32)))
    ms_step = wall * 1e3 / a.steps
    algo, _ = work_model(scene, params[a.warmup:a.warmup + min(a.steps, 64)], None, W, H)
    dropin = None if a.no_drop_in else drop_in_multi(scene, params, W, H, devices)
    out = {
        "metric": METRIC, "value": round(W * H * a.steps / wall / 1e6, 1), "unit": "Mrays/s",
        "n_gpus": len(set(devices)), "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic deterministic 64-frame camera orbit over {desc}",
        "config": {"workload": f"{key}: {desc}, {W}x{H}, "
                               f"{'primary rays (Normal shading, no plane)' if mode == 'primary' else 'default shading'}"
                               f" (BASELINE {cfg})",
                   "resolution": [W, H], "camera": "orbit r=2.5 h=0.5 fovy 45",
                   "parallelism": f"one process, {len(devices)} slots on devices {devices}, row bands of "
                                  f"{a.band_rows} rows, exchange {exch} (rt_multi)"},
        "roofline": roofline(algo, ms_step, scene.device_bytes(), None, "skipped (single-process leg)"),
        "frame_check": {"last_timed_frame_equals_one_frame_kernel": ok},
        "exchange": exch, "slots": len(devices),
        "build_id": rtamd.lib().rt_build_id().decode(),
    }
    if dropin is not None:
        out["drop_in"] = dropin
    scene.close()
    print(json.dumps(out, separators=(",", ":")), file=json_out, flush=True)
    return 0 if ok else 1


def single_process_leg(a, world):
    """N>1, rank 0, after the ranks have left: the same workload over all N
    devices from ONE child process (bench.py --single-process), so the
    driver's multi-GPU run also measures the single-process C-ABI path."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(world), "--single-process",
           "--steps", str(a.steps), "--warmup", str(a.warmup), "--workload", a.workload,
           "--band-rows", str(a.band_rows)]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "TORCHELASTIC_RUN_ID", "MASTER_PORT")}
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 300 s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"rc {r.returncode}: {(r.stderr or '')[-300:]}"}
    o = json.loads(lines[-1])
    return {"value": o["value"], "ms_per_step": o["ms_per_step"], "exchange": o["exchange"],
            "slots": o["slots"], "frame_check": o["frame_check"], "parallelism": o["config"]["parallelism"],
            "drop_in": o.get("drop_in")}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, json_out, grace_s=60.0, cmd=None, ndev=None):
    """`--gpus N` (N > 1) run without a launcher: start N rank processes of this
    same command, one per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their
    environment, rendezvous on 127.0.0.1), as torch.distributed.run would. This
    process never touches the GPU (torch.cuda.device_count() does not initialise
    it), so nothing is exec'd from a GPU-initialised process. Rank 0's JSON line
    is relayed to stdout; the exit code is the worst rank's. When one rank fails
    the others get `grace_s` to finish before their process groups are killed
    (a rank blocked in a collective with a dead peer would wait forever).
    `cmd` / `ndev` replace this command and the device count (tests).
    Returns the exit code."""
    import signal
    import subprocess
    import threading
    backend = os.environ.get("RTAMD_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count() if ndev is None else ndev
    if ndev < 1:
        print("bench.py: --gpus needs a HIP device (the renderer has no CPU path)", file=sys.stderr)
        return 2
    if backend == "nccl" and ndev < n:
        print(f"bench.py: --gpus {n} but {ndev} HIP device(s) visible; refusing to report an {n}-GPU line "
              f"(RTAMD_DIST_BACKEND=gloo shares the devices between ranks as a protocol test)", file=sys.stderr)
        return 2
    port = _free_port()
    cmd = cmd or [sys.executable, os.path.abspath(__file__), *sys.argv[1:]]
    procs = []
    for r in range(n):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n), RANK=str(r),
                   LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr,
                                      start_new_session=True))
    lines = []

    def relay():  # rank 0's stdout: the JSON line to ours, anything else to stderr
        for raw in procs[0].stdout:
            s = raw.decode(errors="replace")
            if s.startswith("{"):
                lines.append(s.strip())
            else:
                sys.stderr.write(s)
    th = threading.Thread(target=relay, daemon=True)
    th.start()

    def kill_all(why):
        for p in procs:
            if p.poll() is None:
                print(f"bench.py: killing rank {procs.index(p)} ({why})", file=sys.stderr)
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass

    # the ranks run in sessions of their own (a timeout's signal to our process
    # group does not reach them), so a SIGTERM / SIGINT to this parent kills
    # every rank still running before it exits, and so does any exception
    def on_signal(signum, _frame):
        kill_all(f"parent got signal {signum}")
        raise SystemExit(128 + signum)
    old = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        failed_at = None
        while any(p.poll() is None for p in procs):
            if failed_at is None and any(p.poll() not in (None, 0) for p in procs):
                failed_at = time.monotonic()
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                kill_all(f"a peer failed {grace_s:.0f} s ago")
            time.sleep(0.2)
    finally:
        kill_all("parent exiting")
        for sig, h in old.items():
            signal.signal(sig, h)
    th.join(timeout=10)
    rcs = [p.wait() for p in procs]
    rc = max((abs(x) for x in rcs), default=0)
    if rc == 0 and not lines:
        print("bench.py: rank 0 printed no JSON line", file=sys.stderr)
        rc = 1
    if rc == 0:
        print(lines[-1], file=json_out, flush=True)
    else:
        print(f"bench.py: rank exit codes {rcs}; no line reported", file=sys.stderr)
    return rc


def main():
    # libraries (RCCL, gloo) print banners to stdout: send fd 1 to stderr and
    # keep the real stdout for the one JSON line
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    a = parse()
    if a.group is None:
        # the timed frames split evenly over the streams, at most 16 per launch
        # (RT_MAX_BATCH): the driver's 20 frames go out as 10 + 10 on two streams,
        # whose last launches then end together; 8 + 8 + 4 left the 4-frame launch
        # alone at the end (N = 1: 0.1023 vs 0.0964 ms/frame, 3 interleaved rounds,
        # profiles/r05/group20.txt). Longer runs take 16 per launch (whole frames
        # level at 8-16; a row-band rank needs the 16).
        a.group = max(1, min(16, -(-a.steps // max(1, a.streams))))
    if not 1 <= a.group <= 16:
        raise SystemExit("--group must be 1..16 (frames per launch)")
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    key, entry = workload_entry(a.workload)
    src, W, H, mode, cfg, desc = entry
    if a.single_process:
        sys.exit(single_process_main(a, json_out))
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus, json_out))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        # never report a line for a GPU count other than the one asked for
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}")
    use_dist = world > 1 or a.dist
    pmc, pmc_err = {}, "skipped (--no-pmc or N>1)"
    if not use_dist and not a.no_pmc:
        WORKLOADS.setdefault(key, entry)
        keys = [key] + ([] if a.no_extra else [k for k in EXTRAS if k != key])
        pmc, pmc_err = pmc_counters(keys, a.group)  # child processes, before this one initialises the GPU
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a HIP device (the renderer has no CPU path)")
    if use_dist and world > ndev and os.environ.get("RTAMD_DIST_BACKEND", "nccl") == "nccl":
        raise SystemExit(f"bench.py: {world} ranks but {ndev} HIP device(s); RCCL needs one GPU per rank")
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

    scene, off = WL.scene_for(src)
    scene.set_plane(rtamd.Plane((0.0, 1.0, 0.0), off) if mode == "default" else None)
    params = orbit_params(max(a.warmup + a.steps, verify_frames(a, a.warmup)), W, H, mode)
    detail = {"cmd": " ".join(sys.argv), "headline": key}

    latency = None
    tile = None
    frame_ok = None
    if not use_dist:
        wall, launches, (lc, lt) = run_single(scene, params, a.warmup, a.steps, W, H, inflight=a.streams,
                                              batch=a.group)
        detail["headline_launch_ms"] = [round(ms, 5) for ms, _ in launches]
        detail["headline_issue_us"] = list(LAST_RUN["issue_each_us"])
        # the last timed frame (the persistent multi-frame kernel) must equal the
        # same frame rendered alone by the one-frame kernel (render_kernel): both
        # are bit-exact against the oracle in tests/, so a timed path that drops
        # or alters work shows here
        k = a.warmup + a.steps - 1
        _, _, (c1, t1) = run_single(scene, params[k:k + 1], 0, 1, W, H, inflight=1)
        frame_ok = bool(torch.equal(c1, lc) and torch.equal(t1.view(torch.int32), lt.view(torch.int32)))
        if a.streams * a.group > 1:  # one frame at a time (latency), reported beside
            nl = min(a.steps, 64)
            lwall, ll, _ = run_single(scene, params, min(a.warmup, 8), nl, W, H, inflight=1)
            lat = [ms for ms, _ in ll]
            latency = {"ms_per_frame": round(lwall * 1e3 / nl, 4), "kernel_ms_p50": round(statistics.median(lat), 5)}
    else:
        wall, kms, rs = run_distributed(scene, params, a.warmup, a.steps, a, W, H)
        tile = rs.tile
        dev_t = "cpu" if dist.get_backend() == "gloo" else "cuda"
        t = torch.tensor([wall], dtype=torch.float64, device=dev_t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        kall = torch.zeros(world, dtype=torch.float64, device=dev_t)
        kall[rank] = kms
        dist.all_reduce(kall, op=dist.ReduceOp.SUM)
        rank_kms = [round(float(x), 5) for x in kall.cpu()]
        if rank == 0:  # the assembled last frame must equal a whole-frame render of it
            _, _, (c1, t1) = run_single(scene, params[a.warmup + a.steps - 1:a.warmup + a.steps], 0, 1, W, H,
                                        inflight=1)
            fc, ft = rs.last()
            check_equal = bool(torch.equal(c1, fc) and torch.equal(t1.view(torch.int32), ft.view(torch.int32)))
        dist.barrier()
        rs.close()

    ms_step = wall * 1e3 / a.steps
    # algorithmic bytes of the WHOLE frame (every rank's bands) over the max-over-ranks wall time
    algo, per_ray = work_model(scene, params[a.warmup:a.warmup + min(a.steps, 64)], None, W, H)
    rl = roofline(algo, ms_step, scene.device_bytes(), pmc.get(key), pmc_err, a.group, pmc.get("_calib"))
    detail["headline_work_per_ray"] = per_ray
    detail["headline_pmc_per_launch"] = pmc.get(key)
    detail["pmc_calibration"] = {str(w): v for w, v in (pmc.get("_calib") or {}).items()}
    value = W * H * a.steps / wall / 1e6
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "Mrays/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic deterministic 64-frame camera orbit over {desc}",
        "config": {"workload": f"{key}: {desc}, {W}x{H}, "
                               f"{'primary rays (Normal shading, no plane)' if mode == 'primary' else 'default shading'}"
                               f" (BASELINE {cfg})",
                   "resolution": [W, H], "camera": "orbit r=2.5 h=0.5 fovy 45",
                   "parallelism": (f"row bands of {a.band_rows} rows x {world} GPUs, exchange "
                                   f"{rs.exchange}, {a.group} frames per launch and signal, {a.streams} streams")
                   if use_dist else "1 GPU, 1 thread per pixel",
                   "frames_per_launch": a.group, "streams": a.streams},
        "roofline": rl,
        # sha256 of the loaded library's sources (rt_build_id): ties the line to a source tree
        "build_id": rtamd.lib().rt_build_id().decode(),
    }
    if frame_ok is not None:
        out["frame_check"] = {"last_timed_frame_equals_one_frame_kernel": frame_ok}
    if latency is not None:
        out["frame_latency"] = latency
    if not use_dist and a.streams > 1:
        out["roofline"]["one_stream"] = one_stream_leg(scene, params, a.warmup, a.steps, W, H, a.group, algo,
                                                       rl["peak"], rl["peak_kind"])
    if use_dist:
        out["rank_kernel_ms_per_frame"] = {"per_rank": rank_kms, "max": max(rank_kms)}
    if use_dist and rank == 0:
        v = rs.verified
        out["frame_check"] = {"assembled_equals_single_render": check_equal and not v["differing"],
                              "last_timed_frame": check_equal,
                              "verify_pass": {"frames_checked": v["frames"], "differing": v["differing"][:16],
                                              **({"p2p_differing": v["p2p_differing"][:16]}
                                                 if "p2p_differing" in v else {})},
                              "backend": dist.get_backend(), "exchange": rs.exchange,
                              "fallback": getattr(rs, "fallback", None)}
        out["host_issue_ms_per_frame"] = round(rs.host_issue_s * 1e3 / a.steps, 4)
    if rank == 0 and not use_dist and not a.no_drop_in:
        out["drop_in"] = drop_in(scene, params, W, H)
        # rt_multi_render's host-buffer path, rehearsed with two slots on this GPU
        out["drop_in"]["multi_rehearsal"] = drop_in_multi(scene, params, W, H, [device, device])
    scene.close()
    if rank == 0 and not use_dist and not a.no_extra:
        out["extra"] = {k: measure(k, WORKLOADS[k], min(a.warmup, 16), min(a.steps, 64), a.streams, a.group, pmc,
                                   pmc_err, detail)
                        for k in EXTRAS if k != key}
    if rank == 0 and not use_dist and not a.no_cpu_baseline:
        share = 1.0 - sum(s for _, s, _ in CPU_SAMPLES) if not a.no_extra else 1.0
        cb, why = cpu_baseline(entry, a.cpu_seconds * share, 64)
        cb.update({"nproc": os.cpu_count(), "cpu_model": cpu_model(), "threads_from": why,
                   "impl": "oracle/cpuref.cpp (ISPC kernels as scalar C++), OpenMP schedule(dynamic) over rows, "
                           "std::chrono around the pixel loop as Renderer::draw"})
        if not a.no_extra:
            for k, s, mx in CPU_SAMPLES:
                if k != key:
                    cb[k], _ = cpu_baseline(WORKLOADS[k], a.cpu_seconds * s, mx)
        out["cpu_baseline"] = cb
    if use_dist:
        dist.barrier()
        sp_leg = (rank == 0 and not a.no_single_process_leg and dist.get_backend() == "nccl" and ndev >= world)
        dist.destroy_process_group()
        if sp_leg:  # the other ranks exit now; their GPUs are free for the child
            out["single_process"] = single_process_leg(a, world)
    if rank == 0:
        try:
            os.makedirs(os.path.dirname(a.detail), exist_ok=True)
            with open(a.detail, "w") as f:
                json.dump(detail, f, indent=1)
            out["detail_file"] = os.path.relpath(a.detail, ROOT)
        except OSError as e:
            out["detail_file"] = f"not written: {e}"
        line = json.dumps(out, separators=(",", ":"))
        print(f"bench line: {len(line)} bytes", file=sys.stderr, flush=True)
        print(line, file=json_out, flush=True)


if __name__ == "__main__":
    main()
