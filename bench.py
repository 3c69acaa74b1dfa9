#!/usr/bin/env python3
"""bench.py -- primary-ray throughput of the MI355X renderer (BASELINE.json metric).

Metric: "Mrays/sec + ms/frame at 1920x1080, bunny tris & SDF grid, 1/2/4/8 MI355X".
Workload (N=1 and N>1): BASELINE configs[1], stanford-bunny.obj triangles at
1920x1080, primary rays (Normal shading, no ground plane: one ray per pixel,
the pure intersection hot path), over a deterministic 64-frame camera orbit
(SURVEY.md 8(d)). A "step" is one frame. Orbit frames are independent: up to
--group (8) of them go out in ONE launch (the persistent kernel pulls 8x8 pixel
tiles of all of them from one work queue), and launches alternate over
--streams (2) HIP streams with their own framebuffers. value = rays of all K
frames / wall time of the K frames.

Warm-up: every stream gets at least one full launch (and its work-queue state
via rt_stream_prepare) before t0, whatever --warmup is, so nothing is
allocated or first-used inside the timed region. The K timed frames are split
into ceil(K / group) launches of near-equal size.

At N=1 the other BASELINE configs are measured the same way under "extra"
(rank 0): the SDF grid (configs[2]; 256^3 GPU-generated stand-in and the
shipped 65^3), the octree (configs[3]; depth-8 stand-in and shipped sdf_6, both
3840x2160), the config-5 mesh stand-in (1.1 M triangles, 3840x2160, one GPU)
and the reference's DEFAULT shading mode on the bunny (plane + Lambert +
shadows + reflections), reported as primary rays/s and as traced rays/s
(primary + shadow + reflection rays, counted by the diagnostic kernel).

Roofline (per workload): achieved = ALGORITHMIC bytes per launch (SURVEY 8(d)
byte model on the reference's data layout, counted exactly by the diagnostic
variant of the same kernel over the same frames) / the render kernel's launch
duration (HIP events on the launch's own stream; frame-weighted, so a short
last launch does not inflate it), against the 8 TB/s HBM peak. These bytes are
served mostly by L1/L2 (every scene is cache-resident), so beside it:
measured DRAM bytes (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate --pmc
passes, MI355X_MICROARCH.md's gfx950 correction), the VALU issue fraction
(SQ_INSTS_VALU x 2 cycles per wave64 instruction on SIMD-32 / (1024 SIMDs x
2.4 GHz x duration); the 4-cycle single-wave form beside it) and the L2 hit
rate. "binding" names the largest of those fractions.

Multi-GPU (torch.distributed.run, one process per GPU; rtamd.rowsplit): every
frame is split into --band-rows (8) row bands dealt round-robin to the ranks,
with the same launches. Exchange p2p (default): each rank's kernel stores its
HIT pixels straight into rank 0's frame slots over xGMI (IPC-mapped) and one
4-byte RCCL all-reduce per group signals completion; exchange gather: one RCCL
gather per group of packed bands + a de-interleave on rank 0. Total work per
step is one 1080p frame whatever N is ("strong"); value = pixels of all frames /
max-over-ranks wall time. Every rank reports its own render-kernel time per
launch (rank_kernel_ms; the max over ranks bounds the scaling). rank 0 checks
that its last assembled frame equals a whole-frame render.

cpu_baseline: the oracle (C++ restatement of the reference's CPU path, ISPC
kernels as scalar C++) on every CPU this process is granted (the smallest of
the affinity set, the cgroup quota and OMP_NUM_THREADS; see host_threads),
OpenMP schedule(dynamic) over rows, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import ctypes
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
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
L2_PEAK_GBS = 34500.0  # aggregate L2 (MI355X_MICROARCH.md, L2 per XCD)
SIMDS, CLOCK_HZ = 1024, 2.4e9  # 256 CUs x 4 SIMDs, max clock
W_IMG, H_IMG = 1920, 1080

# key -> (input, W, H, mode, description); the headline is "bunny"
WORKLOADS = {
    "bunny": ("stanford-bunny.obj", 1920, 1080, "primary", "shipped stanford-bunny.obj (69,451 triangles)"),
    "grid": ("grid", 1920, 1080, "primary", WL.STANDINS["grid"]),
    "grid_shipped": ("example_grid.grid", 1920, 1080, "primary", "shipped example_grid.grid (65^3)"),
    "octree": ("octree", 3840, 2160, "primary", WL.STANDINS["octree"]),
    "octree_shipped": ("sdf_6.octree", 3840, 2160, "primary", "shipped sdf_6.octree (depth 6)"),
    "mesh_large": ("mesh_large", 3840, 2160, "primary", WL.STANDINS["mesh_large"] + ", 1 GPU"),
    "default_mode": ("stanford-bunny.obj", 1920, 1080, "default",
                     "stanford-bunny.obj, the reference's default shading: ground plane + Lambert + shadows + "
                     "one reflection (raytracing.cpp:13-65)"),
}
EXTRAS = ["grid", "grid_shipped", "octree", "octree_shipped", "mesh_large", "default_mode"]


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
                    help="frames per launch (at most 8); N>1: also per completion signal / gather")
    ap.add_argument("--depth", type=int, default=3, help="N>1: groups whose slots are in flight")
    ap.add_argument("--streams", type=int, default=2, help="HIP streams the launches alternate over")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="wall budget of the CPU sample")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 counter passes")
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


def orbit_params(n, W=W_IMG, H=H_IMG, mode="primary"):
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
    serialise the 'overlapping' launches (seen as every 4th rank of
    tools/ab.py split running at one-stream speed). Four consecutive pool
    streams, never the null stream."""
    while len(_POOL) < max(k, 4):
        _POOL.append(torch.cuda.Stream())
    return _POOL[:k]


def run_single(scene, params, warmup, steps, W=W_IMG, H=H_IMG, inflight=2, tile=None, batch=1):
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
    for j, (k, n) in enumerate(split_launches(0, nwarm, batch)):
        issue(j, [params[(k + i) % len(params)] for i in range(n)])
    timed = split_launches(warmup, steps, batch)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in timed]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j, (k, n) in enumerate(timed):
        issue(j, params[k:k + n], evs[j])
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    launches = [(a.elapsed_time(b), n) for (a, b), (_, n) in zip(evs, timed)]
    jl, (kl, nl) = len(timed) - 1, timed[-1]
    return wall, launches, bufs[jl % inflight][nl - 1]


def per_frame_ms(launches):
    """Frame-weighted kernel time per frame over the timed launches."""
    return sum(ms for ms, _ in launches) / sum(n for _, n in launches)


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
        # warm every stream and slot group the timed region will use
        r.render(params[:max(warmup, a.group * a.streams * a.depth)])
        r.drain()
        return r

    rs = make(a.exchange)
    # the warm-up's last assembled frame must equal a whole-frame render on rank 0;
    # a p2p exchange that fails this (IPC mapping, peer-store visibility) is replaced
    # by the RCCL gather before anything is timed
    ok = 1
    nw = max(warmup, a.group * a.streams * a.depth)
    if dist.get_rank() == 0:
        _, _, (c1, t1) = run_single(scene, params[nw - 1:nw], 0, 1, inflight=1)
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
    _, launches, _ = run_single(scene, params[warmup:warmup + n], 0, n, inflight=a.streams, tile=rs.tile,
                                batch=a.group)
    return wall, per_frame_ms(launches) * a.group, rs


def roofline(scene, params, tile, kms, frames_per_launch, W=W_IMG, H=H_IMG):
    """algorithmic bytes per launch (counted exactly by the
    diagnostic kernel over the same frames) / the event-timed launch duration,
    against the HBM peak. The PMC-measured fields are added by attach_pmc()."""
    c = scene.count_work(params, W, H, clear=True, tile=tile)
    npx = (rtamd.lib().rt_tile_pixels(W, H, ctypes.byref(tile)) if tile is not None else W * H)
    algo = scene.algorithmic_bytes(c, npx * len(params)) / len(params) * frames_per_launch
    achieved = algo / (kms * 1e-3) / 1e9
    per_ray = {k: round(v / (npx * len(params)), 4) for k, v in c.items() if v}
    peak, kind = peak_for(achieved)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": peak, "peak_kind": kind, "unit": "GB/s",
            "frac": round(achieved / peak, 4), "traffic": None,
            "basis": "algorithmic bytes (SURVEY.md 8(d) byte model on the reference's data layout); "
                     "the scenes are cache-resident, so these bytes are served mostly by L1/L2, not DRAM",
            "algorithmic_bytes_per_launch": int(algo), "kernel_ms": round(kms, 5),
            "frames_per_launch": frames_per_launch, "work_per_ray": per_ray,
            "algorithmic_vs_l2_peak": round(achieved / L2_PEAK_GBS, 4)}


def peak_for(achieved):
    """The HBM peak, unless the algorithmic bytes arrive faster than HBM can
    deliver -- then they are cache-served by construction and the aggregate L2
    peak is the roof they are held against (a fraction above 1 of the HBM peak
    would say nothing about DRAM)."""
    if achieved <= HBM_PEAK_GBS:
        return HBM_PEAK_GBS, "hbm"
    return L2_PEAK_GBS, "l2 (algorithmic bytes above the 8 TB/s HBM peak: cache-served)"


def one_stream_roof(algo_bytes, kms):
    a = algo_bytes / (kms * 1e-3) / 1e9
    peak, kind = peak_for(a)
    return {"achieved": round(a, 1), "peak": peak, "peak_kind": kind, "frac": round(a / peak, 4)}


# ------------------------------------------------------------ PMC passes --
PMC_PASSES = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"],
    ["SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU",
     "SQ_INSTS_VMEM_RD", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "GRBM_GUI_ACTIVE"],
]
PMC_LAUNCHES = 2


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
    out = {k: {} for k in keys}
    tmp = tempfile.mkdtemp(prefix="rtamd_pmc_", dir="/tmp")
    try:
        for i, ctrs in enumerate(PMC_PASSES):
            d = os.path.join(tmp, f"p{i}")
            cmd = ["timeout", "-k", "10", "240", prof, "--pmc", *ctrs, "--output-format", "csv", "-d", d,
                   "-o", "p", "--", sys.executable, os.path.join(ROOT, "tools", "prof_frames.py"),
                   "--plan", plan, "--group", str(group), "--launches", str(PMC_LAUNCHES)]
            r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True)
            if r.returncode != 0:
                return out, f"pass {ctrs} rc={r.returncode}: {r.stderr[-300:]}"
            rows = {}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if "render_" not in row["Kernel_Name"]:
                            continue
                        rows.setdefault(int(row["Dispatch_Id"]), {})[row["Counter_Name"]] = \
                            float(row["Counter_Value"])
            disp = [rows[k] for k in sorted(rows)]
            if len(disp) != PMC_LAUNCHES * len(keys):
                return out, f"pass {ctrs}: {len(disp)} render dispatches, expected {PMC_LAUNCHES * len(keys)}"
            for j, k in enumerate(keys):
                mine = disp[j * PMC_LAUNCHES:(j + 1) * PMC_LAUNCHES]
                for c in ctrs:
                    out[k][c] = sum(m.get(c, 0.0) for m in mine) / len(mine)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return out, None


def attach_pmc(rl, ctr, err):
    """Add the counter-derived roofs to a roofline dict (per launch of the same shape)."""
    if err or not ctr or "FETCH_SIZE" not in ctr or "SQ_INSTS_VALU" not in ctr:
        rl["pmc_error"] = err or "no counters"
        return rl
    fetch = 2.0 * ctr["FETCH_SIZE"] * 1024.0  # gfx950: FETCH_SIZE reports half of the bytes; KiB -> B
    write = ctr["WRITE_SIZE"] * 1024.0
    dur = rl["kernel_ms"] * 1e-3
    rl["traffic"] = round(fetch + write)
    dram_gbs = (fetch + write) / dur / 1e9
    valu = ctr["SQ_INSTS_VALU"]
    issue2 = valu * 2.0 / (SIMDS * CLOCK_HZ * dur)
    issue4 = valu * 4.0 / (SIMDS * CLOCK_HZ * dur)
    hits, miss = ctr.get("TCC_HIT_sum", 0.0), ctr.get("TCC_MISS_sum", 0.0)
    rl["dram"] = {"fetch_bytes": round(fetch), "write_bytes": round(write), "achieved": round(dram_gbs, 1),
                  "frac": round(dram_gbs / HBM_PEAK_GBS, 4),
                  "correction": "FETCH_SIZE x2 (gfx950), KiB -> B"}
    rl["valu_issue"] = {"insts_per_launch": round(valu), "frac": round(issue2, 4),
                        "frac_4cyc": round(issue4, 4),
                        "model": "SQ_INSTS_VALU x 2 cycles (wave64 on SIMD-32) / (1024 SIMDs x 2.4 GHz x "
                                 "launch duration); frac_4cyc: the single-wave 4-cycle issue cost"}
    rl["l2"] = {"hit_rate": round(hits / (hits + miss), 4) if hits + miss else None,
                "tcp_to_tcc_read_req": round(ctr.get("TCP_TCC_READ_REQ_sum", 0.0)),
                "tcp_accesses": round(ctr.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0))}
    rl["sq"] = {k: round(ctr[k]) for k in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU",
                                           "SQ_INSTS_VMEM_RD", "GRBM_GUI_ACTIVE") if k in ctr}
    roofs = {"dram": rl["dram"]["frac"], "valu_issue": issue2, "algorithmic_vs_l2": rl["algorithmic_vs_l2_peak"]}
    top = max(roofs, key=roofs.get)
    rl["binding"] = top if roofs[top] >= 0.5 else \
        f"latency: no throughput roof above {roofs[top]:.2f} (largest: {top})"
    return rl


# ------------------------------------------------------------ workloads --
def measure(key, warmup, steps, streams, group, pmc, pmc_err, scene=None):
    src, W, H, mode, desc = WORKLOADS[key]
    own = scene is None
    if own:
        scene, off = WL.scene_for(src)
    else:
        off = None
    if mode == "default":
        if off is None:
            off = WL.load_input(src)[2]
        scene.set_plane(rtamd.Plane((0.0, 1.0, 0.0), off))
    else:
        scene.set_plane(None)
    prm = orbit_params(warmup + steps, W, H, mode)
    wall, launches, _ = run_single(scene, prm, warmup, steps, W, H, inflight=streams, batch=group)
    kms = per_frame_ms(launches) * group
    rl = attach_pmc(roofline(scene, prm[warmup:], None, kms, group, W, H), pmc.get(key), pmc_err)
    amort = [ms / n for ms, n in launches]
    out = {"workload": f"{desc}, {W}x{H}, {'primary rays (Normal shading, no plane)' if mode == 'primary' else 'default mode'}, "
                       "same orbit",
           "value": round(W * H * steps / wall / 1e6, 1), "unit": "Mrays/s",
           "ms_per_step": round(wall * 1e3 / steps, 4), "steps": steps,
           "kernel_ms_per_frame": {"mean": round(per_frame_ms(launches), 5),
                                   "p50": round(statistics.median(amort), 5)},
           "roofline": rl}
    if mode == "default":
        rays = rl["work_per_ray"].get("rays", 1.0)
        out["traced_rays_per_pixel"] = rays
        out["traced_value"] = round(W * H * rays * steps / wall / 1e6, 1)
        out["value_note"] = ("value = primary rays (pixels) per second; traced_value counts every ray the "
                             "frame traces (primary + shadow + reflection + reflection shadow)")
    if streams > 1:  # the same launches on ONE stream: a launch's duration is its own
        w1, l1, _ = run_single(scene, prm, warmup, steps, W, H, inflight=1, batch=group)
        k1 = per_frame_ms(l1) * group
        out["one_stream"] = {"ms_per_step": round(w1 * 1e3 / steps, 4), "kernel_ms": round(k1, 5),
                             **one_stream_roof(rl["algorithmic_bytes_per_launch"], k1)}
    if own:
        scene.close()
    torch.cuda.synchronize()
    return out


def cpu_baseline(name, budget_s, mode="primary", max_frames=64):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpuref  # the oracle: test infrastructure, used here only as the CPU baseline
    from rtamd import data
    p = data.path(name)
    threads, why = host_threads()
    v, i = cpuref.load_obj(p)
    sc = cpuref.RefScene.mesh(v, i)
    if mode == "default":
        sc.set_plane(True, (0.0, 1.0, 0.0), float((v[:, 1] / v[:, 3]).min()))
    else:
        sc.set_plane(False)
    orbit = WL.orbit_positions(64)
    frames, ms_total = 0, 0.0
    t0 = time.perf_counter()
    while frames < max_frames and (time.perf_counter() - t0) < budget_s:
        vi, pi = cpuref.camera_matrices(orbit[frames % 64], aspect=W_IMG / H_IMG)
        P = cpuref.make_params(orbit[frames % 64], vi, pi, mode=0 if mode == "primary" else 1)
        _, _, _, ms = sc.render(P, W_IMG, H_IMG, threads=threads)
        ms_total += ms
        frames += 1
    mrays = W_IMG * H_IMG * frames / (ms_total * 1e-3) / 1e6
    return {"value": round(mrays, 2), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "ms_per_frame": round(ms_total / frames, 2), "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "threads_from": why,
            "sample": f"{frames} frames of the 64-frame orbit, {name} {W_IMG}x{H_IMG} "
                      f"{'primary rays' if mode == 'primary' else 'default mode (plane + Lambert + shadows + reflection)'}, "
                      f"OpenMP schedule(dynamic) over rows on {threads} threads ({why}), timed "
                      f"around the pixel loop as Renderer::draw does; ISPC kernels as scalar C++ (oracle/cpuref.cpp)"}


def main():
    # libraries (RCCL, gloo) print banners to stdout: send fd 1 to stderr and
    # keep the real stdout for the one JSON line
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    a = parse()
    if not 1 <= a.group <= 8:
        raise SystemExit("--group must be 1..8 (frames per launch)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    use_dist = world > 1 or a.dist
    headline = "bunny" if a.workload == "stanford-bunny.obj" else None
    pmc, pmc_err = {}, "skipped (--no-pmc or N>1)"
    if not use_dist and not a.no_pmc:
        keys = ([headline] if headline else []) + ([] if a.no_extra else EXTRAS)
        if keys:  # child processes, before this one initialises the GPU
            pmc, pmc_err = pmc_counters(keys, a.group)
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
    params = orbit_params(max(a.warmup + a.steps, a.group * a.streams * a.depth))

    latency = None
    if not use_dist:
        wall, launches, _ = run_single(scene, params, a.warmup, a.steps, inflight=a.streams, batch=a.group)
        kms = per_frame_ms(launches) * a.group
        amort = [ms / n for ms, n in launches]
        tile = None
        if a.streams * a.group > 1:  # one frame at a time (latency), reported beside
            nl = min(a.steps, 64)
            lwall, ll, _ = run_single(scene, params, min(a.warmup, 8), nl, inflight=1)
            lat = [ms for ms, _ in ll]
            latency = {"ms_per_frame": round(lwall * 1e3 / nl, 4), "kernel_ms_mean": round(statistics.mean(lat), 5),
                       "kernel_ms_p50": round(statistics.median(lat), 5), "frames": nl}
    else:
        wall, kms, rs = run_distributed(scene, params, a.warmup, a.steps, a)
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
            _, _, (c1, t1) = run_single(scene, params[a.warmup + a.steps - 1:a.warmup + a.steps], 0, 1, inflight=1)
            fc, ft = rs.last()
            check_equal = bool(torch.equal(c1, fc) and torch.equal(t1.view(torch.int32), ft.view(torch.int32)))
        dist.barrier()
        rs.close()

    rl = roofline(scene, params[a.warmup:a.warmup + a.steps], tile, kms, a.group)
    if headline and not use_dist:
        attach_pmc(rl, pmc.get(headline), pmc_err)
    value = W_IMG * H_IMG * a.steps / wall / 1e6
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
    if not use_dist:
        out["kernel_ms_per_frame"] = {"mean": round(per_frame_ms(launches), 5),
                                      "p50": round(statistics.median(amort), 5)}
    if latency is not None:
        out["frame_latency"] = latency
    if not use_dist and a.streams > 1:
        w1, l1, _ = run_single(scene, params, a.warmup, a.steps, inflight=1, batch=a.group)
        k1 = per_frame_ms(l1) * a.group
        out["roofline_one_stream"] = {"streams": 1, "ms_per_step": round(w1 * 1e3 / a.steps, 4),
                                      "kernel_ms": round(k1, 5),
                                      **one_stream_roof(rl["algorithmic_bytes_per_launch"], k1)}
    if use_dist:
        out["rank_kernel_ms"] = {"per_rank": rank_kms, "max": max(rank_kms),
                                 "note": "render-kernel ms per launch of this rank's bands "
                                         f"({a.group} frames, {a.streams} streams); the max bounds the scaling"}
    if use_dist and rank == 0:
        out["frame_check"] = {"assembled_equals_single_render": check_equal,
                              "backend": dist.get_backend(), "exchange": rs.exchange,
                              "fallback": getattr(rs, "fallback", None)}
        out["host_issue_ms_per_frame"] = round(rs.host_issue_s * 1e3 / a.steps, 4)
    if rank == 0 and not use_dist and not a.no_extra:
        out["extra"] = {k: measure(k, min(a.warmup, 16), min(a.steps, 64), a.streams, a.group, pmc, pmc_err)
                        for k in EXTRAS}
    if rank == 0 and not use_dist and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.workload, a.cpu_seconds)
        if not a.no_extra:
            out["cpu_baseline"]["default_mode"] = cpu_baseline(a.workload, a.cpu_seconds / 3, "default", 16)
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
