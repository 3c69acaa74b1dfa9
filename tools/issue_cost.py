"""Host issue cost of the row-split path, per group of 8 frames (nccl, world 1
under torchrun): rt_render_device_frames alone, the 4-byte RCCL signal alone,
and RowSplitRenderer.render per group (p2p exchange). The host-side time of
each piece is what an N-GPU run pays per group on every rank while its GPU
share of the frame shrinks as 1/N.
usage: python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1
       --master-port P tools/issue_cost.py"""
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))
import bench  # noqa: E402
import rtamd  # noqa: E402
from rtamd import workloads as WL  # noqa: E402
from rtamd.rowsplit import RowSplitRenderer  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
W, H, G = 1920, 1080, 8
scene, _ = WL.scene_for(bench.workload_entry("bunny")[1][0])
params = bench.orbit_params(64, W, H)
dev = torch.device("cuda")
bufs = [(torch.empty((H, W), dtype=torch.int32, device=dev), torch.empty((H, W), dtype=torch.float32, device=dev))
        for _ in range(G)]
st = torch.cuda.Stream()
cp = [c.data_ptr() for c, _ in bufs]
tp = [t.data_ptr() for _, t in bufs]


def per_call(fn, n=16):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    return dt * 1e3


with torch.cuda.stream(st):
    ms_launch = per_call(lambda: scene.render_device_frames(params[:G], cp, tp, W, H, rtamd.RT_FLAG_CLEAR,
                                                            stream=st.cuda_stream))
    sig = torch.zeros(1, dtype=torch.int32, device=dev)
    ms_sig = per_call(lambda: dist.all_reduce(sig, async_op=True))
    ms_sig_wait = per_call(lambda: dist.all_reduce(sig, async_op=True).wait())
    ev = torch.cuda.Event()
    ms_ev = per_call(lambda: (ev.record(st), st.wait_event(ev)))
rs = RowSplitRenderer(scene, W, H, band_rows=8, group=G, depth=3, streams=2, exchange="p2p")
rs.render(params[:48])
rs.drain()
torch.cuda.synchronize()
t0 = time.perf_counter()
rs.render(params[:64])
ms_rs = (time.perf_counter() - t0) * 1e3 / (64 // G)
rs.drain()
print(f"host ms per group of {G} frames: rt_render_device_frames {ms_launch:.3f}, RCCL signal (async) "
      f"{ms_sig:.3f}, signal + wait {ms_sig_wait:.3f}, event record+wait {ms_ev:.3f}, "
      f"RowSplitRenderer.render {ms_rs:.3f} (exchange {rs.exchange})", flush=True)
rs.close()
dist.destroy_process_group()
