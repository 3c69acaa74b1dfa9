"""Multi-rank frame split on CPU (gloo, world_size 2 and 3): each rank renders
its row bands (with the oracle, standing in for its GPU), packs them, one
gather brings them to rank 0, which reassembles the frame: identical to the
single-rank frame. Exercises the same band layout as rt_tile / untile_kernel."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, band, result_path):
    import sys
    sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "oracle", "triangles-sdf-cpu-raytracing_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RTAMD_NO_TORCH="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import scenes as S
    from rtamd.tiles import rank_rows, untile_host
    name, W, H, mode = "stanford-bunny.obj", 160, 90, "default"
    s = S.ref_scene(name)
    S.set_planes(name, mode, s)
    P = S.params(name, W, H, mode)
    rows = rank_rows(H, band, rank, world)
    col = np.zeros((H, W), np.uint32)
    t = np.full((H, W), np.inf, np.float32)
    for r in rows:  # render only this rank's rows
        s.render(P, W, H, col, t, rows=(int(r), int(r) + 1), threads=1)
    packed = np.concatenate([col[rows].view(np.int32), t[rows].view(np.int32)], axis=1)
    cap = max(len(rank_rows(H, band, q, world)) for q in range(world))
    buf = torch.zeros((cap, 2 * W), dtype=torch.int32)
    buf[: len(rows)] = torch.from_numpy(packed)
    gl = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=gl, dst=0)
    if rank == 0:
        parts_c, parts_t = [], []
        for q in range(world):
            n = len(rank_rows(H, band, q, world))
            a = gl[q][:n].numpy()
            parts_c.append(a[:, :W].view(np.uint32))
            parts_t.append(a[:, W:].view(np.float32))
        full_c = untile_host(parts_c, H, band)
        full_t = untile_host(parts_t, H, band)
        rc, rt_ = S.ref_frame(name, W, H, mode)
        ok = np.array_equal(full_c, rc) and np.array_equal(full_t.view(np.uint32), rt_.view(np.uint32))
        with open(result_path, "w") as f:
            f.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 16), (3, 7)])
def test_gloo_band_split_gather(tmp_path, world, band):
    out = tmp_path / "result.txt"
    mp.start_processes(_worker, args=(world, _free_port(), band, str(out)), nprocs=world,
                       join=True, start_method="spawn")
    assert out.read_text() == "ok"
