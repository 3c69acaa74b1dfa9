"""RowSplitRenderer's slot and signal protocol on the CPU (gloo ranks).

The protocol code of rtamd/rowsplit.py runs unchanged; only its device is the
host emulation of tests/rowsplit_host.py (rank 0's exported slots are a shared
file every rank maps, the oracle renders each rank's bands, signals are gloo
all-reduces). Rank 0 checks EVERY assembled frame handed to on_frame against
the oracle's whole frame, over several slot-group wrap-arounds, partial last
groups, two render() calls (frame numbers continue) and ranks slowed down at
chosen frames so they drift apart."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAME, W, H, MODE = "stanford-bunny.obj", 96, 54, "primary"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _orbit(n):
    th = 2 * np.pi * np.arange(n) / 16
    return [(2.5 * float(np.sin(a)), 0.5, 2.5 * float(np.cos(a))) for a in th]


def _worker(rank, world, port, shm, exchange, group, depth, nframes, band, result_path):
    import sys
    sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "oracle", "triangles-sdf-cpu-raytracing_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RTAMD_NO_TORCH="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cpuref
    import scenes as S
    from rowsplit_host import HostDevice
    from rtamd.rowsplit import RowSplitRenderer

    ref = S.ref_scene(NAME)
    S.set_planes(NAME, MODE, ref)
    table = []
    for pos in _orbit(nframes):
        vi, pi = cpuref.camera_matrices(pos, aspect=W / H)
        table.append(cpuref.make_params(pos, vi, pi, mode=0))

    # rank r is slow on frames r, r + 5, ...: the ranks finish groups at different times
    def delay(r, k):
        return 0.02 if (k - r) % 5 == 0 else 0.0

    got = {}

    def keep(k, c, t):
        got[k] = (c.clone().numpy().view(np.uint32), t.clone().numpy())

    dv = HostDevice(shm, rank, delay=delay)
    rs = RowSplitRenderer((ref, table), W, H, band_rows=band, group=group, depth=depth, streams=2,
                          exchange=exchange, device=dv, on_frame=keep)
    assert rs.exchange == exchange
    half = nframes // 2 + 1  # two calls: frame numbers and slot rotation continue across them
    rs.render(list(range(half)))
    rs.render(list(range(half, nframes)))
    rs.drain()
    last = rs.last()
    result = "ok"
    if rank == 0:
        if sorted(got) != list(range(nframes)):
            result = f"frames handed to on_frame: {sorted(got)}"
        else:
            for k in range(nframes):
                rc, rt, _, _ = ref.render(table[k], W, H)
                c, t = got[k]
                if not (np.array_equal(c, rc) and np.array_equal(t.view(np.uint32), rt.view(np.uint32))):
                    result = f"frame {k} differs in {int((c != rc).sum())} pixels"
                    break
            lc, lt = last
            rc, rt, _, _ = ref.render(table[nframes - 1], W, H)
            if result == "ok" and not np.array_equal(lc.numpy().view(np.uint32), rc):
                result = "last() differs"
        with open(result_path, "w") as f:
            f.write(result)
    else:
        assert last is None and not got
    rs.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,exchange,group,depth,nframes,band", [
    (2, "p2p", 3, 2, 17, 8),
    (3, "p2p", 2, 3, 15, 5),
    (2, "gather", 3, 2, 14, 8),
    (3, "gather", 4, 3, 27, 7),
])
def test_rowsplit_protocol_every_frame(tmp_path, world, exchange, group, depth, nframes, band):
    out = tmp_path / "result.txt"
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), exchange, group, depth, nframes, band,
                                      str(out)), nprocs=world, join=True, start_method="spawn")
    assert out.read_text() == "ok"


def _drop_clear_worker(rank, world, port, shm, result_path):
    """A protocol bug must fail the check: with the clear of consumed slots
    disabled, frames reusing a slot keep stale hit pixels of an older frame."""
    import sys
    sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "oracle", "triangles-sdf-cpu-raytracing_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RTAMD_NO_TORCH="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cpuref
    import scenes as S
    from rowsplit_host import HostDevice
    from rtamd.rowsplit import RowSplitRenderer

    ref = S.ref_scene(NAME)
    S.set_planes(NAME, MODE, ref)
    n = 12
    table = []
    for pos in _orbit(n):
        vi, pi = cpuref.camera_matrices(pos, aspect=W / H)
        table.append(cpuref.make_params(pos, vi, pi, mode=0))
    got = {}
    rs = RowSplitRenderer((ref, table), W, H, band_rows=8, group=2, depth=2, streams=2, exchange="p2p",
                          device=HostDevice(shm, rank), on_frame=lambda k, c, t: got.__setitem__(k, c.clone()))
    rs._clear_group_slots = lambda d, st: None  # the bug
    rs.render(list(range(n)))
    rs.drain()
    if rank == 0:
        bad = 0
        for k in range(n):
            rc, _, _, _ = ref.render(table[k], W, H)
            bad += int(not np.array_equal(got[k].numpy().view(np.uint32), rc))
        with open(result_path, "w") as f:
            f.write(str(bad))
    rs.close()
    dist.barrier()
    dist.destroy_process_group()


def test_rowsplit_protocol_check_catches_stale_slots(tmp_path):
    out = tmp_path / "result.txt"
    mp.start_processes(_drop_clear_worker, args=(2, _free_port(), str(tmp_path), str(out)), nprocs=2, join=True,
                       start_method="spawn")
    assert int(out.read_text()) > 0
