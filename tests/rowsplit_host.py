"""Host emulation of the device side of rtamd.rowsplit (test infrastructure).

RowSplitRenderer does every device operation through a `device` object
(rtamd.rowsplit.HipDevice on a GPU). HostDevice implements the same calls on
the CPU so the slot / signal protocol itself can run in gloo ranks here:

- rank 0's exported frame slots (rt_exchange_alloc + rt_ipc_get_handle) are a
  file in a shared directory, mapped by every rank (rt_ipc_open), so peer
  "stores" land in rank 0's memory exactly where the kernel's would;
- the render kernel is the oracle (oracle/cpuref.cpp) rendering the rank's
  row bands, stored as RT_FLAG_TILE_NATURAL | RT_FLAG_HITS_ONLY (hit pixels
  only, at their image rows) or packed (rank-local rows, every pixel);
- streams execute synchronously, so every event is already complete.

A `delay` callback (frame k -> seconds) slows chosen renders down, so ranks
drift apart and the protocol's waits are what keeps slots from being reused
early.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import mmap
import os
import time

import numpy as np
import torch

from rtamd.tiles import rank_rows


class _Stream:
    cuda_stream = 0

    def synchronize(self):
        return None


class HostDevice:
    tensor_device = torch.device("cpu")

    def __init__(self, shm_dir: str, rank: int, delay=None):
        self.dir, self.rank, self.delay = shm_dir, rank, delay
        self.maps = {}  # address -> (mmap, file)
        self.rendered = 0

    # streams and events: synchronous
    def stream(self):
        return _Stream()

    def on(self, st):
        return contextlib.nullcontext()

    def event(self, st):
        return None

    def wait_event(self, st, ev):
        return None

    def release_event(self, ev):
        return None

    def sync_stream(self, st):
        return None

    def synchronize(self):
        return None

    # exported memory: a shared file
    def _map(self, path: str, nbytes: int) -> int:
        f = open(path, "r+b")
        m = mmap.mmap(f.fileno(), nbytes)
        addr = C.addressof(C.c_char.from_buffer(m))
        self.maps[addr] = (m, f)
        return addr

    def exchange_alloc(self, nbytes: int):
        path = os.path.join(self.dir, "slots.bin")
        with open(path, "wb") as f:
            f.truncate(nbytes)
        self.nbytes = nbytes
        return self._map(path, nbytes)

    def _unmap(self, ptr: int):
        m, f = self.maps.pop(ptr)
        # drop the buffer export held by addressof's from_buffer before closing
        import gc
        gc.collect()
        try:
            m.close()
        except BufferError:
            pass
        f.close()

    def exchange_free(self, ptr: int):
        self._unmap(ptr)

    def ipc_handle(self, ptr: int, out: torch.Tensor) -> bool:
        b = f"slots.bin|{self.nbytes}".encode()  # a name in the shared directory every rank was given
        if len(b) > out.numel():
            return False
        out[:len(b)] = torch.tensor(list(b), dtype=torch.uint8)
        return True

    def ipc_open(self, handle: torch.Tensor):
        s = bytes(handle.numpy().tobytes()).rstrip(b"\0").decode()
        name, n = s.rsplit("|", 1)
        return self._map(os.path.join(self.dir, name), int(n))

    def ipc_close(self, ptr: int):
        self._unmap(ptr)

    @staticmethod
    def _arr(ptr: int, n: int, dtype) -> np.ndarray:
        return np.frombuffer((C.c_char * (n * 4)).from_address(ptr), dtype=dtype)

    def clear(self, c: int, t: int, nwords: int, st):
        self._arr(c, nwords, np.uint32)[:] = 0
        self._arr(t, nwords, np.float32)[:] = np.inf

    def render(self, scene, params, cps, tps, W, H, flags, tile, st):
        """scene = (oracle RefScene, frame params list indexed by frame number);
        params = frame numbers. Renders this rank's bands of each frame."""
        from rtamd._lib import RT_FLAG_HITS_ONLY, RT_FLAG_TILE_NATURAL
        ref, table = scene
        rows = rank_rows(H, tile.band_rows, tile.rank, tile.num_ranks)
        for k, cp, tp in zip(params, cps, tps):
            if self.delay:
                time.sleep(self.delay(self.rank, k))
            col = np.zeros((H, W), np.uint32)
            t = np.full((H, W), np.inf, np.float32)
            for r in rows:
                ref.render(table[k], W, H, col, t, rows=(int(r), int(r) + 1), threads=1)
            if flags & RT_FLAG_TILE_NATURAL:
                assert flags & RT_FLAG_HITS_ONLY
                dc = self._arr(cp, W * H, np.uint32).reshape(H, W)
                dt = self._arr(tp, W * H, np.float32).reshape(H, W)
                hit = np.isfinite(t[rows])
                dc[rows] = np.where(hit, col[rows], dc[rows])
                dt[rows] = np.where(hit, t[rows], dt[rows])
            else:
                n = len(rows) * W
                self._arr(cp, n, np.uint32)[:] = col[rows].reshape(-1)
                self._arr(tp, n, np.float32)[:] = t[rows].reshape(-1)
            self.rendered += 1

    def tile_pixels(self, W: int, H: int, tile) -> int:
        return len(rank_rows(H, tile.band_rows, tile.rank, tile.num_ranks)) * W

    def untile(self, c: int, t: int, stride_words: int, fc: torch.Tensor, ft: torch.Tensor, W, H, tile0, st):
        """Packed slot of every rank (rank r at r * stride_words words) -> frame."""
        n = tile0.num_ranks
        for r in range(n):
            rows = rank_rows(H, tile0.band_rows, r, n)
            m = len(rows) * W
            pc = self._arr(c + 4 * r * stride_words, m, np.int32).reshape(-1, W)
            pt = self._arr(t + 4 * r * stride_words, m, np.float32).reshape(-1, W)
            fc.numpy()[rows] = pc
            ft.numpy()[rows] = pt

    def view(self, ptr: int, n: int, dtype: torch.dtype) -> torch.Tensor:
        npt = {torch.int32: np.int32, torch.float32: np.float32}[dtype]
        return torch.from_numpy(self._arr(ptr, n, npt))
