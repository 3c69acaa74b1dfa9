"""Row-split multi-GPU rendering: one process per GPU, frames cut into row bands.

The reference renders a frame with one OpenMP loop over rows
(src/raytracing.cpp:77-96); rows are independent, so here band b of
`band_rows` rows belongs to rank b % world (rt_tile, include/rtamd.h) and the
frame is assembled on rank 0. Two exchanges deliver the bands:

``p2p`` (default): rank 0 owns S = group * depth frame slots in uncached device
memory (rt_exchange_alloc) and exports them (rt_ipc_get_handle); every rank
maps them (rt_ipc_open) and its render kernel stores its HIT pixels straight
into rank 0's frame over xGMI (RT_FLAG_TILE_NATURAL | RT_FLAG_CLEAR |
RT_FLAG_HITS_ONLY). Misses keep the value rank 0's clear wrote, exactly as
FrameBuffer::clear() + draw (src/raytracing.hpp:16-19, raytracing.cpp:91-94),
so the bytes crossing xGMI are 8 per hit pixel (bunny at 1080p: ~14% of the
frame) instead of 8 per pixel. Each wave of those launches ends with a
system-scope release after its last peer store (peer_release, rt_device.hip),
so the peer pixels are visible before the kernel completes. The only
collective is one 4-byte RCCL all-reduce per GROUP of frames, a stream-ordered
completion signal enqueued after the render: when it completes on a rank,
every rank's renders of that group have finished.

``gather``: every rank renders its bands packed into a local buffer, ONE RCCL
gather per group brings 8 B/pixel to rank 0, which de-interleaves them on the
device (rt_untile_device). Used when IPC mapping is unavailable.

Slot protocol (p2p; group g = frames [g*G, (g+1)*G), slots of group g =
g mod depth):
  rank 0: waits until group g-depth's slots were cleared; renders g;
          after signal g-1: hands group g-1's frames to `on_frame`, clears its
          slots (stream B), then sends signal g (so signal g certifies "group g
          rendered everywhere" AND "group g-1's slots are clear for group
          g-1+depth");
  rank r>0: before rendering group g waits for signal g-depth+1 (its slots
          were cleared before rank 0 sent it); renders g; sends signal g.
Each group is ONE launch of G frames (rt_render_device_frames: a frame's
silhouette tail is covered by the next frames' tiles), and groups alternate
over `streams` streams so one launch's tail overlaps the next launch.
With depth 3 a rank renders group g while signals g-1 and g-2 are in flight.
With the gloo backend (ranks sharing one GPU, a protocol test) each signal is
a host-synchronous all-reduce after the rank's stream has drained.

Every device operation goes through a `device` object (HipDevice here), so
the same protocol code runs against a host emulation of the device in the CPU
tests (tests/rowsplit_host.py: gloo ranks, a shared file as rank 0's exported
memory, the oracle as the renderer).
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist

from ._lib import (RT_FLAG_CLEAR, RT_FLAG_HITS_ONLY, RT_FLAG_TILE_NATURAL, RT_IPC_HANDLE_BYTES, Tile,
                   check, lib)

__all__ = ["RowSplitRenderer", "HipDevice"]


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


class _Done:
    def wait(self):
        return None


class _DevBuf:
    """A device pointer as a torch tensor view (no copy), via __cuda_array_interface__."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 2, "strides": None}


def device_view(ptr: int, n: int, dtype: torch.dtype) -> torch.Tensor:
    typestr = {torch.int32: "<i4", torch.float32: "<f4"}[dtype]
    return torch.as_tensor(_DevBuf(ptr, n, typestr), device=torch.device("cuda", torch.cuda.current_device()))


class HipDevice:
    """This rank's GPU as the row-split protocol uses it: torch streams and
    events, and librtamd's exchange allocation, IPC, clear, render and untile
    entry points (include/rtamd.h)."""

    def __init__(self):
        self.tensor_device = torch.device("cuda", torch.cuda.current_device())
        self._free_events = []

    # streams and events
    def stream(self):
        return torch.cuda.Stream()

    def on(self, st):
        return torch.cuda.stream(st)

    def event(self, st):
        # recycled events (release_event): a fresh torch event creates its HIP
        # event lazily at its first record, inside the caller's issue loop
        ev = self._free_events.pop() if self._free_events else torch.cuda.Event()
        ev.record(st)
        return ev

    def release_event(self, ev):
        """ev's last wait is enqueued: it may be recorded again."""
        self._free_events.append(ev)

    def wait_event(self, st, ev):
        st.wait_event(ev)

    def sync_stream(self, st):
        st.synchronize()

    def synchronize(self):
        torch.cuda.synchronize()

    # rank 0's exported frame slots
    def exchange_alloc(self, nbytes: int):
        p = C.c_void_p()
        return p.value if lib().rt_exchange_alloc(nbytes, C.byref(p)) == 0 else None

    def exchange_free(self, ptr: int):
        lib().rt_exchange_free(C.c_void_p(ptr))

    def ipc_handle(self, ptr: int, out: torch.Tensor) -> bool:
        return lib().rt_ipc_get_handle(C.c_void_p(ptr), out.numpy().ctypes.data) == 0

    def ipc_open(self, handle: torch.Tensor):
        p = C.c_void_p()
        return p.value if lib().rt_ipc_open(handle.numpy().ctypes.data, C.byref(p)) == 0 else None

    def ipc_close(self, ptr: int):
        lib().rt_ipc_close(C.c_void_p(ptr))

    # frames
    def clear(self, c: int, t: int, nwords: int, st):
        check(lib().rt_clear_device(C.c_void_p(c), C.c_void_p(t), nwords, C.c_void_p(st.cuda_stream)))

    def render(self, scene, params, cps, tps, W, H, flags, tile, st):
        scene.render_device_frames(params, cps, tps, W, H, flags, tile=tile, stream=st.cuda_stream)

    def tile_pixels(self, W: int, H: int, tile) -> int:
        return lib().rt_tile_pixels(W, H, C.byref(tile))

    def untile(self, c: int, t: int, stride_words: int, fc: torch.Tensor, ft: torch.Tensor, W, H, tile0, st):
        check(lib().rt_untile_device(C.c_void_p(c), C.c_void_p(t), stride_words, C.c_void_p(fc.data_ptr()),
                                     C.c_void_p(ft.data_ptr()), W, H, C.byref(tile0), C.c_void_p(st.cuda_stream)))

    def view(self, ptr: int, n: int, dtype: torch.dtype) -> torch.Tensor:
        return device_view(ptr, n, dtype)


class RowSplitRenderer:
    """Renders frames of `scene` (an rtamd IScene on this rank's GPU) split by
    row bands across the ranks of the default process group.

    `on_frame(k, color [H, W] int32, t [H, W] float32)` is called on rank 0 for
    every assembled frame, k = its position among all frames issued to render()
    (counted across calls), in order, inside the stream context that orders
    the frame's completion before its slot is reused: torch work it enqueues
    (a copy, a checksum) sees the whole frame. The views are valid only during
    the call."""

    def __init__(self, scene, W: int, H: int, band_rows: int = 8, group: int = 8, depth: int = 3,
                 streams: int = 2, exchange: str = "p2p", device=None, on_frame=None):
        if exchange not in ("p2p", "gather"):
            raise ValueError(f"unknown exchange {exchange!r}")
        self.dv = device if device is not None else HipDevice()
        self.scene, self.W, self.H = scene, W, H
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.sync_signals = dist.get_backend() != "nccl"  # gloo: host-synchronous signals
        self.G, self.D = max(1, group), max(2, depth)
        self.S = self.G * self.D
        self.tile = Tile(band_rows, self.rank, self.world, 0)
        self.tiles = [Tile(band_rows, r, self.world, 0) for r in range(self.world)]
        self.dev = self.dv.tensor_device
        self.streams = [self.dv.stream() for _ in range(max(1, streams))]
        self.clear_stream = self.dv.stream() if self.rank == 0 else None
        self._sig = [torch.zeros(1, dtype=torch.int32,
                                 device="cpu" if self.sync_signals else self.dev) for _ in range(self.D)]
        self.on_frame = on_frame
        self.works = {}
        self.ev_clear = {}
        self.nframes = {}
        self.first = {}  # group -> sequence number of its first frame (frames issued before it)
        self.issued = 0
        self.next_group = 0
        self.consumed = -1  # last group handed to on_frame
        self.last_frame = -1
        self._mapped = None
        self._alloc = None
        self.exchange = exchange
        if exchange == "p2p" and not self._setup_p2p():
            self.exchange = "gather"
        if self.exchange == "gather":
            self._setup_gather()

    # ------------------------------------------------------------- setup ---
    def _setup_p2p(self) -> bool:
        npx = self.W * self.H
        self.buf_stride = _round_up(npx * 4, 256)
        self.group_stride = 2 * self.G * self.buf_stride
        nbytes = self.D * self.group_stride
        ok = 1
        handle = torch.zeros(RT_IPC_HANDLE_BYTES, dtype=torch.uint8)
        if self.rank == 0:
            p = self.dv.exchange_alloc(nbytes)
            if p is None:
                ok = 0
            else:
                self._alloc = p
                for d in range(self.D):
                    self._clear_group_slots(d, self.streams[0])
                self.dv.synchronize()
                if not self.dv.ipc_handle(self._alloc, handle):
                    ok = 0
        handle = self._bcast(handle)
        exported = self._all_ok(ok)  # every rank takes part in each collective
        if self.rank == 0:
            self._mapped = self._alloc
        elif exported:
            p = self.dv.ipc_open(handle)
            if p is None:
                ok = 0
            else:
                self._mapped = p
        if not self._all_ok(ok):
            self._close_p2p()
            return False
        return True

    def _bcast(self, t: torch.Tensor) -> torch.Tensor:
        x = t if self.sync_signals else t.to(self.dev)
        dist.broadcast(x, src=0)
        return x.cpu()

    def _all_ok(self, ok: int) -> bool:
        x = torch.tensor([ok], dtype=torch.int32, device="cpu" if self.sync_signals else self.dev)
        dist.all_reduce(x, op=dist.ReduceOp.MIN)
        return bool(x.item())

    def _close_p2p(self):
        if self._mapped is not None and self.rank != 0:
            self.dv.ipc_close(self._mapped)
        if self._alloc is not None:
            self.dv.synchronize()
            self.dv.exchange_free(self._alloc)
        self._mapped = self._alloc = None

    def _setup_gather(self):
        per = max(self.dv.tile_pixels(self.W, self.H, t) for t in self.tiles)
        self.per = _round_up(per, 64)
        # one packed buffer per depth slot: G frames x [colour (per) | t (per)] int32 words
        self.packed = [torch.zeros((self.G, 2 * self.per), dtype=torch.int32, device=self.dev)
                       for _ in range(self.D)]
        if self.rank == 0:
            self.stacked = [torch.empty((self.world, self.G, 2 * self.per), dtype=torch.int32, device=self.dev)
                            for _ in range(self.D)]
            self.frames_c = [torch.empty((self.G, self.H, self.W), dtype=torch.int32, device=self.dev)
                             for _ in range(self.D)]
            self.frames_t = [torch.empty((self.G, self.H, self.W), dtype=torch.float32, device=self.dev)
                             for _ in range(self.D)]

    # --------------------------------------------------------- signalling ---
    def _signal(self, g: int, stream):
        """Completion signal of group g, ordered after `stream`'s work."""
        t = self._sig[g % self.D]
        if self.sync_signals:
            self.dv.sync_stream(stream)
            dist.all_reduce(t)
            return _Done()
        return dist.all_reduce(t, async_op=True)

    # ------------------------------------------------------ frame handoff ---
    def _frame(self, k: int):
        """(colour, t) views of assembled frame k on rank 0."""
        if self.exchange == "p2p":
            c, t = self._slot_ptrs(self._mapped, k % self.S)
            n = self.W * self.H
            return (self.dv.view(c, n, torch.int32).view(self.H, self.W),
                    self.dv.view(t, n, torch.float32).view(self.H, self.W))
        d, i = (k // self.G) % self.D, k % self.G
        return self.frames_c[d][i], self.frames_t[d][i]

    def _consume(self, g: int):
        """Hand group g's assembled frames to on_frame (rank 0, once, in order;
        the caller has made the current stream wait for the group)."""
        if self.rank != 0 or g <= self.consumed:
            return
        assert g == self.consumed + 1, f"group {g} assembled before group {self.consumed + 1}"
        self.consumed = g
        if self.on_frame is not None:
            for i in range(self.nframes[g]):
                self.on_frame(self.first[g] + i, *self._frame(g * self.G + i))

    # ---------------------------------------------------------- p2p path ---
    def _slot_ptrs(self, base: int, s: int):
        # depth slot d = s // G holds G colour buffers, then G t buffers, so a
        # group's slots clear with one rt_clear_device
        d, i = divmod(s, self.G)
        c = base + d * self.group_stride + i * self.buf_stride
        return c, c + self.G * self.buf_stride

    def _clear_group_slots(self, d: int, st):
        c, t = self._slot_ptrs(self._alloc, d * self.G)
        self.dv.clear(c, t, self.G * self.buf_stride // 4, st)

    def _p2p_group(self, g: int, params, st):
        frames = range(g * self.G, g * self.G + len(params))
        if self.rank == 0 and g >= self.D:
            ev = self.ev_clear.pop(g - self.D)
            self.dv.wait_event(st, ev)
            self.dv.release_event(ev)
        if self.rank != 0 and g >= self.D - 1:
            self.works[g - self.D + 1].wait()  # (current stream = st)
        cp, tp = zip(*(self._slot_ptrs(self._mapped, k % self.S) for k in frames))
        flags = RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY | RT_FLAG_TILE_NATURAL
        self.dv.render(self.scene, params, cp, tp, self.W, self.H, flags, self.tile, st)
        if self.rank == 0 and g >= 1:
            B = self.clear_stream
            with self.dv.on(B):
                self.works[g - 1].wait()  # group g-1 is complete in its slots: consume, then clear
                self._consume(g - 1)
                self._clear_group_slots((g - 1) % self.D, B)
                ev = self.dv.event(B)
            self.ev_clear[g - 1] = ev
            self.dv.wait_event(st, ev)
        self.works[g] = self._signal(g, st)
        self.works.pop(g - self.D - 1, None)

    # ------------------------------------------------------- gather path ---
    def _gather_group(self, g: int, params, st):
        d = g % self.D
        pk = self.packed[d]
        w = self.works.pop(g - self.D, None)
        if w is not None:  # this depth slot's previous gather must land before its buffers are reused
            w.wait()
            if self.rank == 0:
                self._untile(d, self.nframes[g - self.D], st)
                self._consume(g - self.D)
        cp = [pk[i].data_ptr() for i in range(len(params))]
        tp = [p + 4 * self.per for p in cp]
        self.dv.render(self.scene, params, cp, tp, self.W, self.H, RT_FLAG_CLEAR, self.tile, st)
        if self.sync_signals:
            self.dv.sync_stream(st)
            host = pk.cpu()
            lst = [torch.empty_like(host) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(host, gather_list=lst, dst=0)
            if self.rank == 0:
                self.stacked[d].copy_(torch.stack(lst))
            self.works[g] = _Done()
            return
        recv = list(self.stacked[d].unbind(0)) if self.rank == 0 else None
        self.works[g] = dist.gather(pk, gather_list=recv, dst=0, async_op=True)

    def _untile(self, d: int, n: int, st):
        sk = self.stacked[d]
        for i in range(n):
            base = sk.data_ptr() + i * 2 * self.per * 4
            self.dv.untile(base, base + 4 * self.per, self.G * 2 * self.per, self.frames_c[d][i],
                           self.frames_t[d][i], self.W, self.H, self.tiles[0], st)

    # ------------------------------------------------------------ public ---
    def render(self, params_list):
        """Issue frames (rt_render_params each), in groups of `group`; returns
        without waiting. Frame numbers continue across calls."""
        i = 0
        while i < len(params_list):
            chunk = params_list[i:i + self.G]
            g = self.next_group
            st = self.streams[g % len(self.streams)]
            self.nframes[g] = len(chunk)
            self.first[g] = self.issued
            self.issued += len(chunk)
            with self.dv.on(st):
                if self.exchange == "p2p":
                    self._p2p_group(g, chunk, st)
                else:
                    self._gather_group(g, chunk, st)
            self.nframes.pop(g - 2 * self.D, None)
            self.first.pop(g - 2 * self.D, None)
            self.last_frame = g * self.G + len(chunk) - 1
            self.next_group += 1
            i += len(chunk)

    def drain(self):
        """Wait (stream-ordered, then host) until every issued frame is
        assembled on rank 0 (and handed to on_frame)."""
        st = self.streams[0]
        with self.dv.on(st):
            if self.exchange == "p2p":
                if self.next_group:
                    self.works[self.next_group - 1].wait()
                    self._consume(self.next_group - 1)
            else:
                for g in sorted(self.works):
                    self.works.pop(g).wait()
                    if self.rank == 0:
                        self._untile(g % self.D, self.nframes[g], st)
                        self._consume(g)
        self.dv.synchronize()

    def last(self):
        """(colour int32 [H, W], t float32 [H, W]) of the last frame on rank 0,
        after drain(); None on other ranks."""
        if self.rank != 0 or self.last_frame < 0:
            return None
        return self._frame(self.last_frame)

    def close(self):
        self.dv.synchronize()
        if self.exchange == "p2p":
            # peers unmap before rank 0 frees
            dist.barrier()
            if self.rank != 0:
                self._close_p2p()
            dist.barrier()
            if self.rank == 0:
                self._close_p2p()
