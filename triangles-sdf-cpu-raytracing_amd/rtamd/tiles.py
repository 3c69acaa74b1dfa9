"""Row-band tiling of a frame across ranks (rt_tile in include/rtamd.h).

Image rows are cut into bands of `band_rows`; band b belongs to rank b % n.
A rank renders its bands packed in increasing band order. These host-side
helpers define the same layout as the device kernels (render_kernel's
image_row / untile_kernel) for planning buffers and for CPU-side checks.
"""
from __future__ import annotations

import numpy as np


def rank_rows(H: int, band_rows: int, rank: int, nranks: int) -> np.ndarray:
    """Image rows owned by `rank`, in packed order."""
    if nranks <= 1:
        return np.arange(H)
    rows = []
    nb = (H + band_rows - 1) // band_rows
    for b in range(rank, nb, nranks):
        rows.extend(range(b * band_rows, min(H, (b + 1) * band_rows)))
    return np.asarray(rows, dtype=np.int64)


def untile_host(packed: list, H: int, band_rows: int) -> np.ndarray:
    """Reassemble per-rank packed [rows_r, W] arrays into the [H, W] frame."""
    n = len(packed)
    W = packed[0].shape[1]
    out = np.empty((H, W), packed[0].dtype)
    for r in range(n):
        out[rank_rows(H, band_rows, r, n)] = packed[r]
    return out
