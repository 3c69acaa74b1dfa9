"""The pageable drop-in's host copy (rth::copy_spans, rt_device.hip
render_cleared_zero_copy) on the CPU, no GPU: every row's recorded span of
the staging frame reaches the caller's colour and t buffers, nothing outside
the spans is touched, whatever the thread count and however the spans are
spread over the rows (the threads split the rows by pixel count)."""
import ctypes as C

import numpy as np
import pytest

NONE = np.iinfo(np.int32).max


def copy_spans(dc, dt, sc, st, span, threads, clear_src=False):
    import rtamd
    L = rtamd.lib()
    L.rtx_copy_spans.argtypes = [C.c_void_p] * 4 + [C.c_int64, C.c_int32, C.c_void_p, C.c_int32, C.c_int32]
    H, W = dc.shape
    rtamd._lib.check(L.rtx_copy_spans(dc.ctypes.data, dt.ctypes.data, sc.ctypes.data, st.ctypes.data, W, H,
                                      span.ctypes.data, threads, int(clear_src)))


def spans_for(kind, H, W, rng):
    span = np.full((H, 2), NONE, np.int32)
    if kind == "empty":
        return span
    if kind == "full":
        span[:, 0], span[:, 1] = 0, -(W - 1)
        return span
    if kind == "middle":  # a centred model: spans only in the middle rows
        rows = np.arange(H // 3, 2 * H // 3)
    elif kind == "one_row":
        rows = np.array([H - 1])
    else:  # random rows
        rows = np.flatnonzero(rng.random(H) < 0.4)
    lo = rng.integers(0, W, len(rows))
    hi = np.minimum(W - 1, lo + rng.integers(0, W, len(rows)))
    span[rows, 0], span[rows, 1] = lo, -hi
    return span


@pytest.mark.parametrize("clear_src", [False, True])
@pytest.mark.parametrize("kind", ["empty", "full", "middle", "one_row", "random"])
@pytest.mark.parametrize("threads", [0, 1, 2, 3, 7, 16])
@pytest.mark.parametrize("H,W", [(1, 5), (61, 203), (1080, 1920)])
def test_copy_spans_matches_rows(kind, threads, H, W, clear_src):
    rng = np.random.default_rng(H * 1000 + W + threads)
    sc = rng.integers(0, 2**32, (H, W), dtype=np.uint32)
    st = rng.random((H, W), dtype=np.float32)
    sc0, st0 = sc.copy(), st.copy()
    dc = np.full((H, W), 0xDEADBEEF, np.uint32)
    dt = np.full((H, W), -1.0, np.float32)
    span = spans_for(kind, H, W, rng)
    copy_spans(dc, dt, sc, st, span, threads, clear_src)
    want_c, want_t = np.full_like(dc, 0xDEADBEEF), np.full_like(dt, -1.0)
    left_c, left_t = sc0.copy(), st0.copy()
    for y in range(H):
        lo, hi = int(span[y, 0]), -int(span[y, 1])
        if lo <= hi:
            want_c[y, lo:hi + 1] = sc0[y, lo:hi + 1]
            want_t[y, lo:hi + 1] = st0[y, lo:hi + 1]
            left_c[y, lo:hi + 1] = 0
            left_t[y, lo:hi + 1] = np.inf
    assert np.array_equal(dc, want_c)
    assert np.array_equal(dt.view(np.uint32), want_t.view(np.uint32))
    if clear_src:
        assert np.array_equal(sc, left_c) and np.array_equal(st.view(np.uint32), left_t.view(np.uint32))
    else:
        assert np.array_equal(sc, sc0) and np.array_equal(st.view(np.uint32), st0.view(np.uint32))
