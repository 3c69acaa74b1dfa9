"""Per-wave timestamp analysis of one frame (diagnostic kernel variant)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))
import torch  # noqa
import rtamd
from rtamd import workloads as WL

name = sys.argv[1] if len(sys.argv) > 1 else "stanford-bunny.obj"
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
kind, payload, off = WL.load_input(name)
s = WL.make_scene(kind, payload)
s.set_plane(None)
P = WL.params_for(WL.orbit_positions(64)[0], W, H, rtamd.ShadingMode.Normal)
L = rtamd.lib()
L.rtx_wave_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_uint32, C.c_void_p,
                              C.POINTER(C.c_int64)]
nb = ((W + 15) // 16) * ((H + 15) // 16)
buf = np.zeros((nb * 4, 4), np.uint64)
n = C.c_int64(nb * 4)
for rep in range(3):
    rtamd._lib.check(L.rtx_wave_stamps(s._h, C.byref(P), W, H, 1, buf.ctypes.data, C.byref(n)))
st, en = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64)
t0 = st.min()
st, en = (st - t0) * 10.0, (en - t0) * 10.0  # ns (100 MHz)
dur = en - st
print(f"{name} {W}x{H}: waves {len(dur)}, span {en.max()/1e3:.1f} us")
for q in (50, 90, 99, 99.9, 100):
    print(f"  wave duration p{q}: {np.percentile(dur, q)/1e3:8.2f} us")
print(f"  start p50 {np.percentile(st,50)/1e3:.1f} us, last start {st.max()/1e3:.1f} us")
# concurrency over time
tgrid = np.linspace(0, en.max(), 40)
conc = [(np.sum((st <= t) & (en > t))) for t in tgrid]
print("  resident waves over time:", " ".join(str(c) for c in conc))
# time split: waves longer than 10 us
long = dur > 10000
print(f"  waves > 10us: {long.sum()}  ({long.mean()*100:.1f}%), their mean {dur[long].mean()/1e3 if long.any() else 0:.1f} us")
mxu = (buf[:, 2] & 0xFFFFFFFF).astype(np.int64)
smu = (buf[:, 2] >> np.uint64(32)).astype(np.int64)
order = np.argsort(dur)[::-1][:8]
print("  slowest waves: dur_us start_us end_us max_lane_units sum_units ns_per_maxunit")
for i in order:
    print(f"    {dur[i]/1e3:8.1f} {st[i]/1e3:8.1f} {en[i]/1e3:8.1f} {mxu[i]:6d} {smu[i]:8d} {dur[i]/max(mxu[i],1):8.0f}")
# waves ending in the last 30% of the span: when did they start?
late = en > 0.7 * en.max()
print(f"  waves ending in the last 30% of the span: {late.sum()}, start p10/p50/p90 "
      f"{np.percentile(st[late], 10)/1e3:.1f}/{np.percentile(st[late], 50)/1e3:.1f}/"
      f"{np.percentile(st[late], 90)/1e3:.1f} us, duration p50 {np.percentile(dur[late], 50)/1e3:.1f} us")
print(f"  SIMD efficiency (sum / 64*max over waves): {smu.sum() / max(64*mxu.sum(),1):.3f}")
xcc = buf[:, 3] & 0xF
u9 = (buf[:, 3] >> np.uint64(8)).astype(np.int64)
heavy = mxu > 40
print(f"  waves with max units > 40: {heavy.sum()}; their units done with >8 lanes busy (u9/max): "
      f"p10/p50/p90 {np.percentile(u9[heavy]/mxu[heavy],10):.2f}/{np.percentile(u9[heavy]/mxu[heavy],50):.2f}/"
      f"{np.percentile(u9[heavy]/mxu[heavy],90):.2f}")
for i in order:
    print(f"    slow wave: max {mxu[i]} u9 {u9[i]} sum {smu[i]}")
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"  xcc {x}: waves {m.sum()}, busy-sum {dur[m].sum()/1e6:.2f} ms, last end {en[m].max()/1e3:.1f} us")
