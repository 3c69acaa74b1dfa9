"""Where a persistent multi-frame launch spends its time (dev tool).

For each workload and frames-per-launch n, on ONE stream: the event-timed
launch duration (mean of several launches; a + b*n fits the fixed per-launch
cost a and the per-frame cost b) and, from the per-wave stamps of one launch
(rtx_set_persist_stamps): when the first wave found the queue drained, when the
last wave ended (the tail between the two), and the spread of wave starts
(the ramp).
The stamps exist only in a diagnostic build of the library:
  bash tools/build_variant.sh stamps -DRT_PERSIST_STAMPS
  RTAMD_LIB=triangles-sdf-cpu-raytracing_amd/lib/var_stamps.so python tools/persist_tail.py bunny
usage: python tools/persist_tail.py [workload ...]   (keys of bench.WORKLOADS)
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "triangles-sdf-cpu-raytracing_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rtamd  # noqa: E402
from rtamd import workloads as WL  # noqa: E402

L = rtamd.lib()
L.rtx_set_persist_stamps.argtypes = [C.c_void_p, C.c_int64]
CAP = 1 << 16


def where(item, n, W, H, g=2):
    """frame and pixel origin of a queue item of G = 2 tiles (16 x 8 pixels)"""
    tx = -(-W // (8 * g))
    per = tx * -(-H // 8)
    f, r = divmod(int(item), per)
    return f"frame {f} x {(r % tx) * 8 * g} y {(r // tx) * 8}"


def main():
    names = sys.argv[1:] or ["bunny"]
    buf = torch.zeros(CAP * 8, dtype=torch.int64, device="cuda")
    for name in names:
        src, W, H, mode = bench.WORKLOADS[name][:4]
        sc, off = WL.scene_for(src)
        sc.set_plane(None)
        prm = bench.orbit_params(64, W, H)
        fits = []
        for n in (2, 4, 8):
            wall, launches, _ = bench.run_single(sc, prm, 16, 8 * n, W, H, inflight=1, batch=n)
            kms = sum(ms for ms, _ in launches) / len(launches)
            fits.append((n, kms))
            # one more launch with stamps
            buf.zero_()
            rtamd._lib.check(L.rtx_set_persist_stamps(C.c_void_p(buf.data_ptr()), CAP))
            bench.run_single(sc, prm, 0, n, W, H, inflight=1, batch=n)
            rtamd._lib.check(L.rtx_set_persist_stamps(None, 0))
            s = buf.view(-1, 8).cpu().numpy()
            s = s[s[:, 1] > 0]
            t0 = s[:, 0].min()
            st, en = (s[:, 0] - t0) / 100.0, (s[:, 1] - t0) / 100.0  # us (100 MHz)
            last_item = (s[:, 3] - t0) / 100.0
            items = s[:, 2] & 0xFFFFFFFF
            drained = en.min()
            print(f"{name} n={n}: launch {kms:.4f} ms (events), stamps span {en.max():.1f} us, "
                  f"{len(s)} waves, start spread p50/max {np.median(st):.1f}/{st.max():.1f} us, "
                  f"first wave out {drained:.1f} us, wave ends p10/p50/p90 {np.percentile(en, 10):.1f}/"
                  f"{np.median(en):.1f}/{np.percentile(en, 90):.1f} us, tail (last end - first out) "
                  f"{en.max() - drained:.1f} us, items/wave mean {items.mean():.1f} max {items.max()}, "
                  f"exit probe after last item max {(en - last_item).max():.1f} us", flush=True)
            # the waves that end last: their last item (start, duration) and
            # the longest items of the launch
            dur = (s[:, 3] - s[:, 4]) / 100.0
            lstart = (s[:, 4] - t0) / 100.0
            for w in np.argsort(-en)[:4]:
                print(f"    late wave: ends {en[w]:.1f} us, last item {s[w, 5]} ({where(s[w, 5], n, W, H)}) "
                      f"started {lstart[w]:.1f} us, ran {dur[w]:.1f} us", flush=True)
            dmax = s[:, 6] / 100.0
            for w in np.argsort(-dmax)[:4]:
                print(f"    longest item: {s[w, 7]} ({where(s[w, 7], n, W, H)}) {dmax[w]:.1f} us", flush=True)
            print(f"    item duration over waves' longest: p50 {np.median(dmax):.1f} us, p99 "
                  f"{np.percentile(dmax, 99):.1f} us", flush=True)
        a = np.polyfit([n for n, _ in fits], [k for _, k in fits], 1)
        print(f"{name}: launch ms ~= {a[1]:.4f} + {a[0]:.4f} * frames", flush=True)
        sc.close()


if __name__ == "__main__":
    main()
