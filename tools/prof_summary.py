"""Per-phase launch durations of the bench's headline kernel from a rocprofv3
kernel trace (the check that bench.py's event-timed kernel_ms agrees with the
profiler).

bench.py issues, on the headline kernel (render_persist_kernel<MeshS, 4,
false> for the bunny): the warm-up launches over the stream pool (max(--warmup,
2 x 8) frames: 2 launches at the defaults), the timed two-stream launches, then
for roofline.one_stream the same warm-up frames on one stream (2 launches) and
the timed one-stream launches. Dispatches are taken in Dispatch_Id order.
usage: python tools/prof_summary.py <kernel_trace.csv> <timed launches> [kernel substring]
                                     [two-stream warm-up launches] [one-stream warm-up launches] [timed frames]
(the driver's command, --steps 20 --warmup 5: 2 timed launches of 10 frames, warm-ups 2 and 1)
With the timed frame count, the one-stream launches' summed duration per frame
is printed too (bench.py's roofline.one_stream.kernel_ms_per_frame).
"""
import csv
import sys


def main():
    f, n = sys.argv[1], int(sys.argv[2])
    key = sys.argv[3] if len(sys.argv) > 3 else "render_persist_kernel<(anonymous namespace)::MeshS, 4, false>"
    rows = [r for r in csv.DictReader(open(f)) if key in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    warm2 = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    warm1 = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    two = d[warm2:warm2 + n]
    one = d[warm2 + n + warm1:warm2 + n + warm1 + n]
    print(f"{len(d)} dispatches of {key}")
    print(f"two-stream timed launches: {len(two)}, mean {sum(two) / len(two):.5f} ms")
    if one:
        print(f"one-stream timed launches: {len(one)}, mean {sum(one) / len(one):.5f} ms")
        if len(sys.argv) > 6:
            print(f"one-stream kernel time per frame: {sum(one) / int(sys.argv[6]):.5f} ms")


if __name__ == "__main__":
    main()
