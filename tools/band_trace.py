"""Timeline of the render launches in a rocprofv3 kernel trace (dev tool for
the row-band split, tools/ab.py split under rocprofv3 --kernel-trace): the
dispatches fall into runs separated by host pauses (> GAP_US); for each run
print its launches (kernel, grid, queue, start offset, duration) and the run's
span against the summed kernel time, so the GPU's idle share inside a timed
region shows.
usage: python tools/band_trace.py <kernel_trace.csv> [min launches per run] [GAP_US]
"""
import csv
import sys


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main():
    path = sys.argv[1]
    min_n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    gap = float(sys.argv[3]) if len(sys.argv) > 3 else 200.0
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if "rocclr" in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Grid_Size_X", "?"), r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    runs, cur, last_end = [], [], None
    for r in rows:
        if cur and (r[0] - last_end) / 1e3 > gap:
            runs.append(cur)
            cur = []
        last_end = r[1] if not cur else max(last_end, r[1])
        cur.append(r)
    if cur:
        runs.append(cur)
    for i, run in enumerate(runs):
        if len(run) < min_n:
            continue
        t0 = run[0][0]
        span = (max(r[1] for r in run) - t0) / 1e3
        busy = sum(r[1] - r[0] for r in run) / 1e3
        print(f"run {i}: {len(run)} launches, span {span:.1f} us, summed kernel time {busy:.1f} us")
        for s, e, name, grid, q in run:
            print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:8.1f} us  q{q:>3}  grid {grid:>8}  {name}")


if __name__ == "__main__":
    main()
