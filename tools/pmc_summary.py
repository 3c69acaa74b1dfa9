"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of the render kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict


def summarise(root, kernel_substr=os.environ.get("PMC_KERNEL", "render_kernel")):
    vals = defaultdict(list)
    durs = []
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_substr not in row["Kernel_Name"]:
                    continue
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
                durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    out = {k: sum(v) / len(v) for k, v in vals.items()}
    out["_dispatches_per_counter"] = max(len(v) for v in vals.values()) if vals else 0
    out["_mean_dur_ns(profiled)"] = sum(durs) / len(durs) if durs else 0
    return out


if __name__ == "__main__":
    for root in sys.argv[1:]:
        s = summarise(root)
        print("==", root)
        for k in sorted(s):
            print(f"  {k:32s} {s[k]:16.1f}")
