"""Per-dispatch summary of rocprofv3 --pmc counter CSVs for the render kernels
(dev tool): one line per dispatch with its scene type and every counter of the
pass, and, when both passes are given, where wave time goes (SQ_WAIT_ANY,
SQ_WAIT_INST_ANY and SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES) and the SALU,
branch and memory instructions per VALU instruction.
usage: python tools/issue_mix.py <pass dir> [<pass dir> ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(root):
    per = defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                if "render_" not in k:
                    continue
                m = re.search(r"(MeshS|OctS|GridS)", k)
                key = (int(row["Dispatch_Id"]), m.group(1) if m else k[:40])
                per[key][row["Counter_Name"].replace("SQ_", "")] = \
                    per[key].get(row["Counter_Name"].replace("SQ_", ""), 0.0) + float(row["Counter_Value"])
    return per


def main():
    merged = defaultdict(dict)
    for root in sys.argv[1:]:
        per = load(root)
        print(os.path.basename(root.rstrip("/")))
        for key in sorted(per):
            print(f"  {key} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(per[key].items())))
        # the passes are separate runs: match dispatches by order within each scene type
        seen = defaultdict(int)
        for key in sorted(per):
            merged[(key[1], seen[key[1]])].update(per[key])
            seen[key[1]] += 1
    print("where wave time goes (fractions of SQ_WAVE_CYCLES) and instructions per VALU instruction")
    for (scene, i), c in sorted(merged.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        wc = c.get("WAVE_CYCLES")
        if not wc or "WAIT_ANY" not in c or "INSTS_VALU" not in c:
            continue
        v = c["INSTS_VALU"]
        print(f"  {scene} #{i}: active {c['ACTIVE_INST_ANY'] / wc:.2f}, waiting on memory {c['WAIT_ANY'] / wc:.2f}, "
              f"issue-stalled {c['WAIT_INST_ANY'] / wc:.2f}; SALU {c['INSTS_SALU'] / v:.3f}, branch "
              f"{c['INSTS_BRANCH'] / v:.3f}, VMEM rd {c['INSTS_VMEM_RD'] / v:.3f}, LDS {c['INSTS_LDS'] / v:.3f} per VALU")


if __name__ == "__main__":
    main()
