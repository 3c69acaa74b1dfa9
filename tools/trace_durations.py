"""Print per-dispatch kernel durations from a rocprofv3 kernel_trace.csv."""
import csv
import sys

for f in sys.argv[1:]:
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row["Kernel_Name"]
            if "rocclr" in name:
                continue
            d = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            short = name.split("(")[0].replace("void (anonymous namespace)::", "")[:60]
            print(f"{d:10.2f} us  grid {row['Grid_Size_X']:>8}  {short}")
