"""Timeline of the last K kernels of a rocprofv3 --kernel-trace CSV: start offset,
duration and the gap before each (where a plan query's time goes)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = rows[-k:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = t0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:7.2f}  gap {(s - prev_end) / 1e3:7.2f}  "
          f"{r['Kernel_Name'].split('(')[0][:70]}")
    prev_end = e
