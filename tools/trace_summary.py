"""Per-kernel totals of a rocprofv3 --kernel-trace CSV (second half of the run =
the timed pass of tools/plan_trace.py): calls, total and mean duration."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 2:]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    k = r["Kernel_Name"].split("(")[0][:60]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
print(f"span {span:.1f} us, kernel busy {busy:.1f} us")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t:10.1f} us {n:6d} calls {t / n:8.2f} us/call  {k}")
