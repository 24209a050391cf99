"""GPU idle inside plans from a rocprofv3 --kernel-trace CSV: the gap before each
kernel (start minus the previous kernel's end), summed by (previous kernel, next
kernel) pair. Gaps longer than --plan-gap-us (default 1000) are taken as the host
between two plans and left out; so is everything before the first k_plan_init /
k_ext_conn_nn of a plan (context setup).

usage: gap_summary.py TRACE.csv [--min-us 2] [--plan-gap-us 1000] [--top 25]
"""
import argparse
import csv
import collections


def short(name):
    n = name.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n.replace("rp::", "")[:48]


ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--min-us", type=float, default=2.0)
ap.add_argument("--plan-gap-us", type=float, default=1000.0)
ap.add_argument("--top", type=int, default=25)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
pairs = collections.defaultdict(lambda: [0, 0.0])
plans = []   # per plan: [wall, busy, idle]
cur = None
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = short(r["Kernel_Name"])
    if prev is not None:
        gap = (s - prev[1]) / 1e3
        if gap > a.plan_gap_us:
            cur = None
        elif cur is not None:
            cur[2] += max(gap, 0.0)
            if gap >= a.min_us:
                k = (prev[2], name)
                pairs[k][0] += 1
                pairs[k][1] += gap
    if cur is None:
        cur = [s, s, 0.0, 0.0]   # start, end, idle, busy
        plans.append(cur)
    cur[1] = max(cur[1], e)
    cur[3] += (e - s) / 1e3
    prev = (s, e, name)
tot = sum(v[1] for v in pairs.values())
print(f"# segments (plans, split at gaps > {a.plan_gap_us:.0f} us): {len(plans)}")
for p in plans:
    if p[3] > 200:
        print(f"wall {(p[1] - p[0]) / 1e3:9.1f} us  busy {p[3]:9.1f}  idle {p[2]:8.1f}")
print(f"# gaps >= {a.min_us} us inside segments: {sum(v[0] for v in pairs.values())}, {tot:.1f} us")
for k, v in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print(f"{v[1]:9.1f} us {v[0]:5d} x  avg {v[1] / v[0]:7.1f}  {k[0]:48s} -> {k[1]}")
