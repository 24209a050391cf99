"""Average duration of one kernel's dispatches in a rocprofv3 kernel trace, over
all of them and over the last K (the timed region of a bench.py run whose first W
launches are warm-up): the figure to set beside bench.py's HIP-event kernel_ms.

    python tools/trace_avg.py KERNEL_TRACE.csv KERNEL_SUBSTRING [K]
"""
import csv
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if name in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    d = [x[1] for x in rows]
    last = d[-k:]
    print(f"{name}: {len(d)} dispatches, avg {sum(d) / len(d) / 1e3:.2f} us (min {min(d) / 1e3:.2f}, "
          f"max {max(d) / 1e3:.2f}); last {len(last)}: avg {sum(last) / len(last) / 1e3:.2f} us "
          f"(min {min(last) / 1e3:.2f}, max {max(last) / 1e3:.2f})")
    print("per dispatch (us): " + " ".join(f"{x / 1e3:.1f}" for x in d))


if __name__ == "__main__":
    main()
