"""Summarise rocprofv3 --pmc CSVs: per-dispatch averages of every counter for the
kernels whose name matches a substring. python tools/pmc_summary.py DIR... --kernel k_validity"""
import argparse
import collections
import csv
import glob
import json
import os


def load(dirs, kernel, grid=None, exclude=None):
    vals = collections.defaultdict(list)
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if kernel not in r["Kernel_Name"] or (exclude and exclude in r["Kernel_Name"]):
                    continue
                if grid is not None and int(r["Grid_Size"]) != int(grid):
                    continue
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                          "SGPR_Count", "Scratch_Size")}
    meta["dispatches"] = max((len(v) for v in vals.values()), default=0)
    tot = {k: sum(v) for k, v in vals.items()}
    return {k: sum(v) / len(v) for k, v in vals.items()}, meta, tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="k_validity")
    ap.add_argument("--exclude", default=None, help="skip kernels whose name contains this")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    v, meta, tot = load(a.dirs, a.kernel, exclude=a.exclude)
    # per-wave figures from the totals over all matching dispatches (dispatches of
    # different sizes weigh by their waves)
    waves = tot.get("SQ_WAVES", 0) or 1
    print(json.dumps(meta))
    print(f"{'counter':28s} {'avg/dispatch':>16s} {'total':>18s}")
    for k in sorted(v):
        extra = f"  per-wave {tot[k] / waves:12.1f}" if k.startswith("SQ_") and k != "SQ_WAVES" else ""
        print(f"{k:28s} {v[k]:16.1f} {tot[k]:18.1f}{extra}")
    if a.json:
        json.dump({"counters": v, "totals": tot, "meta": meta}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
