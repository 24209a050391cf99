"""Summarise rocprofv3 --pmc CSVs: per-dispatch averages of every counter for the
kernels whose name matches a substring. python tools/pmc_summary.py DIR... --kernel k_validity"""
import argparse
import collections
import csv
import glob
import json
import os


def load(dirs, kernel, grid=None, exclude=None):
    """Per-dispatch averages, totals over the matching dispatches, the dispatch
    metadata, and per counter the SQ_WAVES of the passes (files) it was collected in
    (so a per-wave figure divides by the waves of its own pass: SQ_WAVES rides along
    in every pass and must not be summed over them)."""
    vals = collections.defaultdict(list)
    waves_of = collections.defaultdict(float)
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            fv = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                if kernel not in r["Kernel_Name"] or (exclude and exclude in r["Kernel_Name"]):
                    continue
                if grid is not None and int(r["Grid_Size"]) != int(grid):
                    continue
                fv[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                          "SGPR_Count", "Scratch_Size")}
            w = sum(fv.get("SQ_WAVES", []))
            for k, v in fv.items():
                vals[k].extend(v)
                waves_of[k] += w
    meta["dispatches"] = max((len(v) for v in vals.values()), default=0)
    tot = {k: sum(v) for k, v in vals.items()}
    return {k: sum(v) / len(v) for k, v in vals.items()}, meta, tot, waves_of


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="k_validity")
    ap.add_argument("--exclude", default=None, help="skip kernels whose name contains this")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    v, meta, tot, waves_of = load(a.dirs, a.kernel, exclude=a.exclude)
    # the kernel sources + flags these counters were collected on (rp_math.h,
    # rp_model.h, rp_kernels.h: k_validity*, k_edges* live there)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from rbe550_final_project_amd.build import validity_source_hash
    meta["kernel"] = a.kernel
    meta["source_hash"] = validity_source_hash()
    # per-wave figures: a counter's total over the SQ_WAVES of the passes it was
    # collected in (dispatches of different sizes weigh by their waves)
    print(json.dumps(meta))
    print(f"{'counter':28s} {'avg/dispatch':>16s} {'total':>18s}")
    for k in sorted(v):
        extra = (f"  per-wave {tot[k] / (waves_of[k] or 1):12.1f}" if k.startswith("SQ_") and k != "SQ_WAVES"
                 else "")
        print(f"{k:28s} {v[k]:16.1f} {tot[k]:18.1f}{extra}")
    if a.json:
        json.dump({"counters": v, "totals": tot, "meta": meta}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
