"""Summarise rocprofv3 --pmc CSVs per kernel instantiation: per-dispatch averages
of every counter, totals, per-wave figures and the instantiation's own dispatch
metadata (VGPRs, scratch, LDS), for every kernel whose name contains a substring.

    python tools/pmc_summary.py DIR... --kernel k_edges [--exclude packed]
                                [--json out.json] [--split PREFIX]

Rows are grouped by the FULL kernel name (round 6: the round-5 version pooled every
name containing the substring and printed the first dispatch's metadata, so a
k_edges summary blended three instantiations under the resources of one).
--split PREFIX writes one PREFIX_<instantiation>.txt / .json per instantiation."""
import argparse
import collections
import csv
import glob
import json
import os
import re


def load(dirs, kernel, grid=None, exclude=None):
    """{full kernel name: (per-dispatch averages, metadata, totals, waves per counter)}.
    Per counter, the SQ_WAVES of the passes (files) it was collected in, so a per-wave
    figure divides by the waves of its own pass (SQ_WAVES rides along in every pass and
    must not be summed over them)."""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    waves_of = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            fv = collections.defaultdict(lambda: collections.defaultdict(list))
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if kernel not in name or (exclude and exclude in name):
                    continue
                if grid is not None and int(r["Grid_Size"]) != int(grid):
                    continue
                fv[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta.setdefault(name, {k: r[k] for k in ("Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                                         "SGPR_Count", "Scratch_Size")})
            for name, cv in fv.items():
                w = sum(cv.get("SQ_WAVES", []))
                for k, v in cv.items():
                    vals[name][k].extend(v)
                    waves_of[name][k] += w
    out = {}
    for name, cv in vals.items():
        m = dict(meta[name])
        m["dispatches"] = max((len(v) for v in cv.values()), default=0)
        m["kernel_name"] = name
        out[name] = ({k: sum(v) / len(v) for k, v in cv.items()}, m, {k: sum(v) for k, v in cv.items()},
                     dict(waves_of[name]))
    return out


def short(name):
    """file-name form of an instantiation: k_edges<-1, true, false>(...) -> k_edges_m1_true_false"""
    s = re.sub(r"\(.*", "", name).replace("void ", "").replace("rp::", "")
    s = s.replace("-", "m").replace("<", "_").replace(">", "")
    return re.sub(r"[^A-Za-z0-9_]+", "_", s).strip("_")


def render(v, meta, tot, waves_of):
    lines = [json.dumps(meta), f"{'counter':28s} {'avg/dispatch':>16s} {'total':>18s}"]
    for k in sorted(v):
        extra = (f"  per-wave {tot[k] / (waves_of.get(k) or 1):12.1f}" if k.startswith("SQ_") and k != "SQ_WAVES"
                 else "")
        lines.append(f"{k:28s} {v[k]:16.1f} {tot[k]:18.1f}{extra}")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="k_validity")
    ap.add_argument("--exclude", default=None, help="skip kernels whose name contains this")
    ap.add_argument("--json", default=None)
    ap.add_argument("--split", default=None, help="one PREFIX_<instantiation>.txt/.json per instantiation")
    a = ap.parse_args()
    res = load(a.dirs, a.kernel, exclude=a.exclude)
    # the kernel sources + flags these counters were collected on (rp_math.h,
    # rp_model.h, rp_kernels.h: k_validity*, k_edges* live there)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from rbe550_final_project_amd.build import validity_source_hash
    src = validity_source_hash()
    allj = {}
    for name in sorted(res, key=lambda n: -res[n][1]["dispatches"]):
        v, meta, tot, waves_of = res[name]
        meta["kernel"] = a.kernel
        meta["source_hash"] = src
        text = render(v, meta, tot, waves_of)
        print(text + "\n")
        allj[name] = {"counters": v, "totals": tot, "meta": meta}
        if a.split:
            base = f"{a.split}_{short(name)}"
            open(base + ".txt", "w").write(text + "\n")
            json.dump(allj[name], open(base + ".json", "w"), indent=1)
    if a.json:
        json.dump(allj, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
