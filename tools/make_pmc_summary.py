"""Write profiles/pmc_validity.json (HBM bytes per validity launch) from the
rocprofv3 --pmc passes FETCH_SIZE and WRITE_SIZE (separate passes).

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports 1/2 of the
bytes of a wide coalesced streaming read (128-B requests tallied at 64 B); the
validity kernel's state loads form one contiguous 36 B/lane stream, so read bytes
= 2 x FETCH_SIZE x 1024. WRITE_SIZE is exact for streaming stores: x 1024.
usage: python tools/make_pmc_summary.py FETCH_DIR WRITE_DIR STATES_PER_LAUNCH OUT.json"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
sys.path.insert(0, __file__.rsplit("/", 2)[0])
from pmc_summary import load  # noqa: E402
from rbe550_final_project_amd.build import validity_source_hash  # noqa: E402


def main():
    fdir, wdir, n, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    def one(d):   # the bench's headline instantiation (grid = the states per launch: one kernel)
        res = load([d], "k_validity", n)
        assert len(res) == 1, f"{len(res)} k_validity instantiations at grid {n}: {list(res)}"
        return next(iter(res.values()))
    f, meta, _, _ = one(fdir)
    w, _, _, _ = one(wdir)
    read_b = 2.0 * f["FETCH_SIZE"] * 1024.0
    write_b = w["WRITE_SIZE"] * 1024.0
    d = {"kernel": "k_validity", "states_per_launch": n, "fetch_size_kb": f["FETCH_SIZE"],
         "write_size_kb": w["WRITE_SIZE"], "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
         "hbm_bytes_per_launch": read_b + write_b, "algorithmic_bytes_per_launch": 37 * n,
         "correction": "read = 2 x FETCH_SIZE (gfx950 half-count of wide streaming reads), write = WRITE_SIZE",
         "dispatch_meta": meta, "source_hash": validity_source_hash()}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
