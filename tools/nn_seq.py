"""Nearest-node launches of C5 plans in dispatch order (diagnostic): reads a rocprofv3
kernel trace of tools/c5_profile.py (or any plan run) and prints, per k_nn_mfma
dispatch, its grid (blocks), duration and the kernels around it, then a histogram of
where the matrix-core time goes by duration class.

    python tools/nn_seq.py gpurun_out/nnseq/kt_kernel_trace.csv [--all] [--log stderr_with_nnlog_lines]

With RBE_NN_LOG set, the library prints one "nnlog n= T= grid= S= status=" line per
k_nn_mfma launch (host order = dispatch order on the one plan stream); --log pairs
them with the dispatches: per launch (query, node) pairs and pairs/s (status-bounded
searches: n is the largest count, the actual one is on the device)."""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tot = defaultdict(float)
    nn = []

    def short(r):
        n = r["Kernel_Name"]
        for k in ("k_nn_mfma", "k_nn_image", "k_nn_reduce_g"):   # (mangled template names)
            if k in n:
                return k
        return n.split("(")[0].split("<")[0].replace("void ", "").replace("rp::", "")

    for i, r in enumerate(rows):
        sh = short(r)
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[sh] += us
        if sh == "k_nn_mfma":
            blocks = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            nxt = next((short(x) for x in rows[i + 1:i + 4] if not short(x).startswith("k_nn_reduce")), "?")
            nn.append((blocks, us, nxt))
    logs = []
    if "--log" in sys.argv:
        for line in open(sys.argv[sys.argv.index("--log") + 1]):
            if line.startswith("nnlog "):
                logs.append(dict(kv.split("=") for kv in line.split()[1:]))
        if len(logs) != len(nn):
            print(f"(log has {len(logs)} launches, trace {len(nn)}: not paired)")
            logs = []
    if "--all" in sys.argv:
        for k, (b, us, nxt) in enumerate(nn):
            extra = ""
            if logs:
                n, T = int(logs[k]["n"]), int(logs[k]["T"])
                extra = f"  n {n:7d} T {T:7d} S {logs[k]['S']:>3s}" + (" pilot" if "pilot" in logs[k] else "      ")
                if logs[k]["status"] == "0":
                    extra += f"  {n * T / (us * 1e-6) / 1e12:6.2f} e12 pairs/s"
            print(f"{k:4d} blocks {b:6d} {us:9.1f} us  then {nxt}{extra}")
    by = defaultdict(lambda: [0, 0.0])
    for b, us, nxt in nn:
        by[nxt][0] += 1
        by[nxt][1] += us
    print("k_nn_mfma by the kernel that consumes it:", {k: (v[0], round(v[1], 1)) for k, v in by.items()})
    print("kernel time (us) by name:")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
        print(f"  {k:32s} {v:10.1f}")
    edges = [0, 20, 50, 100, 200, 500, 1000, 2000, 5000, 1e9]
    print("k_nn_mfma launches by duration:")
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = [us for b, us, _ in nn if lo <= us < hi]
        if sel:
            print(f"  [{lo:6.0f}, {hi:6.0f}) us: {len(sel):4d} launches, {sum(sel):9.1f} us")
    print(f"  total {len(nn)} launches, {sum(us for b, us, _ in nn):.1f} us")


if __name__ == "__main__":
    main()
