"""Which projection-head weight-gradient launches stretch in the concurrent step, and beside what
(DESIGN.md §4.4). Reads a rocprofv3 --kernel-trace CSV of `bench.py` (tools/gpu.sh
`prof`), picks the heads' split-K dW launches by their grids (ops._dw_plan: dW2 = 16 tiles of
128 x 128 x 32 splits, dW1 = 6 eight-wave tiles x 40 splits; the 8,192-row text head's dW2 = 16 x 16
splits) and prints, per kind, their durations and the share of that time each co-running
(stream, kernel) overlapped them.

usage: python tools/head_dw_trace.py <kernel_trace.csv>
"""
import collections
import csv
import sys

HEADS = {("4096", "32", "256"): "dW2 visual/audio", ("3072", "40", "512"): "dW1 visual/audio",
         ("4096", "16", "256"): "dW2 text"}


def main(path):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["n"] = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
    agg = collections.defaultdict(list)
    for r in rows:
        kind = HEADS.get((r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"]))
        if kind is None or "gemm" not in r["Kernel_Name"]:
            continue
        share = collections.Counter()
        for o in rows:
            if o is not r and o["s"] < r["e"] and o["e"] > r["s"]:
                share[(o["Stream_Id"], o["n"])] += min(o["e"], r["e"]) - max(o["s"], r["s"])
        agg[kind].append((r["e"] - r["s"], r["Stream_Id"], share))
    for kind, v in sorted(agg.items()):
        durs = sorted(d for d, _, _ in v)
        tot = collections.Counter()
        for _, _, s in v:
            tot.update(s)
        print(f"{kind}: {len(v)} launches on stream(s) {sorted(set(s for _, s, _ in v))}; duration us min "
              f"{durs[0] / 1e3:.1f} median {durs[len(durs) // 2] / 1e3:.1f} max {durs[-1] / 1e3:.1f}")
        for (st, name), t in tot.most_common(5):
            print(f"    overlapped {t / sum(durs):5.2f} of its time by stream {st} {name}")


if __name__ == "__main__":
    main(sys.argv[1])
