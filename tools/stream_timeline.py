"""Per-stream occupancy of one bench step from a rocprofv3 --kernel-trace CSV.

The step window runs from one pair-forward launch (pairsim_fwd_multi) to the next; for each HIP
stream the share of each time bucket covered by its kernels is printed, plus the GPU's idle time
(no kernel on any stream) and the window length. Experiments only.

usage: python tools/stream_timeline.py <kernel_trace.csv> [bucket_ms=5] [which=-2]
"""
import csv
import sys


def main(path, bucket_ms=5.0, which=-2):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    fw = [r for r in rows if "pairsim_fwd_multi" in r["Kernel_Name"]]
    t0, t1 = fw[which]["s"], fw[which + 1]["s"]
    win = [r for r in rows if t0 <= r["s"] < t1]
    nb = int((t1 - t0) / 1e6 / bucket_ms) + 1
    streams = sorted({r["Stream_Id"] for r in win}, key=int)
    print(f"window {(t1 - t0) / 1e6:.1f} ms, {len(win)} kernels; % of each {bucket_ms:g} ms bucket per stream")
    for s in streams:
        occ = [0.0] * nb
        for r in win:
            if r["Stream_Id"] != s:
                continue
            a, b = r["s"] - t0, min(r["e"], t1) - t0
            while a < b:
                k = int(a / (bucket_ms * 1e6))
                edge = min(b, (k + 1) * bucket_ms * 1e6)
                occ[k] += edge - a
                a = edge
        print(f"s{s:>2} " + " ".join(f"{100 * o / (bucket_ms * 1e6):3.0f}" for o in occ))
    idle, ce = 0, win[0]["e"]
    for r in win[1:]:
        if r["s"] > ce:
            idle += r["s"] - ce
        ce = max(ce, r["e"])
    print(f"idle (no kernel on any stream): {idle / 1e6:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 5.0, int(sys.argv[3]) if len(sys.argv) > 3 else -2)
