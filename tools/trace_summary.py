"""Steady-state kernel summary from a rocprofv3 --kernel-trace CSV of bench.py.

bench.py (TRIAD_PROFILE_MARK=1) launches one l2norm_rows_kernel right before its timed region
(a kernel the training step never uses); every kernel that starts after it belongs to the K
timed steps. Writes per-kernel ms/step, calls/step and the total, so MIOpen's one-time
algorithm search in the warmup does not drown the profile.

Also writes <out>_by_grid.csv: every launch of the whole trace for the §8 head kernels
(pairsim / tile_gemm) grouped by (kernel, grid size) -- the AV and TV forward launches share a
kernel name, so this is where the AV launch's own average duration is read (bench.py's
roofline.avg_ms names the same launch).

usage: python tools/trace_summary.py <kernel_trace.csv> <steps> <out.csv>
"""
import csv
import sys
from collections import defaultdict


def main(path, steps, out):
    steps = int(steps)
    rows = list(csv.DictReader(open(path)))
    name_k = "Kernel_Name"
    s_k, e_k = "Start_Timestamp", "End_Timestamp"
    rows.sort(key=lambda r: int(r[s_k]))
    marks = [i for i, r in enumerate(rows) if "l2norm_rows_kernel" in r[name_k]]
    if not marks:
        raise SystemExit("no marker kernel in trace")
    t0 = int(rows[marks[-1]][e_k])
    agg = defaultdict(lambda: [0, 0.0])
    t_first, t_last = None, 0
    for r in rows[marks[-1] + 1:]:
        s, e = int(r[s_k]), int(r[e_k])
        if s < t0:
            continue
        t_first = s if t_first is None else t_first
        t_last = max(t_last, e)
        a = agg[r[name_k]]
        a[0] += 1
        a[1] += (e - s) / 1e6
    total = sum(v[1] for v in agg.values())
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls_per_step", "ms_per_step", "avg_us", "pct"])
        for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k[:200], n / steps, round(ms / steps, 4), round(1e3 * ms / n, 2), round(100 * ms / total, 2)])
        w.writerow(["TOTAL_KERNEL_TIME", "", round(total / steps, 3), "", 100])
        w.writerow(["WALL_FIRST_TO_LAST", "", round((t_last - t_first) / 1e6 / steps, 3), "", ""])
    print(f"kernel time {total / steps:.2f} ms/step over {steps} steps; wall {(t_last - t_first) / 1e6 / steps:.2f} ms/step"
          " (kernels on the modality / side streams overlap, so the sum can exceed the wall)")
    cols = [c for c in ("Grid_Size", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z") if c in rows[0]]
    if cols:
        by = defaultdict(list)
        for r in rows:
            if "pairsim" in r[name_k] or "tile_gemm" in r[name_k]:
                by[(r[name_k][:120], "x".join(r[c] for c in cols))].append((int(r[e_k]) - int(r[s_k])) / 1e6)
        with open(out.replace(".csv", "_by_grid.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "grid_size", "launches", "avg_ms", "min_ms", "max_ms"])
            for (k, g), d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([k, g, len(d), round(sum(d) / len(d), 4), round(min(d), 4), round(max(d), 4)])


if __name__ == "__main__":
    main(*sys.argv[1:4])
