"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reads exactly 1/2 of the bytes of a wide coalesced streaming read (16 B/lane,
global_load and LDS-DMA alike), so fetched bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is
exact for 16-B-per-lane streaming stores: written bytes = 1024 * WRITE_SIZE.
Separate passes per counter (FETCH_SIZE and WRITE_SIZE do not fit one pass).

usage: python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        agg[(short, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return agg


def main(fetch_csv, write_csv, out):
    f = load(fetch_csv, "FETCH_SIZE")
    w = load(write_csv, "WRITE_SIZE")
    res = {}
    for key in sorted(set(f) | set(w)):
        short, grid = key
        if not any(t in short for t in ("pairsim", "tile_gemm", "gemm_kernel", "projhead", "adamw", "patch")):
            continue
        fv, wv = f.get(key, []), w.get(key, [])
        res[f"{short}@grid{grid}"] = {
            "launches": max(len(fv), len(wv)),
            "fetch_bytes_per_launch": 2 * 1024 * sum(fv) / max(1, len(fv)),
            "write_bytes_per_launch": 1024 * sum(wv) / max(1, len(wv)),
        }
        res[f"{short}@grid{grid}"]["hbm_bytes_per_launch"] = (res[f"{short}@grid{grid}"]["fetch_bytes_per_launch"]
                                                              + res[f"{short}@grid{grid}"]["write_bytes_per_launch"])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
