"""Per-kernel MFMA utilisation from one rocprofv3 --pmc pass with SQ_VALU_MFMA_BUSY_CYCLES,
SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/gpu.sh pmc:<name>:<counters>).

Units (MI355X_MICROARCH.md, per-instruction constants / DVFS): SQ_VALU_MFMA_BUSY_CYCLES counts
cycles summed over the chip (= 32 x N_mfma for v_mfma_f32_32x32x16_bf16); GRBM_GUI_ACTIVE is
summed over the 8 XCDs, so the kernel's cycle count is GRBM_GUI_ACTIVE / 8. MFMA-busy fraction =
MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the share of all SIMD-cycles of the kernel's
lifetime in which a matrix core was busy (the dense bf16 peak is 1.0 of this).

usage: python tools/mfma_summary.py <counter_collection.csv> <out.json> [substring ...]
"""
import csv
import json
import sys
from collections import defaultdict

SIMDS = 256 * 4


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def main(path, out, *subs):
    subs = subs or ("pairsim", "tile_gemm", "projhead", "gemm")
    agg = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[(short(r["Kernel_Name"]), int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for (k, grid), v in sorted(agg.items()):
        if not any(s in k for s in subs) or "SQ_VALU_MFMA_BUSY_CYCLES" not in v:
            continue
        mean = {c: sum(x) / len(x) for c, x in v.items()}
        cyc = mean["GRBM_GUI_ACTIVE"] / 8
        res[f"{k}@grid{grid}"] = {
            "launches": len(v["GRBM_GUI_ACTIVE"]),
            "mfma_busy_cycles": mean["SQ_VALU_MFMA_BUSY_CYCLES"],
            "gui_active_cycles_per_xcd": cyc,
            "mfma_busy_frac": mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc) if cyc else None,
            "sq_busy_cycles": mean.get("SQ_BUSY_CYCLES"),
        }
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{v['mfma_busy_frac']:.3f}  {v['launches']:3d}  {k}")


if __name__ == "__main__":
    main(*sys.argv[1:])
