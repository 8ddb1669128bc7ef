"""Average rocprofv3 counter_collection.csv values per (kernel, grid) -> text table."""
import collections
import csv
import glob
import os
import sys


def main(d):
    rows = []
    for f in glob.glob(os.path.join(d, "*counter_collection*.csv")):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    if not rows:
        print("no counter rows")
        return
    keyname = "Kernel_Name" if "Kernel_Name" in rows[0] else "Kernel-Name"
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = (r[keyname][:160], r.get("Grid_Size", r.get("Grid-Size", "")))
        agg[k][r.get("Counter_Name", r.get("Counter-Name"))].append(
            float(r.get("Counter_Value", r.get("Counter-Value", 0))))
    for (name, grid), counters in agg.items():
        vals = {c: sum(v) / len(v) for c, v in counters.items()}
        wc = vals.get("SQ_WAVE_CYCLES", 0) or 1
        line = [f"{name} grid={grid}"]
        for c in sorted(vals):
            line.append(f"  {c}={vals[c]:.4g}")
        if "SQ_WAIT_ANY" in vals:
            line.append(f"  wait_any/wave={vals['SQ_WAIT_ANY'] / wc:.2f} "
                        f"wait_inst/wave={vals.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
                        f"active/wave={vals.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}")
        if "SQ_ACTIVE_INST_VALU" in vals:
            line.append(f"  valu_active/wave={vals['SQ_ACTIVE_INST_VALU'] / wc:.3f} "
                        f"lds_active/wave={vals.get('SQ_ACTIVE_INST_LDS', 0) / wc:.3f} "
                        f"valu_insts/mfma={vals.get('SQ_INSTS_VALU', 0) / max(vals.get('SQ_INSTS_MFMA', 0), 1):.1f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "SQ_BUSY_CYCLES" in vals:
            line.append(f"  mfma_busy/busy={vals['SQ_VALU_MFMA_BUSY_CYCLES'] / max(vals['SQ_BUSY_CYCLES'], 1):.3f}")
        print("\n".join(line))


if __name__ == "__main__":
    main(sys.argv[1])
