"""Ordered per-dispatch list (kernel name, duration) from a rocprofv3 kernel-trace directory: the
last --last dispatches, for mapping kernels to layers.

    python tools/trace_dump.py TRACE_DIR [--last 1500] [--min-us 20]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--last", type=int, default=1500)
    ap.add_argument("--min-us", type=float, default=20.0)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Grid_Size_X", r.get("Grid_Size", "")),
                             r.get("Workgroup_Size_X", r.get("Workgroup_Size", ""))))
    rows.sort()
    for s, e, name, grid, wg in rows[-a.last:]:
        us = (e - s) / 1e3
        if us >= a.min_us:
            print(f"{us:9.1f}  grid={grid:>8} wg={wg:>4}  {name[:150]}")


if __name__ == "__main__":
    main()
