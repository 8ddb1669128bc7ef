"""Summarise a rocprofv3 kernel-trace CSV: per-kernel total time / count, grouped by name."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
if not files:
    print("no kernel_trace.csv under", root)
    sys.exit(0)
tot = collections.defaultdict(float)
cnt = collections.Counter()
t_min, t_max = None, None
for f in files:
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name") or row.get("KernelName") or "?"
            s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            tot[name] += (e - s) / 1e6
            cnt[name] += 1
            t_min = s if t_min is None else min(t_min, s)
            t_max = e if t_max is None else max(t_max, e)
allk = sum(tot.values())
print(f"kernels: {sum(cnt.values())} dispatches, {allk:.2f} ms total kernel time, span {(t_max - t_min) / 1e6:.2f} ms")
for name, t in sorted(tot.items(), key=lambda kv: -kv[1])[:60]:
    short = name if len(name) < 140 else name[:137] + "..."
    print(f"{t:10.3f} ms {100 * t / allk:5.1f}% {cnt[name]:6d}x  {short}")
