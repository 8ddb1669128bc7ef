"""GPU idle time inside the last dispatches of a rocprofv3 kernel trace: wall span, the union of
kernel intervals (all streams), the idle remainder and the largest idle gaps with the kernels on
either side -- to tell launch / sync gaps from kernel time before reaching for HIP graphs.

    python tools/trace_gaps.py TRACE_DIR [--last 645] [--top 15]
"""
import argparse
import csv
import glob
import os


def short(name):
    for p in ("void (anonymous namespace)::", "(anonymous namespace)::", "void "):
        name = name.replace(p, "")
    return name.split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--last", type=int, default=645, help="dispatches (ResNet-50: ~645 per step)")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[-a.last:]
    if not rows:
        print("no dispatches")
        return
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    busy, gaps = 0, []
    cur_s, cur_e, prev = rows[0][0], rows[0][1], rows[0][2]
    for s, e, name in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, name))
            cur_s, cur_e = s, e
        elif e > cur_e:
            cur_e = e
        if e >= cur_e:
            prev = name
    busy += cur_e - cur_s
    span = t1 - t0
    kern = sum(e - s for s, e, _ in rows)
    print(f"dispatches {len(rows)}  span {span / 1e6:.3f} ms  busy(union) {busy / 1e6:.3f} ms  "
          f"idle {(span - busy) / 1e6:.3f} ms ({100.0 * (span - busy) / span:.2f} %)  "
          f"kernel sum {kern / 1e6:.3f} ms  gaps {len(gaps)}")
    hist = [(1, 0, 0), (5, 0, 0), (20, 0, 0), (100, 0, 0), (10 ** 9, 0, 0)]
    for g, _, _ in gaps:
        for i, (lim, n, tot) in enumerate(hist):
            if g / 1e3 < lim:
                hist[i] = (lim, n + 1, tot + g)
                break
    lo = 0
    for lim, n, tot in hist:
        print(f"  gaps {lo:>4}-{lim if lim < 10 ** 9 else 'inf':>4} us: {n:5d}  total {tot / 1e6:.3f} ms")
        lo = lim
    for g, p, n in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {g / 1e3:9.1f} us after {short(p)}  before {short(n)}")


if __name__ == "__main__":
    main()
