"""HBM3E bandwidth by access mix on one MI355X: write-only (fill), read-only (sum), copy
(read 1 + write 1) and the 1x1-expansion mix (read 1 + write 4).  Sets the roof for the
output-heavy ResNet-50 kernels: a conv that writes four bytes per byte it reads is bound by the
write rate, not by the 8 TB/s headline.

    python tools/hbm_probe.py [--gb 4]
"""
import argparse
import json

import torch


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    args = ap.parse_args()
    n = int(args.gb * 2**30) // 2
    x = torch.empty(n, dtype=torch.bfloat16, device="cuda").normal_()
    y = torch.empty_like(x)
    small = torch.empty(n // 4, dtype=torch.bfloat16, device="cuda").normal_()
    out = torch.empty(1, dtype=torch.float32, device="cuda")  # out[0]: 0-d view
    rows = []
    t = timeit(lambda: y.fill_(1.0))
    rows.append(("write_only", x.numel() * 2, t))
    t = timeit(lambda: torch.sum(x, 0, dtype=torch.float32, out=out[0]))
    rows.append(("read_only", x.numel() * 2, t))
    t = timeit(lambda: y.copy_(x))
    rows.append(("copy_r1_w1", 2 * x.numel() * 2, t))
    # read 1 / write 4: every element of the small tensor broadcast into four outputs
    t = timeit(lambda: y.view(-1, 4).copy_(small.view(-1, 1).expand(-1, 4)))
    rows.append(("expand_r1_w4", small.numel() * 2 + y.numel() * 2, t))
    for name, nbytes, sec in rows:
        print(json.dumps({"pattern": name, "GB": round(nbytes / 1e9, 2), "us": round(sec * 1e6, 1),
                          "TBps": round(nbytes / sec / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
