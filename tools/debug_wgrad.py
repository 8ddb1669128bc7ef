"""Debug: conv weight-gradient kernel variants vs a fp32 PyTorch reference."""
import sys

import torch

sys.path.insert(0, ".")
from distributedtensorflow_amd.ops import native, reference  # noqa: E402

K_ = native.kernels()


def run(N, H, W, C, K, R, stride, pad, tr, splits):
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
    w = torch.randn(K, R, R, C, device="cuda")
    xr = x.double().cpu()
    wr = w.to(torch.bfloat16).double().cpu().requires_grad_(True)
    y = reference.conv2d(xr, wr, stride, pad)
    g = torch.randn(y.shape, device="cuda").to(torch.bfloat16)
    y.backward(g.double().cpu())
    # also MIOpen's fp32 answer, to compare the library against the fp64 oracle
    wm = w.to(torch.bfloat16).float().requires_grad_(True)
    ym = reference.conv2d(x.float(), wm, stride, pad)
    ym.backward(g.float())
    mi = wm.grad.reshape(K, -1).double().cpu()
    _, P, Q, _ = y.shape
    pt = pad
    taps = [(r - pt, s - pt) for r in range(R) for s in range(R)]
    dW = torch.zeros(K, R * R * C, device="cuda")
    geom = [N, H, W, C, P, Q, stride, stride, K, R * R * C]
    if splits == 0:
        splits = K_.conv_wgrad_splits(N * P * Q, K, R * R * C, 32 << 20)
    ws = torch.empty(splits * K * R * R * C, device="cuda")
    reps = []
    for rep in range(4):
        dW.zero_()
        K_.conv_wgrad(x.data_ptr(), g.contiguous().data_ptr(), dW.data_ptr(), ws.data_ptr(),
                      geom, [t[0] for t in taps], [t[1] for t in taps], splits,
                      torch.cuda.current_stream().cuda_stream, tr)
        torch.cuda.synchronize()
        r = dW.double().cpu().reshape(K, -1)
        reps.append(((r - wr.grad.reshape(K, -1)).norm() / wr.grad.norm()).item())
    print("   rep rel errors:", ["%.3g" % v for v in reps])
    torch.cuda.synchronize()
    ref = wr.grad.reshape(K, -1)
    dW = dW.double().cpu()
    err = (dW - ref).abs()
    rel = ((dW - ref).norm() / ref.norm()).item()
    print(f"   MIOpen fp32 vs fp64 oracle rel={((mi - ref).norm() / ref.norm()).item():.4g}")
    if R == 1 and stride == 1:
        direct = g.double().reshape(-1, K).T.cpu() @ x.double().reshape(-1, C).cpu()
        print(f"   direct g^T x vs oracle rel={((direct - ref).norm() / ref.norm()).item():.4g}; "
              f"mine vs direct rel={((dW - direct).norm() / direct.norm()).item():.4g}")
    bad = (err > 1e-2 * ref.abs().max()).nonzero()
    print(f"case N{N} H{H} C{C} K{K} R{R} s{stride} tr={tr} splits={splits}: rel={rel:.4g} "
          f"bad={bad.shape[0]}/{ref.numel()}", flush=True)
    if bad.shape[0]:
        rows = torch.unique(bad[:, 0])[:20].tolist()
        cols = torch.unique(bad[:, 1])[:20].tolist()
        print("   bad rows", rows, "\n   bad cols", cols, flush=True)


if __name__ == "__main__":
    for tr in (1, 3, 5, 0, 2, 4):
        for splits in (1,):
            run(1, 8, 8, 64, 64, 1, 1, 0, tr, splits)      # M = 64 = one K-step
            run(1, 16, 16, 64, 64, 1, 1, 0, tr, splits)    # 4 K-steps
            run(2, 56, 56, 64, 64, 1, 1, 0, tr, splits)
            run(2, 28, 28, 128, 128, 3, 2, 1, tr, splits)
