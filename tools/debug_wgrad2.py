"""wgrad geometry sweep (fp64 CPU oracle) + forward-conv determinism check."""
import sys
import torch
sys.path.insert(0, ".")
from distributedtensorflow_amd.ops import native, reference  # noqa: E402
K_ = native.kernels()

def wg(N, H, C, K, R, stride, pad, tr=1):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    wr = torch.randn(K, R, R, C, dtype=torch.float64).requires_grad_(True)
    y = reference.conv2d(x.double().cpu(), wr, stride, pad)
    g = torch.randn(y.shape, device="cuda").to(torch.bfloat16)
    y.backward(g.double().cpu())
    _, P, Q, _ = y.shape
    taps = [(r - pad, s - pad) for r in range(R) for s in range(R)]
    tc = R * R * C
    dW = torch.zeros(K, tc, device="cuda")
    K_.conv_wgrad(x.data_ptr(), g.data_ptr(), dW.data_ptr(), 0, [N, H, H, C, P, Q, stride, stride, K, tc],
                  [t[0] for t in taps], [t[1] for t in taps], 1, torch.cuda.current_stream().cuda_stream, tr)
    torch.cuda.synchronize()
    ref = wr.grad.reshape(K, -1)
    d = dW.double().cpu()
    rel = ((d - ref).norm() / ref.norm()).item()
    err = (d - ref).abs().reshape(K, R * R, C).amax(dim=(0, 2))
    print(f"wgrad N{N} H{H} C{C} K{K} R{R} s{stride} p{pad}: rel={rel:.3g}  per-tap max err={[round(v,3) for v in err.tolist()]}", flush=True)

for case in [(1, 8, 64, 64, 3, 1, 1), (1, 8, 64, 64, 1, 2, 0), (1, 8, 64, 64, 3, 2, 1),
             (2, 28, 128, 128, 3, 2, 1), (1, 16, 64, 64, 3, 1, 1), (2, 14, 256, 256, 1, 1, 0)]:
    wg(*case)

# forward determinism
torch.manual_seed(1)
x = torch.randn(8, 56, 56, 64, device="cuda").to(torch.bfloat16)
w = torch.randn(64, 3, 3, 64, device="cuda").to(torch.bfloat16)
outs = [native.conv2d_forward(x, w, 1, 1) for _ in range(6)]
print("fwd repeat max diff:", max((o.float() - outs[0].float()).abs().max().item() for o in outs), flush=True)
dy = torch.randn_like(outs[0])
dxs = [native.conv2d_dgrad(dy, w, x.shape, 1, 1) for _ in range(6)]
print("dgrad repeat max diff:", max((o.float() - dxs[0].float()).abs().max().item() for o in dxs), flush=True)
