"""Convolutions on tensors past 2 GiB (the 32-bit buffer-offset cap).

The conv / dgrad / wgrad kernels rebase their buffer descriptors at each tile's (or split's)
first image with 64-bit pointer math, so only the in-tile offset is 32-bit.  Each case runs a
reduced-spatial layer whose input (and for some its output) is > 2^31 bytes; only a handful of
images -- the first, the ones straddling the 2 GiB byte boundary and the last -- carry data, the
rest are zero, so the fp32 reference only has to run on that small sub-batch: forward rows,
data-gradient rows and the whole weight gradient (zero images contribute nothing) must match it.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"

CASES = [
    # (N, H, W, C, K, R, stride, pad)   -- X bytes
    (5400, 56, 56, 64, 64, 3, 1, 1),      # 2.17 GB in and out: halo 3x3 kernel, dgrad, wgrad
    (5600, 28, 28, 256, 64, 1, 1, 0),     # 2.25 GB in: implicit-GEMM 1x1 (DMA / register)
    (1500, 28, 28, 1024, 256, 1, 2, 0),   # 2.41 GB in: strided projection (sub-pixel dgrad)
    (1400, 28, 28, 1024, 256, 1, 1, 0),   # 2.25 GB in: 1x1 routed to the hand GEMM
    (2700, 28, 28, 128, 128, 3, 2, 1),    # 0.54 GB in, dgrad out; stride-2 3x3 wgrad split span
]


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    yield
    torch.cuda.empty_cache()


@pytest.mark.parametrize("case", CASES)
def test_conv_past_2gib(case):
    from distributedtensorflow_amd.ops import native as nat
    from distributedtensorflow_amd.ops import reference as ref
    N, H, W, C, K, R, stride, pad = case
    img_bytes = H * W * C * 2
    edge = (2 ** 31) // img_bytes                       # the image straddling byte 2^31
    live = sorted({0, 1, min(edge, N - 3), min(edge + 1, N - 2), N - 2, N - 1})
    idx = torch.tensor(live, device=dev)
    torch.manual_seed(0)
    x = torch.zeros(N, H, W, C, device=dev, dtype=torch.bfloat16)
    xs = torch.randn(len(live), H, W, C, device=dev).to(torch.bfloat16)
    x[idx] = xs
    w = torch.randn(K, R, R, C, device=dev) / (R * R * C) ** 0.5

    xn = x.requires_grad_(True)
    wn = w.clone().requires_grad_(True)
    y = nat.conv2d(xn, wn, stride, pad)
    P, Q = y.shape[1], y.shape[2]
    g = torch.zeros(N, P, Q, K, device=dev, dtype=torch.bfloat16)
    gs = torch.randn(len(live), P, Q, K, device=dev).to(torch.bfloat16)
    g[idx] = gs
    y.backward(g)

    xr = xs.float().requires_grad_(True)
    wr = w.to(torch.bfloat16).float().requires_grad_(True)
    yr = ref.conv2d(xr, wr, stride, pad)
    yr.backward(gs.float())
    assert _rel(y.detach()[idx], yr) < 1e-2, _rel(y.detach()[idx], yr)
    assert _rel(xn.grad[idx], xr.grad) < 2e-2, _rel(xn.grad[idx], xr.grad)
    assert _rel(wn.grad, wr.grad) < 2e-2, _rel(wn.grad, wr.grad)
    # zero images stay zero (no tile read another tile's rows through a wrong base)
    mid = (live[1] + live[2]) // 2
    if mid not in live:
        assert not y.detach()[mid].any() and not xn.grad[mid].any()
