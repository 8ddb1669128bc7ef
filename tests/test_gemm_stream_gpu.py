"""The row-streaming GEMM for output-heavy shapes (csrc/kernels/gemm_stream.hip, variant 13)
against the ping-pong GEMM (variant 8) and fp32 references.

Every output element sees the same MFMA sequence as in variant 8 (k = 0..31, 32..63, ... in
order), so C must be BIT-IDENTICAL for the plain, beta = 1 (Cin) and masked residual-gradient
epilogues.  The BatchNorm statistics slab has the same shape as variant 8's ([ceil(M/256)][2][N])
but sums in a different order: compared to fp32 column sums of the bf16 output.  Shapes cover K
64 / 128 / 256, M tails inside a block and inside a wave (rows past M: no stores, no statistics),
a single-block M, and N from one chunk (64) to 32 chunks; plus the ResNet-50 1x1 conv route.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(4096, 256, 64), (1000, 512, 128), (777, 1024, 256), (65536 // 4, 256, 128),
          (300, 64, 64), (256, 2048, 256), (37, 128, 64), (20000, 512, 256)]


def _native():
    from distributedtensorflow_amd.ops import native
    return native


def _run(variant, fn):
    n = _native()
    n._K.gemm_set_variant(variant)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        n._K.gemm_set_variant(-1)


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _operands(M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    return a, b, g


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_stream_matches_pingpong_bitwise(M, N, K):
    n = _native()
    a, b, g = _operands(M, N, K, M + N + K)
    ref8 = _run(8, lambda: n.gemm_nt(a, b))
    out = _run(13, lambda: n.gemm_nt(a, b))
    assert torch.equal(out, ref8)
    exact = a.float() @ b.float().t()
    err = ((out.float() - exact).norm() / exact.norm()).item()
    assert err < 5e-3, err
    # auto dispatch takes the streaming kernel for these shapes when N >= K
    if N >= K:
        assert torch.equal(_run(-1, lambda: n.gemm_nt(a, b)), out)
    cin = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    c8 = _run(8, lambda: n.gemm_nt(a, b, cin=cin.clone()))
    c13 = _run(13, lambda: n.gemm_nt(a, b, cin=cin.clone()))
    assert torch.equal(c13, c8)
    # out-of-place beta = 1 (out != cin) must leave cin untouched
    o13 = torch.empty_like(cin)
    keep = cin.clone()
    _run(13, lambda: n.gemm_nt(a, b, out=o13, cin=cin))
    assert torch.equal(o13, c8) and torch.equal(cin, keep)


@pytest.mark.parametrize("M,N,K", [(4096, 256, 64), (1000, 512, 128), (777, 1024, 256),
                                   (20000, 512, 256), (37, 128, 64)])
def test_stream_masked_accumulate_and_bn_stats(M, N, K):
    n = _native()
    a, b, g = _operands(M, N, K, 7 + K)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    mask = torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8, generator=g)
    acc = n._MaskedGrad(dy, mask)
    m8 = _run(8, lambda: n.gemm_nt(a, b, acc_from=acc))
    m13 = _run(13, lambda: n.gemm_nt(a, b, acc_from=acc))
    assert torch.equal(m13, m8)
    # the masked sum against an fp32 reference of dy * bit
    bits = ((mask.view(-1, 1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1)
    ref = (a.float() @ b.float().t()).bfloat16().float() + dy.float() * bits.view(M, N).float()
    torch.testing.assert_close(m13.float(), ref, rtol=2e-2, atol=2e-2)
    tiles = n._K.gemm_tile_rows(M)
    s13 = torch.full((tiles, 2, N), float("nan"), device="cuda")
    y13 = _run(13, lambda: n.gemm_nt(a, b, stats=s13))
    y8 = _run(8, lambda: n.gemm_nt(a, b))
    assert torch.equal(y13, y8)
    assert not torch.isnan(s13).any(), "every slab row / column is written"
    yf = y13.float()
    torch.testing.assert_close(s13[:, 0].sum(0), yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s13[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-4, atol=1e-1)
    # per-slab-row sums match the 256-row blocks
    for t in (0, tiles - 1):
        blk = yf[t * 256:(t + 1) * 256]
        torch.testing.assert_close(s13[t, 0], blk.sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("C,K", [(64, 256), (128, 512), (256, 1024)])
def test_resnet_output_heavy_1x1_conv_route(C, K):
    """conv2d with fused BN statistics on an expanding 1x1 conv takes the streaming route and
    matches the fp32 conv; its data gradient (w -> 4w) too."""
    n = _native()
    torch.manual_seed(C)
    x = torch.randn(3, 14, 14, C, device="cuda").bfloat16().requires_grad_(True)
    w = (torch.randn(K, 1, 1, C, device="cuda") / C ** 0.5).requires_grad_(True)
    assert n._gemm_1x1(C, K, 1, 1, 1, (0, 0))
    y = n.conv2d(x, w, 1, 0, bn_stats=True)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(y.float(), ref.permute(0, 2, 3, 1), rtol=2e-2, atol=2e-2)
    part, G, M, Kc = y._dtf_bn_part
    assert (G, M, Kc) == (n._K.gemm_tile_rows(3 * 14 * 14), 3 * 14 * 14, K)
    stats = part[:G * 2 * K].view(G, 2, K)
    torch.testing.assert_close(stats[:, 0].sum(0), y.float().reshape(-1, K).sum(0),
                               rtol=1e-4, atol=1e-2)
    dy = torch.randn_like(y)
    y.backward(dy)
    dref = torch.nn.functional.conv_transpose2d(dy.float().permute(0, 3, 1, 2),
                                                w.detach().float().permute(0, 3, 1, 2))
    torch.testing.assert_close(x.grad.float(), dref.permute(0, 2, 3, 1), rtol=3e-2, atol=3e-2)
