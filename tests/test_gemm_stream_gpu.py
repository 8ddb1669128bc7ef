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


@pytest.mark.parametrize("mode", ["plain", "cin", "masked"])
@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(1000, 256, 64), (777, 512, 128), (2048, 1024, 256)])
def test_stream_bn_backward_sums(M, N, K, kind, mode):
    """gemm_stream_bnb: the data gradient (bit-identical to the ping-pong GEMM with the same
    accumulate epilogue) plus the BN-backward sums of the BatchNorm whose output it is the
    gradient of: sum dz and sum dz * (x - mean) * invstd, dz = dx * relu_bit (kind 1: the bit
    mask, kind 2: recomputed from x with the forward scale / shift), vs fp32 sums."""
    n = _native()
    a, b, g = _operands(M, N, K, 11 * K + kind)
    x = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    mean = torch.randn(N, device="cuda", generator=g) * 0.1
    inv = torch.rand(N, device="cuda", generator=g) + 0.5
    sc = torch.rand(N, device="cuda", generator=g) + 0.5
    sh = torch.randn(N, device="cuda", generator=g) * 0.2
    bmask = torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8, generator=g)
    cin = torch.randn(M, N, device="cuda", generator=g).bfloat16() if mode == "cin" else None
    acc = None
    if mode == "masked":
        acc = n._MaskedGrad(torch.randn(M, N, device="cuda", generator=g).bfloat16(),
                            torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8,
                                          generator=g))
    ref8 = _run(8, lambda: n.gemm_nt(a, b, cin=None if cin is None else cin.clone(), acc_from=acc))
    out = cin.clone() if cin is not None else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    G = n._K.gemm_tile_rows(M)
    part = torch.full((n._K.bn_workspace_floats_g(G, N),), float("nan"), device="cuda")
    n._K.gemm_stream_bnb(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, K, K, N,
                         out.data_ptr() if cin is not None else 0,
                         acc.dy.data_ptr() if acc else 0, acc.mask.data_ptr() if acc else 0,
                         x.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                         sc.data_ptr() if kind == 2 else 0, sh.data_ptr() if kind == 2 else 0,
                         bmask.data_ptr() if kind == 1 else 0, kind, part.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(out, ref8)
    slab = part[:G * 2 * N].view(G, 2, N)
    assert not torch.isnan(slab).any()
    d, xf = out.float(), x.float()
    if kind == 1:
        bits = ((bmask.view(-1, 1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1)
        d = d * bits.view(M, N).float()
    elif kind == 2:
        d = d * (xf * sc + sh > 0).float()
    xhat = (xf - mean) * inv
    torch.testing.assert_close(slab[:, 0].sum(0), d.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(slab[:, 1].sum(0), (d * xhat).sum(0), rtol=1e-4, atol=2e-2)


def test_resnet_block_bn_backward_sums_fused_into_streamed_dgrad():
    """A residual+ReLU BatchNorm consumed by an identity-style 1x1 conv (w -> 4w reduction, so
    its data gradient is streamed): the BN backward takes its sums from the dgrad epilogue
    (spy on the entry point) and the gradients match the unfused pass."""
    n = _native()
    torch.manual_seed(3)
    Nb, H, C, Kc = 4, 14, 256, 64
    x = torch.randn(Nb, H, H, C, device="cuda").bfloat16()
    w1 = torch.randn(C, 1, 1, C, device="cuda") / C ** 0.5
    w2 = torch.randn(Kc, 1, 1, C, device="cuda") / C ** 0.5
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda") * 0.1
    r = torch.randn(Nb, H, H, C, device="cuda").bfloat16()
    outs, calls = [], {"n": 0}
    orig, prev = n._K.gemm_stream_bnb, n._FUSE_BN_BWD_STREAM

    def spy(*a):
        calls["n"] += 1
        return orig(*a)
    try:
        for fuse in (True, False):
            n._FUSE_BN_BWD_STREAM = fuse
            n._K.gemm_stream_bnb = spy
            ps = [t.clone().requires_grad_(True) for t in (x.float(), w1, w2, gamma, beta)]
            xi = ps[0].detach().bfloat16().requires_grad_(True)
            y1 = n.conv2d(xi, ps[1], 1, 0, bn_stats=True)
            z = n.batch_norm(y1, ps[3], ps[4], None, None, True, 0.9, 1e-5, relu=True, residual=r)
            y2 = n.conv2d(z, ps[2], 1, 0)
            g = torch.randn(y2.shape, device="cuda", generator=torch.Generator(
                device="cuda").manual_seed(1)).bfloat16()
            y2.backward(g)
            outs.append((xi.grad.float(), ps[1].grad, ps[3].grad, ps[4].grad))
            if fuse:
                assert calls["n"] == 1, "fused BN-backward path did not run"
    finally:
        n._K.gemm_stream_bnb = orig
        n._FUSE_BN_BWD_STREAM = prev
    assert calls["n"] == 1
    for a_, b_ in zip(*outs):
        rel = ((a_ - b_).norm() / b_.norm()).item()
        assert rel < 2e-2, rel


@pytest.mark.parametrize("M,N,K", [(1000, 256, 64), (777, 512, 128), (2048, 1024, 256),
                                   (37, 128, 64)])
def test_stream_pre_bn_relu_bitwise(M, N, K):
    """gemm_stream_pre: relu(x * sc + sh) applied to the A rows in registers == the BN apply
    kernel's output (written back as y) and the GEMM on it, bit for bit; statistics too."""
    n = _native()
    g = torch.Generator(device="cuda").manual_seed(M + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    sc = torch.rand(K, device="cuda", generator=g) + 0.5
    sh = torch.randn(K, device="cuda", generator=g) * 0.3
    y_ref = torch.empty_like(x)
    n._K.bn_apply(x.data_ptr(), 0, y_ref.data_ptr(), sc.data_ptr(), sh.data_ptr(), M, K, 1,
                  torch.cuda.current_stream().cuda_stream, 0)
    G = n._K.gemm_tile_rows(M)
    s_ref = torch.zeros(G, 2, N, device="cuda")
    out_ref = _run(13, lambda: n.gemm_nt(y_ref, b, stats=s_ref))
    y = torch.full_like(x, 7)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    s = torch.zeros(G, 2, N, device="cuda")
    n._K.gemm_stream_pre(x.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, sc.data_ptr(),
                         sh.data_ptr(), y.data_ptr(), s.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    assert torch.equal(out, out_ref)
    assert torch.equal(s, s_ref)
