"""The persistent register-epilogue GEMM (csrc/kernels/gemm.hip gemm_pp_kernel, variant 11) and
the two-blocks-per-CU 256 x 128 kernel (gemm_nt_kernel OCC 2, variant 12) against the round-2
ping-pong kernel (variant 8) and an fp32 reference.

Variant 12 runs 32-deep K-steps instead of 64-deep ones, but every accumulator still sees the
same MFMA sequence (k = 0..31, 32..63, ... in order) and the same two-wave-row statistics
combine, so it is held to the same bit-identity (and is run with its start stagger on).

The new kernel runs the same main loop with the MFMA operands swapped (each lane then holds four
consecutive output columns) and stores straight from the accumulators, with the LDS-DMA stream
continuing across the tiles a persistent block walks.  Per output element the products and
their accumulation order are unchanged, so C must be BIT-IDENTICAL to variant 8 for every
epilogue mode (bias, ReLU, beta = 1 accumulate, masked residual accumulate); the BatchNorm
partial sums (a different summation order) must agree to fp32 rounding.  Shapes cover edge
tiles in M and N, a K tail, K = 128 (two steps: every look-ahead piece belongs to the next
tile) and more tiles than CUs (several tiles per block).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(4096, 768, 768), (1000, 520, 200), (65536 // 4, 2304, 768), (777, 264, 128),
          (300, 256, 3072), (2048, 1024, 136), (256 * 300, 512, 512)]


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


@pytest.mark.parametrize("variant", [11, 12])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_pp_matches_pingpong_bitwise(M, N, K, variant):
    n = _native()
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    ref8 = _run(8, lambda: n.gemm_nt(a, b))
    out = _run(variant, lambda: n.gemm_nt(a, b))
    assert torch.equal(out, ref8)
    exact = a.float() @ b.float().t()
    err = ((out.float() - exact).norm() / exact.norm()).item()
    assert err < 5e-3, err
    r8 = _run(8, lambda: n.gemm_nt(a, b, bias=bias, relu=True))
    r11 = _run(variant, lambda: n.gemm_nt(a, b, bias=bias, relu=True))
    assert torch.equal(r11, r8)
    cin = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    c8 = _run(8, lambda: n.gemm_nt(a, b, cin=cin.clone()))
    c11 = _run(variant, lambda: n.gemm_nt(a, b, cin=cin.clone()))
    assert torch.equal(c11, c8)
    # bias + ReLU + accumulate (the persistent kernel's compile-time ReLU on the accumulate form)
    cr8 = _run(8, lambda: n.gemm_nt(a, b, bias=bias, relu=True, cin=cin.clone()))
    cr = _run(variant, lambda: n.gemm_nt(a, b, bias=bias, relu=True, cin=cin.clone()))
    assert torch.equal(cr, cr8)


@pytest.mark.parametrize("variant", [11, 12])
@pytest.mark.parametrize("M,N,K", [(4096, 768, 768), (1000, 520, 200), (256 * 300, 512, 512)])
def test_pp_masked_accumulate_and_bn_stats(M, N, K, variant):
    n = _native()
    g = torch.Generator(device="cuda").manual_seed(7)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    mask = torch.randint(0, 256, (M * N // 8,), device="cuda", dtype=torch.uint8, generator=g)
    acc = n._MaskedGrad(dy, mask)
    m8 = _run(8, lambda: n.gemm_nt(a, b, acc_from=acc))
    m11 = _run(variant, lambda: n.gemm_nt(a, b, acc_from=acc))
    assert torch.equal(m11, m8)
    tiles = n._K.gemm_tile_rows(M)
    s8 = torch.zeros(tiles, 2, N, device="cuda")
    s11 = torch.zeros(tiles, 2, N, device="cuda")
    y8 = _run(8, lambda: n.gemm_nt(a, b, stats=s8))
    y11 = _run(variant, lambda: n.gemm_nt(a, b, stats=s11))
    assert torch.equal(y11, y8)
    torch.testing.assert_close(s11, s8, rtol=1e-5, atol=1e-3)
    yf = y8.float()
    torch.testing.assert_close(s11[:, 0].sum(0), yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s11[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-4, atol=1e-1)


PP2_SHAPES = [s for s in SHAPES if s[2] % 64 == 0 and s[2] >= 128] + [(65536, 768, 3072)]


@pytest.mark.parametrize("M,N,K", PP2_SHAPES)
def test_pp2_matches_pingpong_bitwise(M, N, K):
    """Round 5's persistent kernel (variant 15: whole-operand descriptors, per-tile piece offsets
    computed once for the current and the next tile) -- the same MFMA sequence per output element
    as variant 8, so bit-identical for every epilogue mode, and the BN partial sums to rounding."""
    test_pp_matches_pingpong_bitwise(M, N, K, 15)
    if K in (768, 512):
        test_pp_masked_accumulate_and_bn_stats(M, N, K, 15)


def test_pp2_refuses_unsupported_shapes():
    n = _native()
    a = torch.zeros(512, 200, device="cuda").bfloat16()
    b = torch.zeros(256, 200, device="cuda").bfloat16()
    with pytest.raises(RuntimeError, match="variant 15"):
        _run(15, lambda: n.gemm_nt(a, b))


@pytest.mark.parametrize("n,hw,c,k,stride", [(8, 14, 256, 256, 1), (4, 28, 128, 256, 1),
                                             (8, 14, 256, 512, 2)])
def test_pp2_conv_matches_pingpong_bitwise(n, hw, c, k, stride):
    """The implicit-GEMM conv on the persistent kernel (gemm_set_pp2 bit 1): forward output (the
    interleaved register-direct epilogue), with BN statistics (the swapped-operand epilogue) and
    the data gradient (stride 2: strided phase outputs) all equal to the ping-pong kernel's."""
    n_ = _native()
    g = torch.Generator(device="cuda").manual_seed(n * hw + c + k)
    x = torch.randn(n, hw, hw, c, device="cuda", generator=g).bfloat16()
    w = (torch.randn(k, 3, 3, c, device="cuda", generator=g) / (9 * c) ** 0.5).bfloat16()
    out = {}
    prev = n_._K.gemm_get_pp2()
    for pp2 in (0, 2):
        n_._K.gemm_set_pp2(pp2)
        try:
            y = n_.conv2d_forward(x, w, stride, 1)
            P = y.shape[1]
            st = torch.zeros(n * P * P // 64 + 1, 2, k, device="cuda")    # >= any slab count
            ys = n_.conv2d_forward(x, w, stride, 1, stats=st)
            dy = torch.randn(y.shape, device="cuda", generator=torch.Generator(
                device="cuda").manual_seed(3)).bfloat16()
            dx = n_.conv2d_dgrad(dy, w, x.shape, stride, 1)
            torch.cuda.synchronize()
            out[pp2] = (y, ys, st, dx)
        finally:
            n_._K.gemm_set_pp2(prev)
    (y0, ys0, st0, dx0), (y2, ys2, st2, dx2) = out[0], out[2]
    assert torch.equal(y2, y0) and torch.equal(ys2, ys0) and torch.equal(dx2, dx0)
    torch.testing.assert_close(st2.sum(0), st0.sum(0), rtol=1e-4, atol=1e-1)


@pytest.mark.parametrize("M,N,K", [(65536 // 8, 3072, 768), (1000, 520, 256)])
def test_pp2_bias_gelu_epilogue_matches_pingpong(M, N, K):
    """BERT's FFN1 (z = x W^T + b, h = gelu(z)) on the persistent kernel's interleaved epilogue
    (two stores per row): z and h bit-identical to the LDS-staged ping-pong kernel."""
    n = _native()
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    out = {}
    prev = n._K.gemm_get_pp2()
    for pp2 in (0, 1):
        n._K.gemm_set_pp2(pp2)
        try:
            z = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            h = torch.empty_like(z)
            n._K.gemm_nt_bias_gelu(a.data_ptr(), b.data_ptr(), z.data_ptr(), h.data_ptr(), M, N,
                                   K, K, K, bias.data_ptr(), n._st())
            torch.cuda.synchronize()
            out[pp2] = (z, h)
        finally:
            n._K.gemm_set_pp2(prev)
    assert torch.equal(out[1][0], out[0][0]) and torch.equal(out[1][1], out[0][1])
    zf = (a.float() @ b.float().t() + bias)
    assert ((out[1][0].float() - zf).norm() / zf.norm()).item() < 5e-3


@pytest.mark.parametrize("M,N,K", [(65536 // 8, 768, 3072), (1000, 520, 256)])
def test_pp2_gelu_backward_epilogue_matches_pingpong(M, N, K):
    """BERT's FFN1 data gradient d(a) = (do W2) * gelu'(a + b) with the per-tile column sums on
    the persistent kernel: d(a) bit-identical to the LDS-staged kernel, colsum to fp32 rounding
    (summation order) and against an fp32 reference."""
    n = _native()
    g = torch.Generator(device="cuda").manual_seed(M + K)
    do = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    wt = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    a = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    tiles = n._K.gemm_tile_rows(M)
    out = {}
    prev = n._K.gemm_get_pp2()
    for pp2 in (0, 1):
        n._K.gemm_set_pp2(pp2)
        try:
            da = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            cs = torch.empty(tiles, N, device="cuda")
            n._K.gemm_nt_gelu_bwd(do.data_ptr(), wt.data_ptr(), da.data_ptr(), M, N, K, K, K,
                                  a.data_ptr(), b.data_ptr(), cs.data_ptr(), n._st())
            torch.cuda.synchronize()
            out[pp2] = (da, cs)
        finally:
            n._K.gemm_set_pp2(prev)
    assert torch.equal(out[1][0], out[0][0])
    torch.testing.assert_close(out[1][1], out[0][1], rtol=1e-4, atol=1e-2)
    col = out[1][0].float().sum(0)
    torch.testing.assert_close(out[1][1].sum(0), col, rtol=2e-2, atol=1.0)


@pytest.mark.parametrize("stages,strips", [(0x44, 0), (0x33, 0), (0x44, 3), (0x33, 3)])
def test_halo_conv_filter_ring_depth_bit_identical(stages, strips):
    """The 3x3 halo convs (stage-0/1 shapes) with a 3- or 4-deep filter-slice ring, with and
    without two strips per block: forward (+ BN statistics) and data gradient bit-identical to
    the double-buffered kernel (same MFMA order per output)."""
    n_ = _native()
    out = {}
    for cfg in ((0, 0), (stages, strips)):
        n_._K.conv_set_halo_stages(cfg[0])
        n_._K.conv_set_halo_strips(cfg[1])
        try:
            res = []
            for (hw, c) in ((56, 64), (28, 128)):
                g = torch.Generator(device="cuda").manual_seed(hw + c)
                x = torch.randn(3, hw, hw, c, device="cuda", generator=g).bfloat16()
                w = (torch.randn(c, 3, 3, c, device="cuda", generator=g) / (9 * c) ** 0.5).bfloat16()
                y = n_.conv2d_forward(x, w, 1, 1)
                st = torch.zeros(3 * hw * hw // 16 + 1, 2, c, device="cuda")
                ys = n_.conv2d_forward(x, w, 1, 1, stats=st)
                dx = n_.conv2d_dgrad(y, w, x.shape, 1, 1)
                torch.cuda.synchronize()
                res += [y, ys, st, dx]
            out[cfg] = res
        finally:
            n_._K.conv_set_halo_stages(0)
            n_._K.conv_set_halo_strips(0)
    a, b = out[(0, 0)], out[(stages, strips)]
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), i


def test_pp2_masked_accumulate_mask_ends_at_the_allocation():
    """The masked-residual epilogue must not read past the bit mask: M = 16 rows (one partial
    tile) with the mask carved from the END of a larger buffer whose next bytes are another
    tensor's -- rows past M read nothing (a 1-byte over-read faulted on unmapped memory)."""
    n = _native()
    M, N, K = 16, 2048, 512
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    big = torch.randint(0, 256, (M * N // 8 + 64,), device="cuda", dtype=torch.uint8, generator=g)
    mask = big[: M * N // 8]
    guard = big[M * N // 8:].clone()
    acc = n._MaskedGrad(dy, mask)
    r8 = _run(8, lambda: n.gemm_nt(a, b, acc_from=acc))
    r15 = _run(15, lambda: n.gemm_nt(a, b, acc_from=acc))
    assert torch.equal(r15, r8)
    assert torch.equal(big[M * N // 8:], guard)
