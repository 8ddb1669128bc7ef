"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op.

Shapes cover the reference's MNIST CNN and ResNet-50's distinct conv
geometries (N-K1..N-K5) at reduced batch.  Inputs are asymmetric random data (never symmetric
operands: a transposed MFMA C-write would pass a symmetric test — guide §3).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def _native():
    from distributedtensorflow_amd.ops import native
    return native


def _ref():
    from distributedtensorflow_amd.ops import reference
    return reference


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CONV_CASES = [
    # (N, H, W, C, K, R, stride, pad)
    (2, 28, 28, 1, 32, 5, 1, "same"),      # MNIST conv1 (generic gather path)
    (2, 14, 14, 32, 64, 5, 1, "same"),     # MNIST conv2 (BK=32)
    (2, 56, 56, 64, 64, 1, 1, 0),          # bottleneck 1x1
    (2, 56, 56, 64, 64, 3, 1, 1),          # bottleneck 3x3
    (2, 56, 56, 64, 256, 1, 1, 0),         # expand 1x1
    (2, 56, 56, 128, 128, 3, 2, 1),        # strided 3x3 (stage transition)
    (2, 56, 56, 256, 512, 1, 2, 0),        # projection 1x1 stride 2
    (2, 14, 14, 1024, 256, 1, 1, 0),
    (2, 7, 7, 512, 512, 3, 1, 1),
    (2, 224, 224, 3, 64, 7, 2, 3),         # stem 7x7/2 (generic)
    (3, 9, 11, 64, 72, 3, 2, 1),           # odd sizes, Kout not a multiple of 64
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case):
    N, H, W, C, K, R, stride, pad = case
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=dev) / (R * R * C) ** 0.5)
    nat = _native()
    ref = _ref()
    xr = x.float().requires_grad_(True)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = ref.conv2d(xr, wr, stride, pad)
    g = torch.randn_like(yr)
    yr.backward(g)

    xn = x.clone().requires_grad_(True)         # C % 8 != 0: channels zero-padded to 8
    wn = w.clone().requires_grad_(True)
    yn = nat.conv2d(xn, wn, stride, pad)
    assert yn.shape == yr.shape
    assert _rel(yn, yr) < 1e-2, _rel(yn, yr)
    yn.backward(g.to(torch.bfloat16))
    assert _rel(xn.grad, xr.grad) < 2e-2, _rel(xn.grad, xr.grad)
    assert _rel(wn.grad, wr.grad) < 2e-2, _rel(wn.grad, wr.grad)


DMA_CASES = [
    # shapes legal for the 8-wave LDS-DMA conv kernel (C % 64 == 0, Kout % 128 == 0) in fwd
    # and/or dgrad; forced on with conv_set_dma_mode(1) and compared BIT-exactly with the
    # register-staged kernel (same MFMA accumulation order per output element)
    (2, 56, 56, 64, 256, 1, 1, 0),
    (2, 56, 56, 128, 128, 3, 2, 1),
    (2, 56, 56, 256, 512, 1, 2, 0),
    (2, 14, 14, 1024, 256, 1, 1, 0),
    (2, 7, 7, 512, 512, 3, 1, 1),
    (3, 9, 11, 128, 384, 3, 1, 1),     # M not a multiple of 256, three N tiles, padding taps
]


@pytest.mark.parametrize("case", DMA_CASES)
def test_conv_dma_kernel_bit_identical(case):
    N, H, W, C, K, R, stride, pad = case
    nat = _native()
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=dev) / (R * R * C) ** 0.5)
    g = None
    outs = []
    try:
        for mode in (0, 1):
            nat._K.conv_set_dma_mode(mode)
            xn = x.clone().requires_grad_(True)
            wn = w.clone().requires_grad_(True)
            yn = nat.conv2d(xn, wn, stride, pad)
            if g is None:
                g = torch.randn(yn.shape, device=dev).to(torch.bfloat16)
            yn.backward(g)
            outs.append((yn.detach(), xn.grad, wn.grad))
    finally:
        nat._K.conv_set_dma_mode(-1)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    ref = _ref()
    xr = x.float().requires_grad_(True)
    yr = ref.conv2d(xr, w.detach().to(torch.bfloat16).float(), stride, pad)
    assert _rel(outs[1][0], yr) < 1e-2


WGRAD_DMA_CASES = [
    (2, 56, 56, 64, 64, 3, 1, 1),      # Kout 64 (half tile), 9 taps
    (2, 28, 28, 128, 128, 3, 2, 1),    # stride 2, padding taps
    (2, 14, 14, 1024, 256, 1, 1, 0),
    (3, 9, 11, 128, 384, 3, 1, 1),     # M not a multiple of 64, TC not a multiple of 128
    (2, 30, 30, 16, 64, 4, 1, 0),      # the space-to-depth stem shape (C 16, 16 taps)
    (2, 17, 19, 8, 72, 7, 2, 3),       # C 8, 49 taps, Kout 72
]


@pytest.mark.parametrize("case", WGRAD_DMA_CASES)
def test_wgrad_dma_kernel_bit_identical(case):
    """LDS-DMA wgrad kernel == the register-staged one (same fragment order -> same bits), and
    both match the fp32 reference."""
    N, H, W, C, K, R, stride, pad = case
    nat, ref = _native(), _ref()
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - R) // stride + 1
    dy = torch.randn(N, P, Q, K, device=dev).to(torch.bfloat16)
    outs = []
    pipe0 = nat._K.wgrad_get_pipe()
    try:
        for mode in (0, 1, 2):     # register-staged, LDS-DMA (narrow for Kout <= 64), DMA 2x2
            nat._K.wgrad_set_dma_mode(mode)
            outs.append(nat.conv2d_wgrad(x, dy, (K, R, R, C), stride, pad))
        nat._K.wgrad_set_dma_mode(-1)
        for pipe in (1, 2, 3):    # LDS-DMA ring variants (32/4, 64/3, 32/2 + half epilogue)
            nat._K.wgrad_set_pipe(pipe)
            outs.append(nat.conv2d_wgrad(x, dy, (K, R, R, C), stride, pad))
    finally:
        nat._K.wgrad_set_dma_mode(-1)
        nat._K.wgrad_set_pipe(pipe0)
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    wr = torch.zeros(K, R, R, C, device=dev, requires_grad=True)
    ref.conv2d(x.float(), wr, stride, pad).backward(dy.float())
    assert _rel(outs[1], wr.grad) < 1e-2


@pytest.mark.parametrize("case", [(2, 28, 28, 1, 32, 5, 1, "same"), (2, 64, 64, 3, 64, 7, 2, 3)])
def test_conv_element_gather_paths(case):
    """The per-element gather kernels (fwd GATHER=1, wgrad GENERIC) on unpadded C=1 / C=3."""
    N, H, W, C, K, R, stride, pad = case
    torch.manual_seed(1)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=dev) / (R * R * C) ** 0.5).to(torch.bfloat16)
    nat, ref = _native(), _ref()
    y = nat.conv2d_forward(x, w, stride, pad)
    yr = ref.conv2d(x.float(), w.float(), stride, pad)
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(yr)
    dw = nat.conv2d_wgrad(x, dy.to(torch.bfloat16), w.shape, stride, pad)
    wr = w.float().requires_grad_(True)
    ref.conv2d(x.float(), wr, stride, pad).backward(dy.to(torch.bfloat16).float())
    assert _rel(dw, wr.grad) < 2e-2


@pytest.mark.parametrize("C,relu,res,shape", [
    (64, True, False, (4, 7, 9)), (256, True, True, (4, 7, 9)), (512, False, False, (4, 7, 9)),
    (2048, True, True, (4, 7, 9)), (32, True, False, (4, 7, 9)),
    # many rows / ragged unroll tails / a channel count that does not divide the block
    (64, True, True, (3, 37, 41)), (96, True, True, (2, 13, 17)), (128, True, False, (5, 29, 31))])
def test_batch_norm(C, relu, res, shape):
    torch.manual_seed(1)
    x = (torch.randn(*shape, C, device=dev) * 2 + 0.5).to(torch.bfloat16)
    r = torch.randn_like(x) if res else None
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    rm1, rv1 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm1.clone(), rv1.clone()
    nat, ref = _native(), _ref()
    xr = x.float().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    yr = ref.batch_norm(xr, gr, br, rm1, rv1, True, 0.9, 1e-5, relu, rr)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    xn = x.clone().requires_grad_(True)
    gn, bn = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    rn = r.clone().requires_grad_(True) if res else None
    yn = nat.batch_norm(xn, gn, bn, rm2, rv2, True, 0.9, 1e-5, relu, rn)
    assert _rel(yn, yr) < 1e-2
    assert torch.allclose(rm1, rm2, atol=1e-4, rtol=1e-4)
    assert torch.allclose(rv1, rv2, atol=1e-3, rtol=1e-3)
    yn.backward(dy.to(torch.bfloat16))
    assert _rel(xn.grad, xr.grad) < 2e-2
    assert _rel(gn.grad, gr.grad) < 1e-2
    assert _rel(bn.grad, br.grad) < 1e-2
    if res:
        assert _rel(rn.grad, rr.grad) < 1e-2


@pytest.mark.parametrize("shape,k,s,p", [((2, 112, 112, 64), 3, 2, 1), ((4, 28, 28, 32), 2, 2, 0),
                                         ((2, 14, 14, 64), 2, 2, 0)])
def test_max_pool(shape, k, s, p):
    torch.manual_seed(2)
    x = torch.randn(*shape, device=dev).to(torch.bfloat16)
    nat, ref = _native(), _ref()
    xr = x.float().requires_grad_(True)
    yr = ref.max_pool2d(xr, k, s, p)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    xn = x.clone().requires_grad_(True)
    yn = nat.max_pool2d(xn, k, s, p)
    assert torch.equal(yn.float(), yr.detach())
    yn.backward(dy.to(torch.bfloat16))
    assert _rel(xn.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("shape", [(2, 112, 112, 64), (3, 15, 13, 16), (1, 7, 8, 8)])
def test_max_pool_3s2_blocked_backward_bit_identical(shape):
    """2x2-blocked 3x3/2/pad-1 pool backward == the generic per-pixel gather, bit for bit
    (ties included: integer-valued inputs make many windows share their maximum)."""
    torch.manual_seed(4)
    nat = _native()
    x = torch.randint(-3, 4, shape, device=dev).to(torch.bfloat16)
    grads = []
    for blocked in (1, 0):
        nat._K.pool_set_blocked(blocked)
        try:
            xn = x.clone().requires_grad_(True)
            y = nat.max_pool2d(xn, 3, 2, 1)
            torch.manual_seed(5)
            y.backward(torch.randn_like(y))
            grads.append(xn.grad.clone())
        finally:
            nat._K.pool_set_blocked(1)
    assert torch.equal(grads[0], grads[1])
    assert grads[0].abs().sum() > 0


def test_global_avg_pool():
    x = torch.randn(8, 7, 7, 2048, device=dev).to(torch.bfloat16)
    nat, ref = _native(), _ref()
    xr = x.float().requires_grad_(True)
    yr = ref.global_avg_pool(xr)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    xn = x.clone().requires_grad_(True)
    yn = nat.global_avg_pool(xn)
    assert _rel(yn, yr) < 1e-2
    yn.backward(dy.to(torch.bfloat16))
    assert _rel(xn.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("B,V", [(128, 10), (256, 1000), (7, 30522)])
def test_softmax_xent(B, V):
    logits = torch.randn(B, V, device=dev) * 3
    labels = torch.randint(0, V, (B,), device=dev)
    nat, ref = _native(), _ref()
    lr = logits.clone().requires_grad_(True)
    l1 = ref.sparse_softmax_cross_entropy(lr, labels)
    l1.backward()
    ln = logits.clone().requires_grad_(True)
    l2 = nat.sparse_softmax_cross_entropy(ln, labels)
    l2.backward()
    assert abs(l1.item() - l2.item()) < 1e-4 * max(1, abs(l1.item()))
    assert _rel(ln.grad, lr.grad) < 1e-5


@pytest.mark.parametrize("T,o,i", [(128, 1024, 3136), (16384, 768, 768), (8192, 3072, 768)])
@pytest.mark.parametrize("direct", [False, True])
def test_dense_fp32_weight_grads(T, o, i, direct):
    """ops.dense backward: dW (split-K batched hipBLASLt, fp32) and db vs an fp32 reference; with
    ``direct`` the gradients land in pre-existing fp32 .grad buffers flagged as flat."""
    nat = _native()
    torch.manual_seed(0)
    x = torch.randn(T, i, device=dev).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(o, i, device=dev) / i ** 0.5).requires_grad_(True)
    b = torch.randn(o, device=dev).requires_grad_(True)
    if direct:
        w.grad = torch.full_like(w, 0.5)
        b.grad = torch.full_like(b, 0.25)
        w._dtf_flat = b._dtf_flat = True
    y = nat.dense(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float()
    wr = w.detach().to(torch.bfloat16).float()
    yr = xr @ wr.t() + b.detach().to(torch.bfloat16).float()
    gf = g.float()
    assert _rel(y, yr) < 1e-2
    off_w, off_b = (0.5, 0.25) if direct else (0.0, 0.0)
    assert _rel(w.grad - off_w, gf.t() @ xr) < 1e-3
    assert _rel(b.grad - off_b, gf.sum(0)) < 1e-3
    assert _rel(x.grad, gf @ wr) < 1e-2


@pytest.mark.parametrize("T,N", [(16384, 2304), (100, 1024), (7, 8), (65536, 768),
                                 (65536, 3072), (1000, 776), (10240, 30522), (33, 6), (5, 30)])
def test_bf16_col_sum(T, N):
    nat = _native()
    x = torch.randn(T, N, device=dev).to(torch.bfloat16)
    out = torch.full((N,), 2.0, device=dev)
    ws = torch.empty(nat._K.bf16_col_sum_ws_floats(N), device=dev)
    nat._K.bf16_col_sum(x.data_ptr(), T, N, ws.data_ptr(), out.data_ptr(), 1,
                        torch.cuda.current_stream().cuda_stream)
    torch.testing.assert_close(out, x.float().sum(0) + 2.0, atol=1e-3 * max(1, T // 8192),
                               rtol=1e-4)


@pytest.mark.parametrize("rows", [1, 0])
@pytest.mark.parametrize("n,h,w,c", [(2, 224, 224, 3), (3, 33, 31, 3), (1, 20, 18, 1),
                                     (2, 24, 16, 2), (1, 19, 8, 3)])
def test_space_to_depth_input_kernel(n, h, w, c, rows):
    """One-pass HIP space-to-depth of the stem input == the torch pad + permute rewrite, in the
    row-staged form (inputs whose rows are whole 16-B chunks: 224 x 3, 16 x 2, 8 x 3) and the
    per-pixel form (every shape)."""
    from distributedtensorflow_amd.ops import reference as ref
    nat = _native()
    x = torch.randn(n, h, w, c, device=dev).to(torch.bfloat16)
    wt = torch.randn(64, 7, 7, c, device=dev)
    xs_ref, _ = ref.space_to_depth_operands(x, wt, 2, 3)
    nat._K.s2d_set_rows(rows)
    try:
        xs = nat.space_to_depth_input(x, 2, 3, 7, 7)
    finally:
        nat._K.s2d_set_rows(1)
    assert xs.shape == xs_ref.shape
    assert torch.equal(xs, xs_ref)


def test_batched_filter_transpose():
    """filter_transpose_kernel: [K,T,C] -> [C,T,K] for a batch of ragged filters (> 48 jobs ->
    two launches), exactly equal to torch's permute."""
    nat = _native()
    torch.manual_seed(0)
    shapes = [(64, 9, 64), (72, 1, 40), (256, 9, 128), (8, 49, 8), (2048, 1, 512)] * 11
    ws = [torch.randn(k, t, c, device=dev).to(torch.bfloat16) for k, t, c in shapes]
    outs = [torch.empty(c, t, k, device=dev, dtype=torch.bfloat16) for k, t, c in shapes]
    nat._K.filter_transpose([w.data_ptr() for w in ws], [o.data_ptr() for o in outs],
                            [s[0] for s in shapes], [s[1] for s in shapes], [s[2] for s in shapes],
                            torch.cuda.current_stream().cuda_stream)
    for w, o in zip(ws, outs):
        assert torch.equal(o, w.permute(2, 1, 0))


@pytest.mark.parametrize("N,H,C,K", [(2, 56, 64, 64), (3, 56, 64, 128), (2, 28, 128, 128),
                                     (2, 28, 128, 256), (3, 28, 128, 128)])
def test_halo_conv3x3_matches_implicit_gemm(N, H, C, K):
    """Halo-tiled 3x3 kernels (56x56x64 and 28x28x128 families) == the implicit-GEMM kernel bit
    for bit (same tap / k order) for the forward and the data gradient, with one and with two
    row strips per block (N=3 at 28x28: an odd strip count, the last block's second strip is
    dead) and with the filter streamed through registers (FREG); fused BN statistics match."""
    nat = _native()
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, 3, 3, C, device=dev) / (3 * C ** 0.5)).to(torch.bfloat16)
    wd = w[:C].contiguous()                     # dgrad operand: Kout = C, so the halo path applies
    dy = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    outs = []
    try:
        for halo, strips, freg in ((3, 0, 0), (3, 0, 3), (3, 3, 0), (0, 0, 0)):
            nat._K.conv_set_halo(halo)
            nat._K.conv_set_halo_strips(strips)
            nat._K.conv_set_halo_freg(freg)
            y = nat.conv2d_forward(x, w, 1, 1)
            dx = nat.conv2d_dgrad(dy, wd, x.shape, 1, 1)
            gamma = torch.ones(K, device=dev)
            beta = torch.zeros(K, device=dev)
            ys = nat.conv2d(x, w.float(), 1, 1, bn_stats=True)
            z = nat.batch_norm(ys, gamma, beta, None, None, True, 0.9, 1e-5, relu=True)
            outs.append((y, dx, z.float()))
    finally:
        nat._K.conv_set_halo(3)
        nat._K.conv_set_halo_strips(0)
        nat._K.conv_set_halo_freg(0)
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0])
        assert torch.equal(outs[0][1], o[1])
    assert torch.equal(outs[0][2], outs[1][2])      # same strips -> same BN statistics slab rows
    assert torch.equal(outs[0][2], outs[2][2])
    torch.testing.assert_close(outs[0][2], outs[3][2], atol=2e-2, rtol=1e-2)
    ref = _ref()
    yr = ref.conv2d(x.float(), w.float(), 1, 1)
    assert _rel(outs[0][0], yr) < 1e-2


_WGRAD_DEEP_DEFAULT = 0     # csrc/kernels/conv_wgrad.hip g_wgrad_deep

WGRAD_PP_CASES = [
    (2, 14, 14, 256, 256, 3, 1, 1),      # stage-3 3x3
    (2, 7, 7, 512, 512, 3, 1, 1),        # stage-4 3x3
    (3, 9, 11, 128, 384, 3, 1, 1),       # partial Kout / T*C tiles, M not a multiple of 64
    (2, 28, 28, 256, 256, 3, 2, 1),      # stride 2, padding taps
    (4, 14, 14, 1024, 256, 1, 1, 0),     # late 1x1
    (4096, 1, 1, 768, 3072, 1, 1, 0),    # a dense layer's dW (tokens as pixels)
]


@pytest.mark.parametrize("case", WGRAD_PP_CASES)
def test_wgrad_pingpong_kernel(case):
    """The 256 x 256 ping-pong wgrad kernel (Kout, T*C >= 256) against the fp32 reference and
    the 128 x 128 LDS-DMA kernel it replaces for these shapes."""
    N, H, W, C, K, R, stride, pad = case
    nat, ref = _native(), _ref()
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - R) // stride + 1
    dy = torch.randn(N, P, Q, K, device=dev).to(torch.bfloat16)
    try:
        nat._K.wgrad_set_pp(1)
        pp = nat.conv2d_wgrad(x, dy, (K, R, R, C), stride, pad)
        nat._K.wgrad_set_pp(0)
        old = nat.conv2d_wgrad(x, dy, (K, R, R, C), stride, pad)
    finally:
        nat._K.wgrad_set_pp(1)
    wr = torch.zeros(K, R, R, C, device=dev, requires_grad=True)
    ref.conv2d(x.float(), wr, stride, pad).backward(dy.float())
    assert _rel(pp, wr.grad) < 1e-3, _rel(pp, wr.grad)
    assert _rel(pp, old) < 1e-4, _rel(pp, old)
    # the per-row (direct) pixel decode and the shuffled one fetch the same rows
    try:
        nat._K.wgrad_set_direct(1)
        direct = nat.conv2d_wgrad(x, dy, (K, R, R, C), stride, pad)
        nat._K.wgrad_set_direct(2)        # the decode moved to the DMA rows by v_readlane
        readl = nat.conv2d_wgrad(x, dy, (K, R, R, C), stride, pad)
        nat._K.wgrad_set_direct(0)
        scheds = []
        for sch in (0, 1, 2):       # double buffer / 5-slot 32-pixel ring / early piece issue
            nat._K.wgrad_set_deep(sch)
            scheds.append(nat.conv2d_wgrad(x, dy, (K, R, R, C), stride, pad))
    finally:
        nat._K.wgrad_set_direct(0)
        nat._K.wgrad_set_deep(_WGRAD_DEEP_DEFAULT)
    assert torch.equal(pp, direct)
    assert torch.equal(pp, readl)
    for o in scheds:                # same MFMA order in every schedule
        assert torch.equal(pp, o)


WGRAD_DENSE_CASES = [
    (4, 14, 14, 1024, 256),              # late 1x1
    (3, 9, 11, 384, 264),                # partial Kout / T*C tiles, M not a multiple of 64
    (4096, 1, 1, 768, 3072),             # dense layer dW
    (40000, 1, 1, 256, 512),             # many splits, ragged last split
    (4, 28, 28, 512, 128),               # Kout 128: the LDS-DMA kernel's dense form
    (3, 23, 29, 64, 256),                # T*C 64: LDS-DMA kernel, ragged pixel count
]


@pytest.mark.parametrize("case", WGRAD_DENSE_CASES)
def test_wgrad_pingpong_dense_form_bit_identical(case):
    """The ping-pong wgrad kernel's DENSE form (one-tap unit-stride layers addressed as plain
    rows, no pixel decode) is bit-identical to its general form and matches the fp32 dW."""
    N, H, W, C, K = case
    nat = _native()
    torch.manual_seed(1)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, H, W, K, device=dev).to(torch.bfloat16)
    try:
        nat._K.wgrad_set_dense(1)
        dense = nat.conv2d_wgrad(x, dy, (K, 1, 1, C), 1, 0)
        others = []
        for sch in (0, 1, 2):
            nat._K.wgrad_set_deep(sch)
            others.append(nat.conv2d_wgrad(x, dy, (K, 1, 1, C), 1, 0))
        nat._K.wgrad_set_deep(_WGRAD_DEEP_DEFAULT)
        nat._K.wgrad_set_dense(0)
        gen = nat.conv2d_wgrad(x, dy, (K, 1, 1, C), 1, 0)
    finally:
        nat._K.wgrad_set_dense(1)
        nat._K.wgrad_set_deep(_WGRAD_DEEP_DEFAULT)
    assert torch.equal(dense, gen)
    for o in others:
        assert torch.equal(dense, o)
    ref = dy.reshape(-1, K).float().t() @ x.reshape(-1, C).float()
    assert _rel(dense.reshape(K, C), ref) < 1e-3


CONV_GEMM_CASES = [
    (2, 28, 28, 128, 128, 3, 1, 1),      # Kout 128: the 256 x 128 ping-pong tile
    (3, 15, 13, 128, 128, 3, 2, 1),      #   strided, odd sizes
    (2, 14, 14, 256, 256, 3, 1, 1),
    (3, 9, 11, 128, 384, 3, 1, 1),       # partial tiles, image edges in every tile
    (2, 28, 28, 256, 256, 3, 2, 1),      # strided: forward + the 4 dgrad phase classes
    (4, 7, 7, 512, 512, 3, 1, 1),
    (2, 14, 14, 512, 256, 1, 2, 0),      # 1x1 stride-2 projection: one dgrad phase, rest zero
]


@pytest.mark.parametrize("case", CONV_GEMM_CASES)
def test_conv_implicit_gemm_route(case):
    """Convs with C % 64 == 0 and Kout >= 256 on the ping-pong GEMM (implicit-GEMM A loader;
    strided data gradients as phase classes with remapped output rows): forward and data
    gradient vs the fp32 reference and vs the conv kernels, plus the BatchNorm statistics."""
    N, H, W, C, K, R, stride, pad = case
    nat, ref = _native(), _ref()
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(K, R, R, C, device=dev) / (R * R * C) ** 0.5
    outs = []
    try:
        for route in (3, 0):
            nat._K.conv_set_gemm(route)
            xn = x.clone().requires_grad_(True)
            wn = w.clone().requires_grad_(True)
            yn = nat.conv2d(xn, wn, stride, pad, bn_stats=True)
            g = torch.randn(yn.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).bfloat16()
            yn.backward(g)
            part = yn._dtf_bn_part
            outs.append((yn.detach(), xn.grad, wn.grad, part))
    finally:
        nat._K.conv_set_gemm(1)
    (y1, dx1, dw1, p1), (y0, dx0, dw0, p0) = outs
    xr = x.float().requires_grad_(True)
    yr = ref.conv2d(xr, w.to(torch.bfloat16).float(), stride, pad)
    yr.backward(g.float())
    assert _rel(y1, yr) < 1e-2 and _rel(y1, y0) < 1e-2
    assert _rel(dx1, xr.grad) < 2e-2 and _rel(dx1, dx0) < 2e-2
    # BN statistics: per-channel sums of the bf16 outputs, whatever the slab's row count
    pt, G = p1[0], p1[1]
    s1 = pt[:G * 2 * K].view(G, 2, K).double().sum(0)
    yf = y1.double().reshape(-1, K)
    torch.testing.assert_close(s1[0], yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s1[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-2)
