"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip), the fused dense / conv bias+ReLU epilogues and
their fused backward (csrc/kernels/dense.hip) against plain PyTorch fp32 references of the same
ops (reference ``run_mnist_distributed.py:52-69``)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1000, 40, 72), (4099, 1000, 2048),
                                   (128, 1024, 3136), (77, 8, 8), (3000, 520, 1000)])
def test_gemm_nt_vs_fp32(M, N, K):
    from distributedtensorflow_amd.ops import native
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = torch.randn(N, K, device="cuda", generator=g).bfloat16()   # asymmetric operands
    ref = a.float() @ b.float().t()
    out = native.gemm_nt(a, b)
    assert out.shape == (M, N)
    assert _rel(out, ref) < 1e-2
    bias = torch.randn(N, device="cuda", generator=g)
    cin = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    out2 = native.gemm_nt(a, b, bias=bias, relu=True)
    assert _rel(out2, torch.relu(ref + bias)) < 1e-2
    out3 = native.gemm_nt(a, b, cin=cin)
    assert _rel(out3, ref + cin.float()) < 1e-2


def test_gemm_nt_strided_rows_and_identity():
    from distributedtensorflow_amd.ops import native
    g = torch.Generator(device="cuda").manual_seed(3)
    big = torch.randn(300, 200, device="cuda", generator=g).bfloat16()
    a = big[:, :128]                                  # lda = 200 > K
    eye = torch.eye(128, device="cuda").bfloat16()
    out = native.gemm_nt(a, eye)                     # A . I^T = A exactly
    assert torch.equal(out, a)


def _dense_case(M, i, o, relu, bias=True):
    from distributedtensorflow_amd.ops import native
    g = torch.Generator(device="cuda").manual_seed(M * 7 + o)
    x = torch.randn(M, i, device="cuda", generator=g).bfloat16().requires_grad_()
    w = (torch.randn(o, i, device="cuda", generator=g) / i ** 0.5).requires_grad_()
    b = torch.randn(o, device="cuda", generator=g).requires_grad_() if bias else None
    y = native.dense(x, w, b, relu, "native")
    dy = torch.randn(M, o, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().bfloat16().float().requires_grad_()
    br = b.detach().float().requires_grad_() if bias else None
    yr = xr @ wr.t() + (br if bias else 0)
    yr = torch.relu(yr) if relu else yr
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    if bias:
        assert _rel(b.grad, br.grad) < 2e-2


@pytest.mark.parametrize("M,i,o,relu", [(128, 3136, 1024, True), (128, 1024, 10, False),
                                        (256, 2048, 1000, False), (100, 784, 104, True)])
def test_native_dense_fwd_bwd(M, i, o, relu):
    """MNIST dense 3136->1024+ReLU and logits 1024->10 (padded to 16 internally), ResNet FC."""
    _dense_case(M, i, o, relu)


@pytest.mark.parametrize("C,K,H", [(1, 32, 28), (32, 64, 14)])
def test_conv_bias_relu_fused(C, K, H):
    """tf.layers.conv2d(5x5 SAME, activation=relu) on the MNIST shapes, fwd + bwd vs fp32."""
    from distributedtensorflow_amd.ops import native, reference
    g = torch.Generator(device="cuda").manual_seed(C * K)
    x = torch.randn(16, H, H, C, device="cuda", generator=g).bfloat16().requires_grad_()
    w = (torch.randn(K, 5, 5, C, device="cuda", generator=g) * 0.1).requires_grad_()
    b = (torch.randn(K, device="cuda", generator=g) * 0.1).requires_grad_()
    y = native.conv2d_bias_relu(x, w, b, 1, "same", True)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().bfloat16().float().requires_grad_()
    br = b.detach().float().requires_grad_()
    yr = torch.relu(reference.conv2d(xr, wr, 1, "same") + br)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2
    assert _rel(x.grad, xr.grad) < 2e-2


def test_mnist_cnn_trains_on_native_kernels():
    """The reference CNN (run_mnist_distributed.py:46-70) on the GPU: every conv, pool, dense,
    loss and Adam update on our kernels; no hipBLASLt."""
    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import MnistCNN
    from distributedtensorflow_amd.parallel import OneDeviceStrategy
    torch.manual_seed(0)
    with OneDeviceStrategy("/gpu:0").scope():
        model = MnistCNN()
        opt = dtf.train.AdamOptimizer(1e-3)
        opt.build(list(model.parameters()))
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.rand(128, 784, device="cuda", generator=g).bfloat16()
    y = torch.randint(0, 10, (128,), device="cuda", generator=g)
    losses = []
    for _ in range(30):
        loss = ops.sparse_softmax_cross_entropy(model(x), y)
        opt.minimize(loss)
        losses.append(float(loss))
    assert losses[-1] < 0.5 * losses[0], losses


# ----------------------------------------------------------------------------- fp32 path
def _rel64(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("layout", ["OI", "IO"])
def test_fp32_dense_fwd_bwd(layout):
    """f32-input MFMA GEMM (exact fp32 fma chains): tight agreement with fp64."""
    from distributedtensorflow_amd.ops import native_f32
    g = torch.Generator(device="cuda").manual_seed(5)
    M, i, o = 128, 784, 100
    x = torch.randn(M, i, device="cuda", generator=g).requires_grad_()
    w = torch.randn(*((o, i) if layout == "OI" else (i, o)), device="cuda", generator=g)
    w = (w / i ** 0.5).requires_grad_()
    b = torch.randn(o, device="cuda", generator=g).requires_grad_()
    y = native_f32.dense(x, w, b, True, layout)
    dy = torch.randn(M, o, device="cuda", generator=g)
    y.backward(dy)
    xr, wr, br = (t.detach().double().requires_grad_() for t in (x, w, b))
    yr = torch.relu(xr @ (wr.t() if layout == "OI" else wr) + br)
    yr.backward(dy.double())
    assert _rel64(y, yr) < 1e-5
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert _rel64(got, ref) < 1e-5


@pytest.mark.parametrize("C,K,H", [(1, 32, 28), (32, 64, 14)])
def test_fp32_conv_bias_relu_and_pool(C, K, H):
    from distributedtensorflow_amd.ops import native_f32
    g = torch.Generator(device="cuda").manual_seed(C + K)
    x = torch.randn(8, H, H, C, device="cuda", generator=g).requires_grad_()
    w = (torch.randn(K, 5, 5, C, device="cuda", generator=g) * 0.1).requires_grad_()
    b = (torch.randn(K, device="cuda", generator=g) * 0.1).requires_grad_()
    y = native_f32.max_pool2d(native_f32.conv2d_bias_relu(x, w, b, 1, "same", True), 2, 2)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().double().requires_grad_() for t in (x, w, b))
    conv = torch.nn.functional.conv2d(xr.permute(0, 3, 1, 2), wr.permute(0, 3, 1, 2), br,
                                      padding=2)
    yr = torch.nn.functional.max_pool2d(torch.relu(conv), 2, 2).permute(0, 2, 3, 1)
    yr.backward(dy.double())
    assert _rel64(y, yr) < 1e-5
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert _rel64(got, ref) < 1e-5


def test_clipped_softmax_xent_matches_reference_formula():
    """templates/00_mnist_replica.py:160-164 loss and its TF gradient (clip passes inside)."""
    from distributedtensorflow_amd.ops import native_f32, reference
    g = torch.Generator(device="cuda").manual_seed(9)
    z = (torch.randn(100, 10, device="cuda", generator=g) * 3).requires_grad_()
    t = torch.nn.functional.one_hot(torch.randint(0, 10, (100,), device="cuda", generator=g),
                                    10).float()
    loss = native_f32.softmax_cross_entropy_clipped_sum(z, t)
    loss.backward()
    zr = z.detach().double().requires_grad_()
    lr = reference.softmax_cross_entropy_clipped_sum(zr, t.double())
    lr.backward()
    assert abs(float(loss) - float(lr)) < 1e-4 * abs(float(lr))
    assert _rel64(z.grad, zr.grad) < 1e-5


def test_fused_u8_gather_normalise():
    from distributedtensorflow_amd.data import DeviceArrayDataset
    import numpy as np
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (300, 784), dtype=np.uint8)
    labs = rng.integers(0, 10, 300).astype(np.int32)
    for dt in (torch.float32, torch.bfloat16):
        ds = DeviceArrayDataset(imgs, labs, 128, "cuda", dtype=dt, shuffle=True, seed=3)
        x, y = next(ds)
        idx = ds._order[:128]
        ref = torch.as_tensor(imgs, device="cuda")[idx].float() / 255.0
        assert torch.equal(x, ref.to(dt)) and torch.equal(y, ds.labels[idx])


def test_mnist_cnn_and_mlp_train_fp32_on_native_kernels():
    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import MnistCNN, MnistMLP
    from distributedtensorflow_amd.parallel import OneDeviceStrategy
    torch.manual_seed(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.rand(128, 784, device="cuda", generator=g)
    y = torch.randint(0, 10, (128,), device="cuda", generator=g)
    with OneDeviceStrategy("/gpu:0").scope():
        cnn, mlp = MnistCNN(), MnistMLP()
        o1, o2 = dtf.train.AdamOptimizer(1e-3), dtf.train.AdamOptimizer(1e-3)
        o1.shadow_dtype = o2.shadow_dtype = None
        o1.build(list(cnn.parameters()))
        o2.build(list(mlp.parameters()))
    assert o1.space.shadow is None
    onehot = torch.nn.functional.one_hot(y, 10).float()
    l1, l2 = [], []
    for _ in range(30):
        loss = ops.sparse_softmax_cross_entropy(cnn(x), y)
        o1.minimize(loss)
        l1.append(float(loss))
        loss2 = ops.softmax_cross_entropy_clipped_sum(mlp(x), onehot)
        o2.minimize(loss2)
        l2.append(float(loss2))
    assert l1[-1] < 0.6 * l1[0] and l2[-1] < 0.7 * l2[0], (l1, l2)


def test_gemm_bn_stats_and_masked_residual_epilogues():
    """The 1x1-conv epilogues of the GEMM: per-M-tile BatchNorm sums of the bf16 output and the
    masked residual-gradient add (dy * relu bit) -- vs the same quantities computed by torch."""
    from distributedtensorflow_amd.ops import native
    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K = 1000, 256, 128
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    G = native.kernels().gemm_tile_rows(M)
    stats = torch.empty(G, 2, N, device="cuda")
    y = native.gemm_nt(a, b, stats=stats)
    yf = y.float()
    torch.testing.assert_close(stats[:, 0].sum(0), yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(stats[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-4, atol=1e-1)
    torch.testing.assert_close(stats[0, 0], yf[:256].sum(0), rtol=1e-4, atol=1e-2)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    bits = torch.randint(0, 2, (M, N), device="cuda", generator=g, dtype=torch.uint8)
    w8 = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], device="cuda", dtype=torch.int32)
    mask = (bits.view(M, N // 8, 8).int() * w8).sum(-1).to(torch.uint8).contiguous()
    y2 = native.gemm_nt(a, b, acc_from=native._MaskedGrad(dy, mask))
    ref = (y.float() + dy.float() * bits.float())
    assert _rel(y2, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(1000, 776, 200), (4096, 2304, 768), (300, 264, 1000),
                                   (513, 512, 64), (256, 256, 4096)])
def test_gemm_pingpong_schedule_bit_identical(M, N, K):
    """The ping-pong (two-group, barrier-staggered) K-loops of gemm.hip -- variant 8 (256 x 256)
    and variant 10 (256 x 128, three LDS slots) -- accumulate every output in the same MFMA
    order as the default pipeline: results must be bit-identical, with bias+ReLU, with Cin
    accumulation, and on M / N / K tails."""
    from distributedtensorflow_amd.ops import native
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    cin = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    outs = []
    try:
        for v in (0, 8, 10):
            native._K.gemm_set_variant(v)
            outs.append((native.gemm_nt(a, b), native.gemm_nt(a, b, bias=bias, relu=True),
                         native.gemm_nt(a, b, cin=cin.clone())))
    finally:
        native._K.gemm_set_variant(-1)
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)
    ref = a.float() @ b.float().t()
    assert ((outs[1][0].float() - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.parametrize("T,i,o", [(40000, 256, 512), (65536, 768, 768)])
def test_native_dense_wgrad_many_tokens(T, i, o):
    """dW of the native dense layer over more tokens than the wgrad kernels' packed pixel
    coordinates could once index (tokens run as T images of 1x1, not one T x 1 image): every
    token must contribute."""
    from distributedtensorflow_amd.ops import native
    g = torch.Generator(device="cuda").manual_seed(T + i)
    x = torch.randn(T, i, device="cuda", generator=g).bfloat16()
    w = (torch.randn(o, i, device="cuda", generator=g) / i ** 0.5).requires_grad_(True)
    dy = torch.randn(T, o, device="cuda", generator=g).bfloat16()
    native.dense(x, w, None, False, impl="native").backward(dy)
    ref = dy.float().t() @ x.float()
    assert ((w.grad.float() - ref).norm() / ref.norm()).item() < 1e-3
