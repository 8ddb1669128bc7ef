"""Model zoo + NHWC reference ops on CPU: parameter counts / TF variable names of the
reference's models (``run_mnist_distributed.py:46-70``, ``templates/00_mnist_replica.py:138-164``),
TF padding / batch-norm semantics, forward/backward sanity and a short convergence run."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from distributedtensorflow_amd import ops
from distributedtensorflow_amd.models import MnistCNN, MnistMLP, collect_variables, resnet50
from distributedtensorflow_amd.models.resnet import num_params
from distributedtensorflow_amd.ops import reference as R
from distributedtensorflow_amd.optimizers import AdamOptimizer, GradientDescentOptimizer
from distributedtensorflow_amd.parallel import OneDeviceStrategy


def test_mnist_cnn_params_and_names():
    m = MnistCNN()
    assert num_params(m) == 3_274_634
    names = [n for n, _, _ in collect_variables(m)]
    assert names == ["conv2d/kernel", "conv2d/bias", "conv2d_1/kernel", "conv2d_1/bias",
                     "dense/kernel", "dense/bias", "dense_1/kernel", "dense_1/bias"]
    # a second model in a new scope starts numbering again (per-graph uniquification)
    names2 = [n for n, _, _ in collect_variables(MnistCNN())]
    assert names2 == names


def test_mnist_cnn_forward_backward():
    torch.manual_seed(0)
    m = MnistCNN()
    x = torch.rand(8, 784)
    y = torch.randint(0, 10, (8,))
    logits = m(x)
    assert logits.shape == (8, 10) and logits.dtype == torch.float32
    loss = ops.sparse_softmax_cross_entropy(logits, y)
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


def test_mnist_mlp_template():
    m = MnistMLP(hidden_units=100)
    names = [n for n, _, _ in collect_variables(m)]
    assert names == ["hid_w", "hid_b", "sm_w", "sm_b"]
    assert m.hid_w.abs().max() <= 2.0 / 28 + 1e-6          # truncated normal, stddev 1/28
    onehot = torch.eye(10)[torch.randint(0, 10, (4,))]
    loss = ops.softmax_cross_entropy_clipped_sum(m(torch.rand(4, 784)), onehot)
    assert loss.ndim == 0 and loss.item() > 0


def test_resnet50_params_names_and_step():
    torch.manual_seed(0)
    m = resnet50()
    assert num_params(m) == 25_557_032
    names = [n for n, _, _ in collect_variables(m)]
    assert names[0] == "conv1_conv/kernel"
    assert "conv2_block1_0_conv/kernel" in names and "conv5_block3_3_bn/moving_variance" in names
    assert names[-1] == "predictions/bias"
    assert len(names) == len(set(names))
    x = torch.randn(2, 64, 64, 3)
    y = torch.randint(0, 1000, (2,))
    with OneDeviceStrategy("cpu").scope():
        opt = GradientDescentOptimizer(0.01)
        loss = ops.sparse_softmax_cross_entropy(m(x), y)
        opt.minimize(loss)
    assert torch.isfinite(loss)


@pytest.mark.parametrize("h,r,stride,padding", [(28, 5, 1, "same"), (7, 3, 2, "SAME"),
                                                 (8, 3, 2, "same"), (9, 1, 2, "valid"),
                                                 (224, 7, 2, 3)])
def test_conv_padding_matches_tf(h, r, stride, padding):
    torch.manual_seed(0)
    x = torch.randn(2, h, h, 4, dtype=torch.float64)
    w = torch.randn(6, r, r, 4, dtype=torch.float64)
    y = R.conv2d(x, w, stride, padding)
    # direct TF definition: SAME -> out = ceil(h/s), pad_total split low=floor(total/2)
    if isinstance(padding, str) and padding.lower() == "same":
        out = -(-h // stride)
        tot = max((out - 1) * stride + r - h, 0)
        lo, hi = tot // 2, tot - tot // 2
    elif isinstance(padding, str):
        lo = hi = 0
    else:
        lo = hi = padding
    xp = F.pad(x.permute(0, 3, 1, 2), (lo, hi, lo, hi))
    want = F.conv2d(xp, w.permute(0, 3, 1, 2), stride=stride).permute(0, 2, 3, 1)
    torch.testing.assert_close(y, want)


def test_batch_norm_tf_semantics():
    torch.manual_seed(0)
    x = torch.randn(4, 3, 3, 5, dtype=torch.float64) * 3 + 1
    g, b = torch.rand(5, dtype=torch.float64), torch.randn(5, dtype=torch.float64)
    rm, rv = torch.zeros(5, dtype=torch.float64), torch.ones(5, dtype=torch.float64)
    res = torch.randn_like(x)
    y = R.batch_norm(x, g, b, rm, rv, True, 0.9, 1e-3, relu=True, residual=res)
    xf = x.reshape(-1, 5).numpy()
    mu, var = xf.mean(0), xf.var(0)
    want = np.maximum((xf - mu) / np.sqrt(var + 1e-3) * g.numpy() + b.numpy()
                      + res.reshape(-1, 5).numpy(), 0)
    np.testing.assert_allclose(y.reshape(-1, 5).numpy(), want, rtol=2e-5, atol=1e-6)
    n = xf.shape[0]
    np.testing.assert_allclose(rm.numpy(), 0.1 * mu, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(rv.numpy(), 0.9 + 0.1 * var * n / (n - 1), rtol=2e-5, atol=1e-6)
    # inference uses the moving statistics
    yi = R.batch_norm(x, g, b, rm, rv, False, 0.9, 1e-3)
    want_i = (xf - rm.numpy()) / np.sqrt(rv.numpy() + 1e-3) * g.numpy() + b.numpy()
    np.testing.assert_allclose(yi.reshape(-1, 5).numpy(), want_i, rtol=2e-5, atol=1e-6)


def test_maxpool_same_padding_and_gap():
    x = torch.randn(1, 5, 5, 2)
    y = R.max_pool2d(x, 3, 2, "same")
    assert y.shape == (1, 3, 3, 2)
    torch.testing.assert_close(y[0, 0, 0], x[0, :2, :2].reshape(-1, 2).max(0).values)
    torch.testing.assert_close(R.global_avg_pool(x), x.mean((1, 2)))


def test_cnn_learns_synthetic_mnist():
    """The reference CNN + Adam(5e-4) drives the loss down on the offline MNIST stand-in."""
    from distributedtensorflow_amd.data.mnist import synthetic_mnist
    torch.manual_seed(0)
    imgs, labels = synthetic_mnist(512, seed=3)
    x = torch.from_numpy(imgs.reshape(512, 784).astype(np.float32) / 255.0)
    y = torch.from_numpy(labels.astype(np.int64))
    m = MnistCNN()
    with OneDeviceStrategy("cpu").scope():
        opt = AdamOptimizer(5e-4)
        first = None
        for step in range(30):
            i = (step * 64) % 512
            loss = ops.sparse_softmax_cross_entropy(m(x[i:i + 64]), y[i:i + 64])
            opt.minimize(loss)
            first = first if first is not None else loss.item()
    assert loss.item() < 0.5 * first


def test_space_to_depth_stem_rewrite_is_exact():
    """The stem's 7x7/2 conv == a 4x4/1 VALID conv on the space-to-depth image (forward and the
    weight gradient mapped back through the rewrite), incl. odd sizes."""
    from distributedtensorflow_amd.ops import reference as ref
    torch.manual_seed(0)
    for (h, w_, c, R, pad) in [(32, 32, 3, 7, 3), (17, 23, 3, 7, 3), (12, 10, 5, 3, 1)]:
        x = torch.randn(2, h, w_, c, dtype=torch.float64)
        w = torch.randn(6, R, R, c, dtype=torch.float64, requires_grad=True)
        y0 = ref.conv2d(x, w, 2, pad)
        g = torch.randn_like(y0)
        (gw0,) = torch.autograd.grad((y0 * g).sum(), w)
        xs, ws = ref.space_to_depth_operands(x, w, 2, pad)
        assert xs.shape[-1] % 8 == 0 and ws.shape[1] == -(-R // 2)
        y1 = ref.conv2d(xs, ws, 1, 0)
        assert y1.shape == y0.shape
        torch.testing.assert_close(y1, y0)
        (gw1,) = torch.autograd.grad((y1 * g).sum(), w)
        torch.testing.assert_close(gw1, gw0)
