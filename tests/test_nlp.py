"""BERT-base MLM path (BASELINE config 5): model structure / TF names on CPU, and the HIP
transformer kernels (csrc/kernels/nlp.hip) against fp32 PyTorch references of the same op —
including bit-identical hash dropout masks, so dropout-on numerics are compared exactly."""
import pytest
import torch

from distributedtensorflow_amd import ops
from distributedtensorflow_amd.models import collect_variables
from distributedtensorflow_amd.models.bert import BertConfig, BertForPreTraining, bert_base
from distributedtensorflow_amd.models.resnet import num_params
from distributedtensorflow_amd.ops import reference as R
from distributedtensorflow_amd.optimizers import LAMBOptimizer
from distributedtensorflow_amd.parallel import OneDeviceStrategy

TINY = dict(vocab_size=1000, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
            intermediate_size=512, max_position_embeddings=128)


def _batch(B=4, S=64, P=10, V=1000, device="cpu", seed=0):
    g = torch.Generator().manual_seed(seed)
    cpu = dict(device="cpu")
    ids = torch.randint(0, V, (B, S), generator=g, **cpu)
    tt = (torch.arange(S, **cpu) >= S // 2).long().expand(B, S).contiguous()
    am = torch.ones(B, S, **cpu)
    am[1, S - 9:] = 0
    pos = torch.randint(0, S - 10, (B, P), generator=g, **cpu)
    lab = torch.randint(0, V, (B, P), generator=g, **cpu)
    w = torch.ones(B, P, **cpu)
    w[:, P - 2:] = 0
    return [t.to(device) for t in (ids, tt, am, pos, lab, w)]


# ----------------------------------------------------------------------------- CPU
def test_bert_base_size_and_tf_names():
    m = bert_base()
    names = [n for n, _, _ in collect_variables(m)]
    for n in ("bert/embeddings/word_embeddings", "bert/embeddings/LayerNorm/gamma",
              "bert/encoder/layer_0/attention/self/query/kernel",
              "bert/encoder/layer_11/attention/self/value/bias",
              "bert/encoder/layer_5/intermediate/dense/kernel",
              "bert/encoder/layer_5/output/LayerNorm/beta",
              "cls/predictions/transform/dense/kernel", "cls/predictions/output_bias"):
        assert n in names, n
    assert not any("qkv" in n for n in names)
    shapes = {n: tuple(t.shape) for n, t, _ in collect_variables(m)}
    assert shapes["bert/embeddings/word_embeddings"] == (30522, 768)
    assert shapes["cls/predictions/output_bias"] == (30522,)
    total = sum(t.numel() for _, t, _ in collect_variables(m))
    assert total == m.num_params_tf()
    # the tied vocabulary is stored padded to 30528 rows (table and output bias)
    assert num_params(m) == total + 6 * (768 + 1)


def test_bert_param_count_exact():
    cfg = BertConfig()
    H, I, V, L = 768, 3072, 30522, 12
    per_layer = 4 * (H * H + H) + 2 * 2 * H + (H * I + I) + (I * H + H)
    emb = (V + 512 + 2) * H + 2 * H
    head = H * H + H + 2 * H + V
    assert BertForPreTraining(cfg).num_params_tf() == emb + L * per_layer + head


def test_bert_padded_vocab_is_the_unpadded_model_cpu():
    """The tied decoder's vocabulary rows are padded to a multiple of 64 (1000 -> 1024 here):
    the padding rows start at zero, receive an exact zero gradient (the loss leaves their logits
    out of the softmax, ids never gather them) and stay zero through LAMB updates, the loss
    equals the unpadded model's, and checkpoints hold the TF shapes."""
    from distributedtensorflow_amd.models.bert import padded_vocab
    from distributedtensorflow_amd.train import Saver, list_variables
    torch.manual_seed(0)
    cfg = BertConfig(**TINY, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    V, Vp = cfg.vocab_size, padded_vocab(cfg.vocab_size)
    assert Vp == 1024
    m = BertForPreTraining(cfg)
    assert m.word_embeddings.shape == (Vp, 256) and m.mlm_bias.shape == (Vp,)
    assert torch.count_nonzero(m.word_embeddings[V:]) == 0
    batch = _batch()
    # the loss of the padded model == cross-entropy over the first V logits of an unpadded head
    ids, tt, am, pos, lab, w = batch
    logits = m(ids, tt, am, pos)
    assert logits.shape == (4 * 10, V)
    ref = R.mlm_loss(logits, lab, w)
    with OneDeviceStrategy("cpu").scope():
        opt = LAMBOptimizer(5e-3, weight_decay=0.01)
        loss = m(*batch)
        torch.testing.assert_close(loss, ref)
        g = opt.compute_gradients(loss, list(m.parameters()))
        grads = {id(v): gv for gv, v in g}
        assert torch.count_nonzero(grads[id(m.word_embeddings)][V:]) == 0
        assert torch.count_nonzero(grads[id(m.mlm_bias)][V:]) == 0
        opt.apply_gradients(g)
        for _ in range(3):
            opt.minimize(m(*batch))
    assert torch.count_nonzero(m.word_embeddings.detach()[V:]) == 0
    assert torch.count_nonzero(m.mlm_bias.detach()[V:]) == 0
    names = dict(list_variables(Saver(model=m, optimizer=opt).save(None, str(
        __import__("tempfile").mkdtemp()) + "/bert.ckpt")))
    assert names["bert/embeddings/word_embeddings"] == [V, 256]
    assert names["cls/predictions/output_bias"] == [V]
    assert names["bert/embeddings/word_embeddings/adam_m"] == [V, 256]


def test_bert_tiny_trains_with_lamb_cpu():
    torch.manual_seed(0)
    m = BertForPreTraining(BertConfig(**TINY, hidden_dropout_prob=0.0,
                                      attention_probs_dropout_prob=0.0))
    batch = _batch()
    with OneDeviceStrategy("cpu").scope():
        opt = LAMBOptimizer(5e-3)
        first = None
        for _ in range(15):
            loss = m(*batch)
            opt.minimize(loss)
            first = first if first is not None else loss.item()
    assert loss.item() < first - 0.3


def test_qkv_split_checkpoint_roundtrip(tmp_path):
    from distributedtensorflow_amd.train import Saver, list_variables, load_variable
    torch.manual_seed(0)
    m = BertForPreTraining(BertConfig(**TINY))
    with OneDeviceStrategy("cpu").scope():
        opt = LAMBOptimizer(1e-3)
        opt.minimize(m(*_batch()))
    p = Saver(model=m, optimizer=opt).save(None, str(tmp_path / "bert.ckpt"))
    names = dict(list_variables(p))
    assert names["bert/encoder/layer_1/attention/self/key/kernel"] == [256, 256]
    assert "bert/encoder/layer_1/attention/self/key/kernel/adam_m" in names
    qk = m.layers[1].qkv_kernel.detach()
    torch.testing.assert_close(
        torch.from_numpy(load_variable(p, "bert/encoder/layer_1/attention/self/key/kernel")),
        qk[256:512].t())
    m2 = BertForPreTraining(BertConfig(**TINY))
    Saver(model=m2).restore(None, p)
    torch.testing.assert_close(m2.layers[1].qkv_kernel, m.layers[1].qkv_kernel)


def test_keep_mask_rate_and_determinism():
    idx = torch.arange(200_000)
    k = R.keep_mask(1234, idx, 0.1)
    assert abs(k.float().mean().item() - 0.9) < 0.005
    assert torch.equal(k, R.keep_mask(1234, idx, 0.1))
    assert not torch.equal(k, R.keep_mask(1235, idx, 0.1))


def test_reference_attention_matches_naive():
    torch.manual_seed(0)
    B, S, H, D = 2, 16, 3, 64
    qkv = torch.randn(B * S, 3 * H * D)
    mask = torch.zeros(B, S)
    mask[0, 10:] = -10000.0
    out = R.attention_qkv(qkv, mask, B, S, H)
    x = qkv.view(B, S, 3, H, D)
    for b in range(B):
        for h in range(H):
            q, k, v = x[b, :, 0, h], x[b, :, 1, h], x[b, :, 2, h]
            p = torch.softmax(q @ k.t() / 8.0 + mask[b], -1)
            torch.testing.assert_close(out.view(B, S, H, D)[b, :, h], p @ v, atol=1e-5, rtol=1e-5)


# ----------------------------------------------------------------------------- GPU kernels
def _leaf(t, dtype=torch.bfloat16):
    return t.to("cuda", dtype).detach().requires_grad_(True)


def _grads_of(fn, inputs, dy):
    for t in inputs:
        if t is not None:
            t.grad = None
    y = fn()
    y.backward(dy)
    return y.detach().float(), [None if t is None else t.grad.detach().float() for t in inputs]


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("H", [768, 1024])
@pytest.mark.parametrize("wide", [0, 3])
def test_fused_layer_norm_gpu(p, H, wide):
    """bias + dropout + residual + LayerNorm forward / backward against fp32, with the 8-B and the
    16-B half-wave-per-row kernels (``wide``: bit 0 forward, bit 1 backward; M = 300 leaves a
    partial last block)."""
    from distributedtensorflow_amd.ops import native
    native.kernels().ln_set_wide(wide)
    try:
        _fused_layer_norm_case(p, H)
    finally:
        native.kernels().ln_set_wide(1)


def _fused_layer_norm_case(p, H):
    torch.manual_seed(0)
    M = 300
    a32, r32 = torch.randn(M, H), torch.randn(M, H)
    bias = torch.randn(H) * 0.1
    gamma, beta = 1 + 0.1 * torch.randn(H), 0.1 * torch.randn(H)
    dy = torch.randn(M, H)
    # native
    a, r = _leaf(a32), _leaf(r32)
    b, g, be = (_leaf(t, torch.float32) for t in (bias, gamma, beta))
    torch.manual_seed(7)
    y, (da, dr, db, dg, dbe) = _grads_of(
        lambda: ops.bias_dropout_add_layer_norm(a, b, r, g, be, p, True),
        [a, r, b, g, be], dy.cuda().bfloat16())
    # fp32 reference on the same bf16-rounded inputs and the same dropout seed
    a_, r_ = (t.bfloat16().float().requires_grad_(True) for t in (a32, r32))
    b_, g_, be_ = (t.clone().requires_grad_(True) for t in (bias, gamma, beta))
    torch.manual_seed(7)
    y_, (da_, dr_, db_, dg_, dbe_) = _grads_of(
        lambda: R.bias_dropout_add_layer_norm(a_, b_, r_, g_, be_, p, True),
        [a_, r_, b_, g_, be_], dy.bfloat16().float())
    torch.testing.assert_close(y.cpu(), y_, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(da.cpu(), da_, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(dr.cpu(), dr_, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(db.cpu(), db_, atol=0.3, rtol=2e-2)
    torch.testing.assert_close(dg.cpu(), dg_, atol=0.3, rtol=2e-2)
    torch.testing.assert_close(dbe.cpu(), dbe_, atol=0.3, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("with_tt,B", [(True, 3), (False, 5)])
def test_embedding_layer_norm_gpu(with_tt, B):
    torch.manual_seed(0)
    V, P, T, H, S = 500, 128, 2, 768, 128
    word, pos, typ = torch.randn(V, H) * 0.02, torch.randn(P, H) * 0.02, torch.randn(T, H) * 0.02
    gamma, beta = 1 + 0.1 * torch.randn(H), 0.1 * torch.randn(H)
    ids = torch.randint(0, 50, (B, S))          # many repeats -> exercises the segment sum
    tt = torch.randint(0, 2, (B, S)) if with_tt else None
    dy = torch.randn(B * S, H)
    leaves = [_leaf(t, torch.float32) for t in (word, pos, typ, gamma, beta)]
    torch.manual_seed(3)
    y, gr = _grads_of(lambda: ops.embedding_layer_norm(ids.cuda(), tt.cuda() if with_tt else None,
                                                       *leaves, p=0.1),
                      leaves, dy.cuda().bfloat16())
    leaves_ = [t.clone().requires_grad_(True) for t in (word, pos, typ, gamma, beta)]
    torch.manual_seed(3)
    y_, gr_ = _grads_of(lambda: R.embedding_layer_norm(ids, tt, *leaves_, p=0.1,
                                                       dtype=torch.bfloat16).float(),
                        leaves_, dy.bfloat16().float())
    torch.testing.assert_close(y.cpu(), y_, atol=3e-2, rtol=2e-2)
    # d(LN input) is stored in bf16 (|ds| ~ 30 here: rstd of 0.02-scale tables) and then summed
    # over up to ~10 rows per id, so allow bf16-of-the-summands absolute error
    for a, b in zip(gr, gr_):
        torch.testing.assert_close(a.cpu(), b, atol=0.02 * b.abs().max().item(), rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N", [(257, 3072), (16390, 768)])
def test_bias_gelu_gpu(M, N):
    torch.manual_seed(0)
    a32, bias, dy = torch.randn(M, N) * 2, torch.randn(N), torch.randn(M, N)
    a, b = _leaf(a32), _leaf(bias, torch.float32)
    y, (da, db) = _grads_of(lambda: ops.bias_gelu(a, b), [a, b], dy.cuda().bfloat16())
    a_, b_ = a32.bfloat16().float().requires_grad_(True), bias.clone().requires_grad_(True)
    y_, (da_, db_) = _grads_of(lambda: R.bias_gelu(a_, b_), [a_, b_], dy.bfloat16().float())
    torch.testing.assert_close(y.cpu(), y_, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(da.cpu(), da_, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(db.cpu(), db_, atol=0.2, rtol=2e-2)


@pytest.mark.gpu
def test_bias_gelu_gpu_large_magnitudes():
    """The r = 1 / (1 + e^{2u}) GELU form (csrc/kernels/common.h) at pre-activations where
    e^{2u} overflows to inf or underflows to 0: gelu -> x / 0 and gelu' -> 1 / 0 exactly as the
    fp32 tanh form, no NaN."""
    torch.manual_seed(0)
    vals = torch.tensor([-3e4, -200.0, -40.0, -9.5, -4.0, -1e-3, 0.0, 1e-3, 4.0, 9.5, 40.0, 200.0,
                         3e4])
    a32 = vals.repeat(64, 8)[:, :96].contiguous()           # [64, 96]
    bias = torch.zeros(96)
    dy = torch.randn(64, 96)
    a, b = _leaf(a32), _leaf(bias, torch.float32)
    y, (da, db) = _grads_of(lambda: ops.bias_gelu(a, b), [a, b], dy.cuda().bfloat16())
    a_, b_ = a32.bfloat16().float().requires_grad_(True), bias.clone().requires_grad_(True)
    y_, (da_, db_) = _grads_of(lambda: R.bias_gelu(a_, b_), [a_, b_], dy.bfloat16().float())
    assert torch.isfinite(y.float()).all() and torch.isfinite(da.float()).all()
    torch.testing.assert_close(y.cpu(), y_, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(da.cpu(), da_, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("B,S,H,p,masked", [(2, 128, 2, 0.0, True), (2, 128, 3, 0.1, True),
                                            (1, 512, 2, 0.0, False), (1, 64, 1, 0.1, False),
                                            (2, 192, 2, 0.1, True)])
def test_attention_gpu(B, S, H, p, masked):
    torch.manual_seed(0)
    D = 64
    qkv32 = torch.randn(B * S, 3 * H * D)
    mask = torch.zeros(B, S)
    if masked:
        mask[0, S - 37:] = -10000.0
    dy = torch.randn(B * S, H * D)
    x = _leaf(qkv32)
    torch.manual_seed(11)
    y, (dx,) = _grads_of(lambda: ops.attention_qkv(x, mask.cuda() if masked else None, B, S, H,
                                                   p, True), [x], dy.cuda().bfloat16())
    x_ = qkv32.bfloat16().float().requires_grad_(True)
    torch.manual_seed(11)
    y_, (dx_,) = _grads_of(lambda: R.attention_qkv(x_, mask if masked else None, B, S, H, p,
                                                   True), [x_], dy.bfloat16().float())
    torch.testing.assert_close(y.cpu(), y_, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(dx.cpu(), dx_, atol=5e-2, rtol=5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_wide_blocks_bit_identical(p):
    """8-wave / 128-row attention blocks (fwd and dQ, S % 128 == 0) == the 4-wave / 64-row shape: same
    per-lane summation order, so forward output and dQKV match bit for bit."""
    from distributedtensorflow_amd.ops import native
    torch.manual_seed(0)
    B, S, H = 3, 256, 2
    qkv = torch.randn(B * S, 3 * H * 64, device="cuda").bfloat16().requires_grad_(True)
    mask = torch.zeros(B, S, device="cuda")
    mask[1, S - 50:] = -10000.0
    dy = torch.randn(B * S, H * 64, device="cuda").bfloat16()
    outs = []
    for wide in (1, 0):
        native._K.attn_set_wide(wide)
        try:
            torch.manual_seed(5)
            y = ops.attention_qkv(qkv, mask, B, S, H, p, True)
            (g,) = torch.autograd.grad(y, [qkv], dy)
            torch.cuda.synchronize()
        finally:
            native._K.attn_set_wide(1)
        outs.append((y, g))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_fused_bwd_bit_identical(p):
    """S == 128: the fused one-block-per-(b, h) backward (dQ, dK, dV from one staging of Q / K /
    V / dO) == the split dQ + dK/dV kernels bit for bit -- every accumulator sums in the same
    order and P / dS are rounded to bf16 the same way -- with a padded key mask and dropout."""
    from distributedtensorflow_amd.ops import native
    torch.manual_seed(0)
    B, S, H = 5, 128, 3
    qkv = torch.randn(B * S, 3 * H * 64, device="cuda").bfloat16().requires_grad_(True)
    mask = torch.zeros(B, S, device="cuda")
    mask[1, S - 50:] = -10000.0
    mask[4, 7:] = -10000.0
    dy = torch.randn(B * S, H * 64, device="cuda").bfloat16()
    outs = []
    for fused in (1, 0):
        native._K.attn_set_fused(fused)
        try:
            torch.manual_seed(5)
            y = ops.attention_qkv(qkv, mask, B, S, H, p, True)
            (g,) = torch.autograd.grad(y, [qkv], dy)
            torch.cuda.synchronize()
        finally:
            native._K.attn_set_fused(1)
        outs.append((y, g))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.gpu
def test_attention_keep_bits_bit_identical():
    """S == 128 with dropout: the forward stores its keep decisions (one bit per score) and the
    fused backward reads them instead of re-hashing: outputs and gradients bit-identical to the
    re-hashing backward, and the buffer really holds the decisions (~keep rate of ones)."""
    from distributedtensorflow_amd.ops import native
    torch.manual_seed(0)
    B, S, H, p = 3, 128, 4, 0.1
    qkv = torch.randn(B * S, 3 * H * 64, device="cuda").bfloat16().requires_grad_(True)
    mask = torch.zeros(B, S, device="cuda")
    mask[2, 90:] = -10000.0
    dy = torch.randn(B * S, H * 64, device="cuda").bfloat16()
    assert native._K.attn_keep_words(B, S, H, p) == B * H * S * 4
    outs = []
    for keep in (1, 0):
        native._K.attn_set_keep(keep)
        try:
            torch.manual_seed(5)
            y = ops.attention_qkv(qkv, mask, B, S, H, p, True)
            (g,) = torch.autograd.grad(y, [qkv], dy)
            torch.cuda.synchronize()
        finally:
            native._K.attn_set_keep(1)
        outs.append((y, g))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    # the stored words: about (1 - p) of the bits set
    kw = torch.empty(B * H * S * 4, device="cuda", dtype=torch.int32)
    out = torch.empty(B * S, H * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device="cuda")
    native._K.attn_fwd(qkv.detach().data_ptr(), mask.data_ptr(), out.data_ptr(), lse.data_ptr(),
                       B, S, H, 0.125, p, 77, torch.cuda.current_stream().cuda_stream,
                       kw.data_ptr())
    torch.cuda.synchronize()
    bits = torch.stack([(kw >> i) & 1 for i in range(32)]).sum().item()
    assert abs(bits / (32 * kw.numel()) - (1 - p)) < 0.01


@pytest.mark.gpu
def test_qkv_bias_grad_from_fused_attention_partials():
    """S == 128: the fused attention backward leaves per-sequence column sums of dQKV, and the
    QKV projection's bias gradient is their B-row sum (no pass over dQKV).  It must equal the
    column sum of the very dQKV the kernel stored (the split path, which re-reads dQKV), up to
    fp32 summation order, and the other gradients must not change at all."""
    from distributedtensorflow_amd.ops import native
    torch.manual_seed(0)
    B, S, H, D = 6, 128, 2, 64
    x = torch.randn(B * S, 96, device="cuda").bfloat16().requires_grad_(True)
    w = torch.nn.Parameter(torch.randn(3 * H * D, 96, device="cuda") * 0.1)
    b = torch.nn.Parameter(torch.randn(3 * H * D, device="cuda") * 0.1)
    mask = torch.zeros(B, S, device="cuda")
    mask[2, 100:] = -10000.0
    dy = torch.randn(B * S, H * D, device="cuda").bfloat16()
    res = []
    for fused in (1, 0):
        native._K.attn_set_fused(fused)
        try:
            torch.manual_seed(3)
            qkv = ops.dense(x, w, b, impl="library")      # BERT's QKV projection path
            y = ops.attention_qkv(qkv, mask, B, S, H, 0.1, True)
            gx, gw, gb = torch.autograd.grad(y, [x, w, b], dy)
            torch.cuda.synchronize()
        finally:
            native._K.attn_set_fused(1)
        res.append((gx, gw, gb))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    torch.testing.assert_close(res[0][2], res[1][2], rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_mlm_loss_gpu():
    torch.manual_seed(0)
    N, V = 80, 30522
    lg32 = torch.randn(N, V) * 3
    lab = torch.randint(0, V, (N,))
    lab[0], lab[1], lab[2] = 0, V - 1, 7          # labels on the misaligned row ends
    w = (torch.rand(N) > 0.2).float()
    w[:3] = 1.0
    lg = _leaf(lg32)
    loss, (dl,) = _grads_of(lambda: ops.mlm_loss(lg, lab.cuda(), w.cuda()), [lg], None)
    lg_ = lg32.bfloat16().float().requires_grad_(True)
    loss_, (dl_,) = _grads_of(lambda: R.mlm_loss(lg_, lab, w), [lg_], None)
    torch.testing.assert_close(loss.cpu(), loss_, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(dl.cpu(), dl_, atol=1e-4, rtol=2e-2)


@pytest.mark.gpu
def test_bert_tiny_gpu_matches_cpu_and_trains():
    torch.manual_seed(0)
    cfg = BertConfig(**TINY, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m_cpu = BertForPreTraining(cfg)
    m_gpu = BertForPreTraining(cfg)
    m_gpu.load_state_dict(m_cpu.state_dict())
    m_gpu.cuda()
    batch = _batch()
    ref = m_cpu(*batch).item()
    with OneDeviceStrategy("cuda").scope():
        loss = m_gpu(*[t.cuda() for t in batch])
        assert abs(loss.item() - ref) < 0.05 * abs(ref)
        opt = LAMBOptimizer(5e-3)
        first = loss.item()
        for _ in range(15):
            loss = m_gpu(*[t.cuda() for t in _batch()])
            opt.minimize(loss)
    assert loss.item() < first - 0.3


def _bert_grads(model, batch, direct, to_dense):
    from distributedtensorflow_amd.ops import native, native_nlp
    prev = native._DIRECT_GRAD, native_nlp._RESIDUAL_TO_DENSE
    native._DIRECT_GRAD, native_nlp._RESIDUAL_TO_DENSE = direct, to_dense
    try:
        with OneDeviceStrategy("cuda").scope():
            opt = LAMBOptimizer(1e-3)
            loss = model(*batch)
            opt.compute_gradients(loss, list(model.parameters()))
            torch.cuda.synchronize()
            return loss.item(), opt.space.grad.clone()
    finally:
        native._DIRECT_GRAD, native_nlp._RESIDUAL_TO_DENSE = prev


@pytest.mark.gpu
def test_bert_fused_grad_paths_match_autograd():
    """LayerNorm / bias-GELU parameter gradients written straight into the flat buffer, and
    d(residual) summed by the consuming dense's dgrad GEMM (beta = 1), vs plain autograd."""
    import copy
    torch.manual_seed(0)
    cfg = BertConfig(**TINY, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1)
    base = BertForPreTraining(cfg).cuda()
    batch = [t.cuda() for t in _batch()]
    torch.manual_seed(1)
    la, ga = _bert_grads(copy.deepcopy(base), batch, True, True)
    torch.manual_seed(1)
    lb, gb = _bert_grads(copy.deepcopy(base), batch, False, False)
    torch.manual_seed(1)
    lc, gc = _bert_grads(copy.deepcopy(base), batch, True, False)
    assert la == lb == lc
    assert torch.equal(gc, gb)            # direct-to-buffer writes only: bit-identical
    cos = torch.nn.functional.cosine_similarity(ga.double(), gb.double(), dim=0).item()
    assert cos > 0.9999, cos              # GEMM beta=1 rounds once instead of twice
    assert (ga - gb).abs().max() <= 0.02 * gb.abs().max()



@pytest.mark.gpu
@pytest.mark.parametrize("T,I,O", [(1024, 3072, 768), (777, 256, 96), (300, 128, 64)])
def test_bias_gelu_dense_fused_backward(T, I, O):
    """gelu(a + b1) @ W2^T with d(a) formed by ONE GEMM pass carrying the GELU derivative and the
    b1 column sums in its epilogue == the unfused bias_gelu + library dense (and an fp32
    reference)."""
    torch.manual_seed(0)
    a32 = torch.randn(T, I) * 2
    b1 = torch.randn(I) * 0.5
    w2 = torch.randn(O, I) * I ** -0.5
    do = torch.randn(T, O)

    def run(fused):
        a = a32.cuda().bfloat16().requires_grad_(True)
        b = b1.cuda().requires_grad_(True)
        w = w2.cuda().requires_grad_(True)
        if fused:
            y = ops.bias_gelu_dense(a, b, w)
        else:
            y = ops.dense(ops.bias_gelu(a, b), w, None, impl="library")
        y.backward(do.cuda().bfloat16())
        return y.float().cpu(), a.grad.float().cpu(), b.grad.cpu(), w.grad.cpu()

    fy, fa, fb, fw = run(True)
    uy, ua, ub, uw = run(False)
    torch.testing.assert_close(fy, uy, atol=0, rtol=0)          # same forward kernels
    a_ = a32.bfloat16().float().requires_grad_(True)
    b_ = b1.clone().requires_grad_(True)
    w_ = w2.bfloat16().float().requires_grad_(True)
    y_ = R.bias_gelu(a_, b_) @ w_.t()
    y_.backward(do.bfloat16().float())
    for got, unf, ref in ((fa, ua, a_.grad), (fb, ub, b_.grad), (fw, uw, w_.grad)):
        scale = ref.abs().max()
        assert (got - ref).abs().max() <= 2e-2 * scale, (got - ref).abs().max() / scale
        assert (got - unf).abs().max() <= 2e-2 * scale


@pytest.mark.gpu
@pytest.mark.parametrize("T,H,I", [(4096, 768, 3072), (1000, 256, 1024), (600, 128, 96)])
def test_dense_gelu_dense_fused_epilogue(T, H, I):
    """BERT's FFN as one op: the first GEMM on our MFMA kernel with the bias + GELU epilogue
    (gemm.hip gelu_out: pre-activation and activation in one pass) == the two-pass form (library
    GEMM + bias_gelu kernel) and an fp32 reference, forward and every gradient."""
    from distributedtensorflow_amd.ops import native
    torch.manual_seed(0)
    x32 = torch.randn(T, H)
    w1 = torch.randn(I, H) * H ** -0.5
    b1 = torch.randn(I) * 0.5
    w2 = torch.randn(H, I) * I ** -0.5
    do = torch.randn(T, H)
    calls = []
    orig = native._K.gemm_nt_bias_gelu

    def spy(*a):
        calls.append(1)
        return orig(*a)

    def run(fused):
        prev = native._FFN_GEMM_GELU
        native._FFN_GEMM_GELU = fused
        native._K.gemm_nt_bias_gelu = spy
        try:
            x = x32.cuda().bfloat16().requires_grad_(True)
            p = [t.cuda().requires_grad_(True) for t in (w1, b1, w2)]
            y = ops.dense_gelu_dense(x, *p)
            y.backward(do.cuda().bfloat16())
            torch.cuda.synchronize()
            return [y.float().cpu(), x.grad.float().cpu()] + [t.grad.cpu() for t in p]
        finally:
            native._FFN_GEMM_GELU = prev
            native._K.gemm_nt_bias_gelu = orig

    got = run(True)
    assert calls, "the fused bias + GELU GEMM did not run"
    unf = run(False)
    x_ = x32.bfloat16().float().requires_grad_(True)
    p_ = [w1.bfloat16().float().requires_grad_(True), b1.clone().requires_grad_(True),
          w2.bfloat16().float().requires_grad_(True)]
    y_ = R.bias_gelu(x_ @ p_[0].t(), p_[1]) @ p_[2].t()
    y_.backward(do.bfloat16().float())
    refs = [y_.detach(), x_.grad] + [t.grad for t in p_]
    for name, g, u, r in zip(("y", "dx", "dw1", "db1", "dw2"), got, unf, refs):
        scale = r.abs().max()
        assert (g - r).abs().max() <= 2e-2 * scale, (name, ((g - r).abs().max() / scale).item())
        assert (g - u).abs().max() <= 2e-2 * scale, (name, ((g - u).abs().max() / scale).item())


@pytest.mark.gpu
def test_tied_decoder_padded_vocab_on_our_kernels(monkeypatch):
    """BERT's tied MLM decoder on the padded vocabulary (768 -> 30528, 30522 classes): forward,
    data gradient and weight gradient run on our GEMM / weight-gradient kernels -- the torch
    (hipBLASLt) entry points are booby-trapped -- and match an fp32 reference over the 30522
    classes; the 6 padding logits are exactly 0 and the padding rows of the table and the bias
    get exactly zero gradient."""
    from distributedtensorflow_amd.ops import native
    torch.manual_seed(0)
    T, H, V, Vp = 1000, 768, 30522, 30528
    h32 = torch.randn(T, H)
    w32 = torch.randn(Vp, H) * 0.05
    w32[V:] = 0
    b32 = torch.randn(Vp) * 0.1
    b32[V:] = 0
    lab = torch.randint(0, V, (T,))
    lab[:2] = torch.tensor([V - 1, V - 2])         # classes next to the padding
    wts = (torch.rand(T) > 0.2).float()

    def trap(*a, **k):
        raise AssertionError("library GEMM called on the decoder path")

    for mod, name in ((torch.nn.functional, "linear"), (torch, "mm"), (torch, "bmm"),
                      (torch, "addmm"), (torch, "matmul"), (torch.Tensor, "__matmul__"),
                      (torch.Tensor, "addmm_")):
        monkeypatch.setattr(mod, name, trap)
    h = _leaf(h32)
    w = _leaf(w32, torch.float32)
    b = _leaf(b32, torch.float32)
    calls = []
    orig = native._K.conv_wgrad
    monkeypatch.setattr(native._K, "conv_wgrad", lambda *a: (calls.append(1), orig(*a))[1])
    logits = ops.dense(h, w, b, impl="library")
    assert logits.shape == (T, Vp)
    loss = ops.mlm_loss(logits, lab.cuda(), wts.cuda(), vocab=V)
    loss.backward()
    torch.cuda.synchronize()
    monkeypatch.undo()
    assert calls, "the decoder weight gradient did not run on our wgrad kernel"
    lg = logits.detach().float().cpu()
    assert torch.count_nonzero(lg[:, V:]) == 0
    assert torch.count_nonzero(w.grad[V:]) == 0 and torch.count_nonzero(b.grad[V:]) == 0
    # fp32 reference over the classes only, on the same bf16-rounded operands
    h_ = h32.bfloat16().float().requires_grad_(True)
    w_ = w32[:V].bfloat16().float().requires_grad_(True)
    b_ = b32[:V].clone().requires_grad_(True)
    lg_ = h_ @ w_.t() + b_
    loss_ = R.mlm_loss(lg_, lab, wts)
    loss_.backward()
    for name, got, ref in (("logits", lg[:, :V], lg_.detach()), ("dx", h.grad.float().cpu(), h_.grad),
                           ("dw", w.grad[:V].cpu(), w_.grad), ("db", b.grad[:V].cpu(), b_.grad)):
        scale = ref.abs().max()
        err = (got - ref).abs().max()
        assert err <= 2e-2 * scale, (name, (err / scale).item())
    torch.testing.assert_close(loss.detach().cpu(), loss_.detach(), atol=2e-3, rtol=2e-3)
