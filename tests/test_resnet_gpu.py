"""ResNet-50 end to end on the GPU: the native op graph against the PyTorch reference graph on
the same weights, and the direct-to-flat-buffer gradient path against plain autograd
accumulation (must be bit-identical)."""
import copy

import pytest
import torch

from distributedtensorflow_amd import ops
from distributedtensorflow_amd.models import resnet50
from distributedtensorflow_amd.ops import native
from distributedtensorflow_amd.optimizers import MomentumOptimizer
from distributedtensorflow_amd.parallel import OneDeviceStrategy

pytestmark = pytest.mark.gpu


def _inputs(n=4, s=64):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(n, s, s, 3, generator=g, device="cpu")
    y = torch.randint(0, 1000, (n,), generator=g, device="cpu")
    return x.cuda().bfloat16(), y.cuda()


def _grads(model, direct, fuse_res=True, share=True, fuse_bnb=False, lazy=True):
    """Gradients of one step.  The fused BN-backward sums (summation order differs from the
    reduce kernel; both the register-kernel and the streamed-GEMM forms) stay off unless asked
    for, so the other fusions can be checked bit-exactly."""
    prev, prev_r, prev_s = native._DIRECT_GRAD, native._FUSE_RESIDUAL_GRAD, native._SHARE_INPUT_GRAD
    prev_b, prev_l = native._FUSE_BN_BWD, native._LAZY_RESIDUAL_GRAD
    prev_bs, prev_c1 = native._FUSE_BN_BWD_STREAM, native._FUSE_C1_BWD
    prev_d, prev_h = native._FUSE_DUAL_BNB, native._FUSE_BN_BWD_HALO
    prev_s2 = native._FUSE_BN_BWD_S2
    native._FUSE_BN_BWD_HALO = native._FUSE_BN_BWD_S2 = fuse_bnb
    native._FUSE_BN_BWD = fuse_bnb
    native._FUSE_BN_BWD_STREAM = fuse_bnb
    native._FUSE_C1_BWD = fuse_bnb
    native._FUSE_DUAL_BNB = fuse_bnb
    native._LAZY_RESIDUAL_GRAD = lazy
    native._DIRECT_GRAD = direct
    native._FUSE_RESIDUAL_GRAD = fuse_res
    native._SHARE_INPUT_GRAD = share
    try:
        with OneDeviceStrategy("cuda").scope():
            opt = MomentumOptimizer(0.1, 0.9)
            x, y = _inputs()
            loss = ops.sparse_softmax_cross_entropy(model(x), y)
            opt.compute_gradients(loss, list(model.parameters()))
            torch.cuda.synchronize()
            return loss.item(), opt.space.grad.clone()
    finally:
        native._DIRECT_GRAD, native._FUSE_RESIDUAL_GRAD = prev, prev_r
        native._SHARE_INPUT_GRAD = prev_s
        native._FUSE_BN_BWD, native._LAZY_RESIDUAL_GRAD = prev_b, prev_l
        native._FUSE_BN_BWD_STREAM, native._FUSE_C1_BWD = prev_bs, prev_c1
        native._FUSE_DUAL_BNB, native._FUSE_BN_BWD_HALO = prev_d, prev_h
        native._FUSE_BN_BWD_S2 = prev_s2


def test_direct_grad_path_bit_identical():
    torch.manual_seed(0)
    base = resnet50().cuda()
    a = copy.deepcopy(base)
    b = copy.deepcopy(base)
    la, ga = _grads(a, True)
    lb, gb = _grads(b, False)
    assert la == lb
    assert torch.equal(ga, gb)
    assert ga.abs().sum() > 0


def test_resnet50_eval_native_matches_reference_graph():
    """Whole-network inference forward, native bf16 kernels vs the fp32 PyTorch reference."""
    torch.manual_seed(0)
    m = resnet50().cuda().eval()
    x, _ = _inputs()
    with torch.no_grad():
        nat = m(x).float()
        ops.set_backend("reference")
        try:
            ref = m(x.float()).float()
        finally:
            ops.set_backend("auto")
    rel = ((nat - ref).norm() / ref.norm()).item()
    assert rel < 0.05, rel


def test_resnet50_train_first_stage_matches_reference():
    """Training-mode (batch-statistics BN) forward through the stem and stage 1.

    Deeper outputs are not compared: a random-init BN ResNet is chaotic — feeding the fp32
    reference graph the bf16-ROUNDED input (0.17% change) already moves the final block by 23%
    (a per-layer probe in round 1), so end-to-end agreement is not a kernel-accuracy test."""
    torch.manual_seed(0)
    m = resnet50().cuda().train()
    x, _ = _inputs(n=16, s=96)
    outs = {}

    def grab(tag):
        def hook(mod, i, o):
            outs.setdefault(tag, []).append(o.detach().float())
        return hook
    hs = [b.register_forward_hook(grab(k)) for k, b in
          [("stem", m.stem)] + [(f"b{i}", m.blocks[i]) for i in range(3)]]
    rm = [b.clone() for b in m.buffers()]
    with torch.no_grad():
        m(x)
        for b, r in zip(m.buffers(), rm):
            b.copy_(r)
        ops.set_backend("reference")
        try:
            m(x.float())
        finally:
            ops.set_backend("auto")
    for h in hs:
        h.remove()
    for tag, (nat, ref) in outs.items():
        rel = ((nat - ref).norm() / ref.norm()).item()
        assert rel < 0.03, (tag, rel)


@pytest.mark.parametrize("shape", [(4, 56, 56, 64, 64, 1), (4, 28, 28, 128, 256, 3),
                                   (3, 9, 11, 64, 72, 3), (8, 14, 14, 256, 256, 3)])
def test_conv_epilogue_bn_stats_match_separate_pass(shape):
    """conv2d(bn_stats=True) + batch_norm (statistics from the conv epilogue) == the separate
    statistics kernel path: outputs, batch stats and moving averages."""
    N, H, W, C, K, R = shape
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5
    gamma = torch.rand(K, device="cuda") + 0.5
    beta = torch.randn(K, device="cuda") * 0.1
    outs = []
    for fused in (True, False):
        rm, rv = torch.zeros(K, device="cuda"), torch.ones(K, device="cuda")
        y = native.conv2d(x, w, 1, (R - 1) // 2, bn_stats=fused)
        assert hasattr(y, "_dtf_bn_part") == fused
        z = native.batch_norm(y, gamma, beta, rm, rv, True, 0.9, 1e-5, relu=True)
        outs.append((y.float(), z.float(), rm, rv))
    (y1, z1, m1, v1), (y2, z2, m2, v2) = outs
    assert torch.equal(y1, y2)
    torch.testing.assert_close(z1, z2, atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(m1, m2, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(v1, v2, atol=1e-5, rtol=1e-4)


def test_bn_relu_conv_fusion_bit_identical():
    """Bottleneck c2's BN + ReLU applied inside c3's streaming GEMM (ops.batch_norm_relu_conv1x1)
    == the separate BN apply pass + conv, for the whole ResNet-50 step (loss and every
    gradient)."""
    from distributedtensorflow_amd.models import resnet as R
    torch.manual_seed(0)
    base = resnet50().cuda()
    calls = {"n": 0}
    orig = native._K.gemm_stream_pre

    def spy(*a):
        calls["n"] += 1
        return orig(*a)
    prev = R.FUSE_BN_CONV
    try:
        R.FUSE_BN_CONV = True
        native._K.gemm_stream_pre = spy
        la, ga = _grads(copy.deepcopy(base), True)
        native._K.gemm_stream_pre = orig
        R.FUSE_BN_CONV = False
        lb, gb = _grads(copy.deepcopy(base), True)
    finally:
        R.FUSE_BN_CONV = prev
        native._K.gemm_stream_pre = orig
    assert calls["n"] == 13          # c3 of every stage-1..3 bottleneck (w = 64 / 128 / 256)
    assert la == lb
    assert torch.equal(ga, gb)


def _c1_grads(x, gamma, beta, w, g, fused):
    prev = native._FUSE_C1_BWD
    native._FUSE_C1_BWD = fused
    try:
        xs = x.detach().clone().requires_grad_(True)
        ps = [t.detach().clone().requires_grad_(True) for t in (gamma, beta, w)]
        C = x.shape[-1]
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        out = native.bn_relu_conv1x1(xs, ps[0], ps[1], rm, rv, ps[2], 0.9, 1e-5)
        seen = {}
        orig = native._bn_backward_core

        def spy(ctx, dy, *a, **k):
            seen["dy"] = dy.detach().clone()
            return orig(ctx, dy, *a, **k)
        native._bn_backward_core = spy
        try:
            grads = torch.autograd.grad(out, [xs] + ps, g)
        finally:
            native._bn_backward_core = orig
        torch.cuda.synchronize()
        return seen["dy"], grads
    finally:
        native._FUSE_C1_BWD = prev


@pytest.mark.parametrize("c,n,hw,grid", [(64, 4, 28, 0), (64, 4, 28, 3), (64, 1, 8, 0),
                                          (64, 2, 8, 1), (64, 3, 8, 1), (128, 4, 16, 0),
                                          (128, 4, 16, 5), (128, 1, 8, 1), (128, 6, 4, 1)])
def test_fused_c1_backward_matches_separate_passes(c, n, hw, grid):
    """Stage-0 / stage-1 c3 (64 -> 256, 128 -> 512) backward as ONE pass
    (csrc/kernels/conv1x1_bwd.hip: data gradient + weight gradient + the BN backward sums) ==
    the separate wgrad / dgrad / BN reduce passes: the data gradient bit for bit, dW / dgamma /
    dbeta / dx to fp32 summation order, and all of them against fp32 math of the op; persistent-
    grid walks of 1, 2, 3 and many tiles per block (``grid`` forces the block count)."""
    torch.manual_seed(0)
    k = 4 * c
    x = torch.randn(n, hw, hw, c, device="cuda").bfloat16()
    w = torch.randn(k, 1, 1, c, device="cuda") / c ** 0.5
    gamma = torch.rand(c, device="cuda") + 0.5
    beta = torch.randn(c, device="cuda") * 0.2
    g = torch.randn(n, hw, hw, k, device="cuda").bfloat16()
    assert native._K.conv1x1_bwd_ok(n * hw * hw, c, k)
    native._K.conv1x1_bwd_set_grid(grid)
    try:
        dy1, g1 = _c1_grads(x, gamma, beta, w, g, True)
    finally:
        native._K.conv1x1_bwd_set_grid(0)
    dy2, g2 = _c1_grads(x, gamma, beta, w, g, False)
    assert torch.equal(dy1, dy2)
    for a, b, name in zip(g1, g2, ("dx", "dgamma", "dbeta", "dw")):
        a, b = a.float(), b.float()
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < (2e-2 if name == "dx" else 1e-4), (name, rel)
    xs = x.float().requires_grad_(True)
    ps = [t.clone().requires_grad_(True) for t in (gamma, beta, w)]
    mean = xs.mean((0, 1, 2))
    var = xs.var((0, 1, 2), unbiased=False)
    yb = torch.relu((xs - mean) / torch.sqrt(var + 1e-5) * ps[0] + ps[1])
    ref = torch.einsum("nhwc,kc->nhwk", yb, ps[2].view(k, c))
    gr = torch.autograd.grad(ref, [xs] + ps, g.float())
    for a, b, name in zip(g1, gr, ("dx", "dgamma", "dbeta", "dw")):
        rel = ((a.float() - b).norm() / b.norm()).item()
        assert rel < 3e-2, (name, rel)


def test_residual_grad_fusion_bit_identical():
    """d(residual) accumulated in c1's dgrad epilogue == autograd's separate bf16 add."""
    torch.manual_seed(0)
    base = resnet50().cuda()
    la, ga = _grads(copy.deepcopy(base), True, fuse_res=True)
    lb, gb = _grads(copy.deepcopy(base), True, fuse_res=False)
    assert la == lb
    assert torch.equal(ga, gb)


@pytest.mark.parametrize("dma", [-1, 0, 1])
def test_lazy_residual_grad_bit_identical(dma):
    """Identity blocks: d(residual) formed as dy * relu_mask inside c1's dgrad epilogue (geom
    acc mode 2, never materialised) == the BN writing it and the epilogue reading it back; for
    the register-staged and the LDS-DMA dgrad kernels."""
    torch.manual_seed(0)
    base = resnet50().cuda()
    native._K.conv_set_dma_mode(dma)
    try:
        la, ga = _grads(copy.deepcopy(base), True, lazy=True)
        lb, gb = _grads(copy.deepcopy(base), True, lazy=False)
    finally:
        native._K.conv_set_dma_mode(-1)
    assert la == lb
    assert torch.equal(ga, gb)


def test_fused_stem_bn_relu_maxpool_bit_identical():
    """Stem BN + ReLU + 3x3/2 max-pool in one kernel (BN output never stored) == BN apply then
    max-pool: same rounded values, same argmax, so loss and every gradient match exactly."""
    from distributedtensorflow_amd.models import resnet as rn
    torch.manual_seed(0)
    base = resnet50().cuda()
    prev, prev_b = rn.FUSE_STEM_POOL, native._FUSE_STEM_POOL_BWD
    try:
        native._FUSE_STEM_POOL_BWD = False      # its reduce sums in another (fixed) order
        rn.FUSE_STEM_POOL = True
        la, ga = _grads(copy.deepcopy(base), True)
        rn.FUSE_STEM_POOL = False
        lb, gb = _grads(copy.deepcopy(base), True)
        native._FUSE_STEM_POOL_BWD = True
        rn.FUSE_STEM_POOL = True
        lc, gc = _grads(copy.deepcopy(base), True)
        ld, gd = _grads(copy.deepcopy(base), True)
    finally:
        rn.FUSE_STEM_POOL, native._FUSE_STEM_POOL_BWD = prev, prev_b
    assert la == lb == lc
    assert torch.equal(ga, gb)
    # pool gather fused into the stem BN backward: deterministic, and equal to the unfused
    # path up to the fp32 summation order of the BN reduction
    assert torch.equal(gc, gd)
    cos = torch.nn.functional.cosine_similarity(gc.double(), ga.double(), dim=0).item()
    assert cos > 0.99999, cos
    assert (gc - ga).abs().max() <= 1e-3 * ga.abs().max()


def test_masked_grad_materialize():
    """Fallback of the lazy residual gradient: dy * bit mask, vs torch."""
    torch.manual_seed(0)
    dy = torch.randn(4, 7, 5, 24, device="cuda").to(torch.bfloat16)
    keep = torch.rand(dy.shape, device="cuda") > 0.4
    bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)
    mask = bits.sum(dim=1).to(torch.uint8)
    out = native._MaskedGrad(dy, mask).materialize()
    assert torch.equal(out, torch.where(keep, dy, torch.zeros_like(dy)))


def test_shared_input_dgrad_bit_identical():
    """Projection blocks: proj's and c1's dgrads accumulated into one buffer in the epilogue ==
    autograd summing two separate dgrad tensors (round(round(a) + round(b)) either way)."""
    torch.manual_seed(0)
    base = resnet50().cuda()
    la, ga = _grads(copy.deepcopy(base), True, share=True)
    lb, gb = _grads(copy.deepcopy(base), True, share=False)
    assert la == lb
    assert torch.equal(ga, gb)


@pytest.mark.parametrize("stride,R,res,C,K", [(1, 3, False, 64, 128), (2, 3, False, 64, 128),
                                             (1, 1, True, 64, 128), (2, 1, True, 64, 128),
                                             (1, 3, True, 256, 256)])   # LDS-DMA dgrad kernel
def test_bn_backward_sums_fused_into_dgrad_epilogue(stride, R, res, C, K):
    """conv -> BN(+res)(+ReLU) -> conv: the second conv's dgrad epilogue emits the BN backward
    sums (incl. stride-2 multi-phase dgrads and the residual bit mask); gradients match the
    separate reduce pass to fp32 summation-order noise, and the fused path really ran."""
    torch.manual_seed(0)
    N, H = 4, 14
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w1 = torch.randn(C, 3, 3, C, device="cuda") / (9 * C) ** 0.5
    w2 = torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda") * 0.1
    r = torch.randn(N, H, H, C, device="cuda").bfloat16() if res else None
    outs = []
    prev = native._FUSE_BN_BWD
    seen = {}
    orig = native._K.bn_bwd_finalize_g

    def spy(*a):
        seen["g"] = True
        return orig(*a)
    try:
        for fuse in (True, False):
            native._FUSE_BN_BWD = fuse
            ps = [t.clone().requires_grad_(True) for t in (x.float(), w1, w2, gamma, beta)]
            xi = ps[0].detach().bfloat16().requires_grad_(True)
            y1 = native.conv2d(xi, ps[1], 1, 1, bn_stats=True)
            z = native.batch_norm(y1, ps[3], ps[4], None, None, True, 0.9, 1e-5, relu=True,
                                  residual=r)
            y2 = native.conv2d(z, ps[2], stride, (R - 1) // 2)
            g = torch.randn(y2.shape, device="cuda", generator=torch.Generator(
                device="cuda").manual_seed(1)).bfloat16()
            if fuse:
                native._K.bn_bwd_finalize_g = spy
            y2.backward(g)
            native._K.bn_bwd_finalize_g = orig
            outs.append((xi.grad.float(), ps[1].grad, ps[3].grad, ps[4].grad))
    finally:
        native._FUSE_BN_BWD = prev
        native._K.bn_bwd_finalize_g = orig
    assert seen.get("g"), "fused BN-backward path did not run"
    for a, b in zip(*outs):
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 2e-2, rel


def test_resnet50_grads_with_fused_bn_backward_sums():
    torch.manual_seed(0)
    base = resnet50().cuda()
    ma, mb = copy.deepcopy(base), copy.deepcopy(base)
    la, ga = _grads(ma, True, fuse_bnb=True)
    lb, gb = _grads(mb, True, fuse_bnb=False)
    assert la == lb
    # per-variable relative difference, from the loss end backwards: summation-order noise is
    # amplified layer by layer through the backward of a random-init BN network (chaotic, see
    # test_resnet50_train_first_stage_matches_reference), so the layers next to the loss must
    # agree tightly and the whole gradient must stay aligned
    cos = torch.nn.functional.cosine_similarity(ga, gb, dim=0).item()
    assert cos > 0.99, cos
    n_tail = 2048 * 1000                 # the fc kernel lives first in the flat buffer
    tail = ((ga[:n_tail] - gb[:n_tail]).norm() / gb[:n_tail].norm()).item()
    assert tail < 1e-2, tail


@pytest.mark.parametrize("block,cin,hw", [(0, 64, 16), (1, 256, 16), (3, 256, 16), (4, 512, 8)])
def test_lazy_residual_bn_dx_formed_in_fused_c3_backward(block, cin, hw):
    """Stage-0/1 blocks: the residual BN's backward (the identity block's, or the projection
    block's dual BN) hands d(c3 output) over unformed (_LazyBnDx) and the fused c3 backward forms
    it per tile (conv1x1_bwd.hip LZ: 32-row tiles at stage 0, 16-row tiles with a 16-deep weight-
    gradient MFMA at stage 1) instead of the apply pass storing it: same block output, the
    block-input gradient and every parameter gradient match the stored-dO path (c3's data
    gradient bit for bit; dW / BN sums to summation order)."""
    torch.manual_seed(0)
    m = resnet50().cuda()
    blk = m.blocks[block]                     # s0b0 / s0b1 / s1b0 / s1b1
    x = torch.randn(2, hw, hw, cin, device="cuda").bfloat16()
    calls = {"n": 0}
    orig = native._K.conv1x1_bwd_lazy
    orig_core = native._bn_backward_core
    seen = {}

    def spy(*a):
        calls["n"] += 1
        return orig(*a)

    def core_spy(ctx, dy, *a, **k):
        if type(ctx).__name__.startswith("_BnReluConv1x1"):
            seen.setdefault(lz_now[0], []).append(dy.detach().clone())   # c3's data gradient
        return orig_core(ctx, dy, *a, **k)
    out = {}
    prev = native._FUSE_C3_LAZY
    g = None
    lz_now = [None]
    try:
        native._K.conv1x1_bwd_lazy = spy
        native._bn_backward_core = core_spy
        for lz in (True, False):
            lz_now[0] = lz
            native._FUSE_C3_LAZY = lz
            b = copy.deepcopy(blk)
            xi = x.clone().requires_grad_(True)
            y = b(xi)
            if g is None:
                g = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(
                    device="cuda", dtype=y.dtype)
            y.backward(g)
            torch.cuda.synchronize()
            out[lz] = (y.detach().float(), xi.grad.float(),
                       [p.grad.float() for p in b.parameters()])
    finally:
        native._K.conv1x1_bwd_lazy = orig
        native._bn_backward_core = orig_core
        native._FUSE_C3_LAZY = prev
    assert calls["n"] == 1
    # d(c3 output) formed in the kernel (from dy3, x3 or its recomputation, mask) is bit-identical
    # to the apply pass's stored one, so c3's data gradient is too
    assert len(seen[True]) == len(seen[False]) == 1
    assert torch.equal(seen[True][0], seen[False][0])
    (ya, dxa, ga), (yb, dxb, gb) = out[True], out[False]
    assert torch.equal(ya, yb)
    rel = ((dxa - dxb).norm() / dxb.norm()).item()
    assert rel < 2e-2, rel
    for i, (a, b) in enumerate(zip(ga, gb)):
        r = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        assert r < 2e-2, (i, r)


def _default_step_grads(model, dual):
    """One step's loss and flat gradient with the default fusions, the dual-BN sums on or off."""
    prev = native._FUSE_DUAL_BNB
    native._FUSE_DUAL_BNB = dual
    try:
        with OneDeviceStrategy("cuda").scope():
            opt = MomentumOptimizer(0.1, 0.9)
            x, y = _inputs()
            loss = ops.sparse_softmax_cross_entropy(model(x), y)
            opt.compute_gradients(loss, list(model.parameters()))
            torch.cuda.synchronize()
            return loss.item(), opt.space.grad.clone()
    finally:
        native._FUSE_DUAL_BNB = prev


@pytest.mark.parametrize("H,C,res", [(56, 64, False), (56, 64, True), (28, 128, False)])
def test_bn_backward_sums_fused_into_halo_dgrad(H, C, res):
    """conv -> BN(+res)(+ReLU) -> 3x3 conv on a halo-kernel shape (56 x 56 x 64, 28 x 28 x 128):
    the halo data-gradient kernel's epilogue emits the BN backward sums (ReLU recomputed from x,
    or the residual bit mask); every gradient matches the separate reduce pass to fp32
    summation-order noise, the data gradient itself bit for bit, and the halo kernel took it."""
    torch.manual_seed(0)
    N = 2
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w1 = torch.randn(C, 3, 3, C, device="cuda") / (9 * C) ** 0.5
    w2 = torch.randn(C, 3, 3, C, device="cuda") / (9 * C) ** 0.5
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda") * 0.1
    r = torch.randn(N, H, H, C, device="cuda").bfloat16() if res else None
    taps = [(1 - i // 3, 1 - i % 3) for i in range(9)]
    geom = native._fwd_geom((N, H, H, C), C, taps, H, H, 1, 1, H, H)
    assert native._K.conv_tile_rows(geom, [t[0] for t in taps], [t[1] for t in taps], 1) == \
        N * H // 4, "the fused-sum data gradient would not run on the halo kernel"
    outs, seen = [], {}
    prev = native._FUSE_BN_BWD, native._FUSE_BN_BWD_HALO
    orig = native._K.bn_bwd_finalize_g

    def spy(*a):
        seen["g"] = True
        return orig(*a)
    try:
        native._FUSE_BN_BWD = False
        for fuse in (True, False):
            native._FUSE_BN_BWD_HALO = fuse
            ps = [t.clone().requires_grad_(True) for t in (x.float(), w1, w2, gamma, beta)]
            xi = ps[0].detach().bfloat16().requires_grad_(True)
            y1 = native.conv2d(xi, ps[1], 1, 1, bn_stats=True)
            z = native.batch_norm(y1, ps[3], ps[4], None, None, True, 0.9, 1e-5, relu=True,
                                  residual=r)
            z.retain_grad()
            y2 = native.conv2d(z, ps[2], 1, 1)
            g = torch.randn(y2.shape, device="cuda", generator=torch.Generator(
                device="cuda").manual_seed(1)).bfloat16()
            if fuse:
                native._K.bn_bwd_finalize_g = spy
            y2.backward(g)
            native._K.bn_bwd_finalize_g = orig
            outs.append((z.grad.float(), xi.grad.float(), ps[1].grad, ps[3].grad, ps[4].grad))
    finally:
        native._FUSE_BN_BWD, native._FUSE_BN_BWD_HALO = prev
        native._K.bn_bwd_finalize_g = orig
    assert seen.get("g"), "fused BN-backward path did not run"
    assert torch.equal(outs[0][0], outs[1][0])          # the data gradient itself: same kernel
    for a, b in zip(outs[0][1:], outs[1][1:]):
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 2e-2, rel


def test_dual_bn_sums_from_streamed_dgrad():
    """A projection block's relu(BN(x) + BN_p(xp)) backward takes BOTH BatchNorms' sums from the
    next block's streamed c1 data gradient (gemm_stream DUAL epilogue) instead of its own dual
    reduce pass: used at the three stream-shaped stages, and the step's gradients match the
    separate-pass form to summation order."""
    torch.manual_seed(0)
    base = resnet50().cuda()
    calls = {"n": 0}
    orig = native._K.gemm_stream_bnb_dual

    def spy(*a):
        calls["n"] += 1
        return orig(*a)
    native._K.gemm_stream_bnb_dual = spy
    try:
        la, ga = _default_step_grads(copy.deepcopy(base), True)
    finally:
        native._K.gemm_stream_bnb_dual = orig
    assert calls["n"] == 3, calls          # s0b1 / s1b1 / s2b1 c1 (s3: reduction 512)
    lb, gb = _default_step_grads(copy.deepcopy(base), False)
    assert la == lb
    cos = torch.nn.functional.cosine_similarity(ga, gb, dim=0).item()
    assert cos > 0.99, cos
    n_tail = 2048 * 1000
    tail = ((ga[:n_tail] - gb[:n_tail]).norm() / gb[:n_tail].norm()).item()
    assert tail < 1e-2, tail


def _run_part(part, x, g, mode, **kw):
    """One forward + backward of ``part`` alone (training-mode BN, batch statistics) on input x:
    mode "native" (our kernels), "fp32" (the PyTorch reference graph in fp32) or "bf16" (the same
    reference graph on bf16 tensors: PyTorch's own bf16 storage path).  -> (y, dx, {name: grad})."""
    for p in part.parameters():
        p.grad = None
    saved = [b.clone() for b in part.buffers()]
    if mode != "native":
        ops.set_backend("reference")
    try:
        xi = (x.float() if mode == "fp32" else x).detach().clone().requires_grad_(x.requires_grad)
        y = part(xi, **kw)
        y.backward(g.to(y.dtype))
    finally:
        ops.set_backend("auto")
        for b, s in zip(part.buffers(), saved):
            b.copy_(s)
    torch.cuda.synchronize()
    return (y.detach().float(), xi.grad.float() if xi.grad is not None else None,
            {n: p.grad.float() for n, p in part.named_parameters()})


def test_resnet50_per_block_teacher_forced_vs_fp32():
    """Every stage of the training step checked ALONE against the fp32 reference graph, each fed
    the native network's own bf16 activation (teacher forcing): stem (+fused BN/ReLU/pool), all 16
    bottlenecks, and the head.  Forward output, input gradient and every parameter gradient.

    The bar is PyTorch's own bf16 path on the same graph, measured against the same fp32 result:
    with a random upstream gradient, ReLU masks that flip where a bf16-stored pre-activation
    rounds across zero (~0.1 % of elements) move gradient sums by sqrt(flip fraction) ~ 3-8 %,
    for any bf16-storage implementation (measured with tools/block_grad_probe.py).  The native
    kernels must be within 1.2x (+0.3 %) of that floor on every tensor, and the forward within
    2 % absolute.  Parameters are pre-rounded to bf16 so all sides see the same weights."""
    torch.manual_seed(0)
    m = resnet50().cuda().train()
    with torch.no_grad():
        for mod in m.modules():
            if hasattr(mod, "gamma"):
                mod.gamma.uniform_(0.5, 1.5)
                mod.beta.normal_(0.0, 0.1)
        for p in m.parameters():
            p.copy_(p.bfloat16().float())
    x, _ = _inputs(n=16, s=96)
    gen = torch.Generator(device="cuda").manual_seed(1)
    rel = lambda a, b: ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
    failures, lines = [], []

    def check(tag, part, xin, **kw):
        with torch.no_grad():           # the native activation handed to the next part
            y0 = part(xin.clone(), **kw)
        g = torch.randn(y0.shape, device="cuda", generator=gen).bfloat16()
        runs = {mode: _run_part(part, xin, g, mode, **kw) for mode in ("native", "fp32", "bf16")}
        (yn, dxn, gn), (yr, dxr, gr), (yb, dxb, gb) = (runs[k] for k in ("native", "fp32", "bf16"))
        pairs = [("fwd", yn, yb, yr)]
        if dxn is not None:
            pairs.append(("dx", dxn, dxb, dxr))
        pairs += [(n, gn[n], gb[n], gr[n]) for n in gn]
        for name, a, b, r in pairs:
            en, eb = rel(a, r), rel(b, r)
            lines.append(f"  {tag:8s} {name:18s} native {en:.5f}  torch-bf16 {eb:.5f}")
            bad = en > 0.02 if name == "fwd" else en > 1.2 * eb + 0.003
            if bad:
                failures.append((tag, name, en, eb))
        return y0.detach()

    act = check("stem", m.stem, x, pool=True)
    for i, blk in enumerate(m.blocks):
        act = check(f"block{i}", blk, act.bfloat16().requires_grad_(True))

    class _Head(torch.nn.Module):
        def __init__(self, fc):
            super().__init__()
            self.fc = fc

        def forward(self, a):
            return self.fc(ops.global_avg_pool(a)).float()
    check("head", _Head(m.fc), act.bfloat16().requires_grad_(True))
    print("\nteacher-forced relative errors vs fp32:\n" + "\n".join(lines))
    assert not failures, failures


def test_fused_projection_bn_bit_identical():
    """Projection blocks with the shortcut BN fused into the block-output BN
    (ops.batch_norm_add_batch_norm: one apply pass forward, one reduce + one apply pass backward
    for both BNs) against the two-op form: loss, every gradient and the moving statistics are
    bit-identical (the fused kernels round the shortcut BN output to bf16 in registers exactly
    as its own pass stored it, and each reduce slab is the single-BN slab)."""
    from distributedtensorflow_amd.models import resnet as rn
    torch.manual_seed(0)
    base = resnet50().cuda()
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    prev = rn.FUSE_PROJ_BN
    try:
        rn.FUSE_PROJ_BN = True
        la, ga = _grads(a, True)
        rn.FUSE_PROJ_BN = False
        lb, gb = _grads(b, True)
    finally:
        rn.FUSE_PROJ_BN = prev
    assert la == lb
    assert torch.equal(ga, gb)
    for (n1, t1), (n2, t2) in zip(a.named_buffers(), b.named_buffers()):
        assert n1 == n2 and torch.equal(t1, t2), n1


def test_batch_norm_add_batch_norm_vs_fp32():
    """The fused op against the fp32 reference formula relu(bn(x) + bn(xp)) with batch
    statistics, forward and backward."""
    g = torch.Generator(device="cuda").manual_seed(3)
    M, C = 4096, 256
    x = (torch.randn(8, 16, 32, C, device="cuda", generator=g) * 2 + 1).bfloat16().requires_grad_()
    xp = (torch.randn(8, 16, 32, C, device="cuda", generator=g) - 0.5).bfloat16().requires_grad_()
    gam, bet = torch.rand(C, device="cuda", generator=g) + 0.5, torch.randn(C, device="cuda", generator=g)
    gp, bp = torch.rand(C, device="cuda", generator=g) + 0.5, torch.randn(C, device="cuda", generator=g)
    params = [t.clone().requires_grad_() for t in (gam, bet, gp, bp)]
    rm, rv, rmp, rvp = (torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"),
                        torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"))
    y = native.batch_norm_add_batch_norm(x, params[0], params[1], rm, rv, xp, params[2],
                                         params[3], rmp, rvp, True, 0.9, 1e-5)
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)

    def bn(t, ga, be):
        t = t.float()
        mu = t.mean((0, 1, 2))
        var = t.var((0, 1, 2), unbiased=False)
        return (t - mu) / torch.sqrt(var + 1e-5) * ga + be

    xr, xpr = x.detach().float().requires_grad_(), xp.detach().float().requires_grad_()
    rp = [t.clone().requires_grad_() for t in (gam, bet, gp, bp)]
    # the ReLU mask of the native (bf16-rounded) output, so mask flips at ~0 do not count
    yr = (bn(xr, rp[0], rp[1]) + bn(xpr, rp[2], rp[3])) * (y.detach().float() > 0)
    yr.backward(dy.float())

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))
    assert rel(y, yr) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2 and rel(xp.grad, xpr.grad) < 1e-2
    for p, r in zip(params, rp):
        assert rel(p.grad, r.grad) < 1e-2
    torch.testing.assert_close(rm, 0.1 * x.detach().float().mean((0, 1, 2)), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("n", [2, 5])
def test_stem_halo_conv_bit_identical(n):
    """The space-to-depth stem conv (4x4 taps over 16 channels -> 64) on the halo kernel (input
    rows + whole filter in LDS) against the register kernel's chunk gather: identical outputs and
    BatchNorm partial sums; and against the fp32 7x7/2 convolution of the image."""
    from distributedtensorflow_amd.ops import reference
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, 224, 224, 3, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 7, 7, 3, device="cuda", generator=g) * 0.1)
    xs = native.space_to_depth_input(x, 2, 3, 7, 7)
    _, ws = reference.space_to_depth_operands(x, w, 2, 3, want_x=False)
    ws = ws.bfloat16().contiguous()
    outs = []
    try:
        for halo in (1, 0):
            native._K.conv_set_stem_halo(halo)
            y = native.conv2d(xs, ws, 1, 0, bn_stats=True)
            part, G, M, K = y._dtf_bn_part
            s = part[: G * 2 * K].view(G, 2, K)
            outs.append((y.clone(), s.sum(0)))
    finally:
        native._K.conv_set_stem_halo(1)
    (y1, s1), (y0, s0) = outs
    assert torch.equal(y1, y0)
    torch.testing.assert_close(s1, s0, rtol=1e-5, atol=1e-2)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2),
                                     w.bfloat16().float().permute(0, 3, 1, 2), stride=2, padding=3)
    ref = ref.permute(0, 2, 3, 1)
    assert float((y1.float() - ref).norm() / ref.norm()) < 1e-2


@pytest.mark.parametrize("n,acc", [(3, False), (8, True)])
def test_wgrad_halo_kernel_vs_fp32(n, acc):
    """Stage-1 3x3 weight gradient (56x56x64 -> 64) on the halo kernel (strip-persistent blocks,
    one tap per wave, per-block fp32 slabs reduced in order) against the fp32 reference and the
    tiled kernel; with accumulation into an existing gradient."""
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, 56, 56, 64, device="cuda", generator=g).bfloat16()
    dy = torch.randn(n, 56, 56, 64, device="cuda", generator=g).bfloat16()
    base = torch.randn(64, 3, 3, 64, device="cuda", generator=g)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 64, 3, 3),
                                      dy.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    if acc:
        ref = ref + base
    outs = []
    try:
        for halo in (1, 0):
            native._K.wgrad_set_halo(halo)
            out = base.clone().contiguous() if acc else None
            outs.append(native.conv2d_wgrad(x, dy, (64, 3, 3, 64), 1, 1, out=out))
    finally:
        native._K.wgrad_set_halo(1)
    for o in outs:
        assert float((o - ref).norm() / ref.norm()) < 1e-5, float((o - ref).norm() / ref.norm())
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n,acc", [(3, False), (6, True)])
def test_wgrad_stem_kernel_vs_fp32(n, acc):
    """The stem's weight gradient on its space-to-depth image (4x4 VALID taps over 16 channels,
    115x115 -> 112x112x64) on the strip kernel (one tap row per wave pair, the strip's dY and X
    rows LDS-DMA'd once, per-block fp32 slabs reduced in order) against the fp32 reference and
    the tiled kernel; n = 6 gives the blocks two strips each (both LDS stages, both chunk-parity
    assignments); with accumulation into an existing gradient."""
    g = torch.Generator(device="cuda").manual_seed(n)
    xs = torch.randn(n, 115, 115, 16, device="cuda", generator=g).bfloat16()
    dy = torch.randn(n, 112, 112, 64, device="cuda", generator=g).bfloat16()
    base = torch.randn(64, 4, 4, 16, device="cuda", generator=g)
    ref = torch.nn.grad.conv2d_weight(xs.float().permute(0, 3, 1, 2), (64, 16, 4, 4),
                                      dy.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    if acc:
        ref = ref + base
    outs = []
    try:
        for stem in (1, 0):
            native._K.wgrad_set_stem(stem)
            out = base.clone().contiguous() if acc else None
            outs.append(native.conv2d_wgrad(xs, dy, (64, 4, 4, 16), 1, 0, out=out))
    finally:
        native._K.wgrad_set_stem(1)
    for o in outs:
        assert float((o - ref).norm() / ref.norm()) < 1e-5, float((o - ref).norm() / ref.norm())
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n", [2, 5])
def test_stem_wgrad_forms_pool_bn_backward_on_load_bit_identical(n):
    """The stem's BN + ReLU + max-pool backward apply folded into the stem weight gradient
    (conv_wgrad_stem_kernel<true>: d(stem conv output) formed per strip from the pooled gradient,
    argmax bytes and BN input, never stored) against the apply pass + the strip wgrad kernel:
    the conv weight gradient and BN gamma / beta gradients bit for bit; n = 5 leaves the last
    blocks' second strip past the batch.  The lazy record must be consumed (the apply pass not
    run) on the fused arm."""
    torch.manual_seed(0)
    m = resnet50().cuda()
    x = torch.randn(n, 224, 224, 3, device="cuda").bfloat16()
    dy = torch.randn(n, 56, 56, 64, device="cuda").bfloat16()
    calls = {"apply": 0, "dz": 0}
    o_apply, o_dz = native._K.pool_bn_bwd_apply, native._K.conv_wgrad_stem_dz

    def c_apply(*a):
        calls["apply"] += 1
        return o_apply(*a)

    def c_dz(*a):
        calls["dz"] += 1
        return o_dz(*a)

    grads = []
    try:
        native._K.pool_bn_bwd_apply, native._K.conv_wgrad_stem_dz = c_apply, c_dz
        for fuse in (False, True):
            native._FUSE_STEM_WGRAD = fuse
            stem = m.stem
            for p in stem.parameters():
                p.grad = None
            y = stem(x, pool=True)
            y.backward(dy)
            torch.cuda.synchronize()
            grads.append([p.grad.clone() for p in stem.parameters()])
            assert calls == ({"apply": 1, "dz": 0} if not fuse else {"apply": 1, "dz": 1}), calls
    finally:
        native._FUSE_STEM_WGRAD = True
        native._K.pool_bn_bwd_apply, native._K.conv_wgrad_stem_dz = o_apply, o_dz
    assert len(grads[0]) == len(grads[1]) >= 3
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_lazy_x3_never_stores_stage0_c3_output_bit_identical():
    """the stage-0 identity blocks' c3 output (x3, [M, 256]) is never written --
    the c3 GEMM runs NOST (statistics only), the residual BN's apply recomputes x3 in a stream
    GEMM (gemm_stream_apply), the next conv's BN-sum epilogue recomputes it (RC) and the fused c3
    backward recomputes it (LZ stage 0).  Blocks s0b1 -> s0b2 -> s1b0 (a stride-2 projection reads
    s0b2's output too) against the stored-x3 path: output, input gradient and every parameter
    gradient bit for bit."""
    torch.manual_seed(0)
    m = resnet50().cuda()
    blks = [m.blocks[1], m.blocks[2], m.blocks[3]]
    x = torch.randn(2, 16, 16, 256, device="cuda").bfloat16()
    calls = {"apply": 0, "nost": 0, "rc": 0}
    o_apply, o_pre, o_bnb = (native._K.gemm_stream_apply, native._K.gemm_stream_pre,
                             native._K.gemm_stream_bnb)

    def s_apply(*a):
        calls["apply"] += 1
        return o_apply(*a)

    def s_pre(*a):
        calls["nost"] += int(len(a) > 11 and a[11] == 1)
        return o_pre(*a)

    def s_bnb(*a):
        calls["rc"] += int(len(a) > 21 and a[21] != 0)
        return o_bnb(*a)
    out = {}
    prev = native._LAZY_X3
    g = None
    try:
        native._K.gemm_stream_apply = s_apply
        native._K.gemm_stream_pre = s_pre
        native._K.gemm_stream_bnb = s_bnb
        for lz in (True, False):
            native._LAZY_X3 = lz
            bs = [copy.deepcopy(b) for b in blks]
            assert bs[0].lazy_c3 and not bs[1].lazy_c3      # the network's choice ...
            bs[1].lazy_c3 = True      # ... forced here: the projection's dgrad recomputes x3 too
            xi = x.clone().requires_grad_(True)
            y = xi
            for b in bs:
                y = b(y)
            if g is None:
                g = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(
                    device="cuda", dtype=y.dtype)
            y.backward(g)
            torch.cuda.synchronize()
            out[lz] = (y.detach().float(), xi.grad.float(),
                       [p.grad.float() for b in bs for p in b.parameters()])
            if lz:
                seen = dict(calls)
    finally:
        native._K.gemm_stream_apply, native._K.gemm_stream_pre = o_apply, o_pre
        native._K.gemm_stream_bnb = o_bnb
        native._LAZY_X3 = prev
    # two identity blocks at stage 0: two no-store c3 GEMMs, two recomputing applies, and the
    # s0b2 c1 data gradient's BN-sum epilogue recomputes s0b1's x3
    assert seen["nost"] == 2 and seen["apply"] == 2 and seen["rc"] >= 1, seen
    assert calls == seen, "the stored-x3 path must not take the lazy kernels"
    (ya, dxa, ga), (yb, dxb, gb) = out[True], out[False]
    assert torch.equal(ya, yb)
    assert torch.equal(dxa, dxb)
    for i, (a, b) in enumerate(zip(ga, gb)):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("C,W,K", [(64, 56, 64), (128, 28, 128)])
def test_halo_conv_bn_relu_on_load_bit_identical(C, W, K):
    """VERDICT r4 #5 (halo families): the 3x3 conv reads the BatchNorm INPUT and applies
    y = bf16(max(x sc + sh, 0)) to its LDS patch (padding stays zero), writing y for the rows it
    owns -- y, the conv output and its BN statistics slab equal the apply pass + conv bit for
    bit."""
    torch.manual_seed(0)
    x = (torch.randn(3, W, W, C, device="cuda") * 2 + 0.3).bfloat16()
    w = (torch.randn(K, 3, 3, C, device="cuda") / (9 * C) ** 0.5).bfloat16()
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda") * 0.5
    M = x.numel() // C
    y_ref = torch.empty_like(x)
    native._K.bn_apply(x.data_ptr(), 0, y_ref.data_ptr(), sc.data_ptr(), sh.data_ptr(), M, C, 1,
                       torch.cuda.current_stream().cuda_stream, 0)
    taps = [(r - 1, s - 1) for r in range(3) for s in range(3)]
    geom = native._fwd_geom(x.shape, K, taps, W, W, 1, 1, W, W)
    assert native._K.conv_bnl_ok(geom, [t[0] for t in taps], [t[1] for t in taps])
    G = native._K.conv_tile_rows(geom, [t[0] for t in taps], [t[1] for t in taps])
    outs = []
    for bnl in (False, True):
        part = torch.full((native._K.bn_workspace_floats_g(G, K),), float("nan"), device="cuda")
        if bnl:
            y = torch.full_like(x, float("nan"))
            y._dtf_bnl = native._BnDeferred(x, sc, sh, y)
        else:
            y = y_ref
        z = native.conv2d_forward(y, w, 1, 1, stats=part)
        torch.cuda.synchronize()
        if bnl:
            assert y._dtf_bnl.done
        outs.append((y.clone(), z, part[:G * 2 * K]))
    assert torch.equal(outs[1][0], y_ref)
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("bi,shape", [(1, (2, 56, 56, 256)), (4, (2, 28, 28, 512))])
def test_bottleneck_c2_bn_on_load_bit_identical(bi, shape):
    """c1's BN + ReLU applied on the c2 halo conv's input load (ops.batch_norm(defer=True)):
    an identity block's output, input gradient and every parameter gradient equal the apply
    pass + conv path bit for bit, and the BN-on-load launch really ran."""
    torch.manual_seed(0)
    m = resnet50().cuda()
    blk = m.blocks[bi]
    x = torch.randn(*shape, device="cuda").bfloat16()
    calls = {"bnl": 0}
    orig = native._K.conv_igemm

    def spy(*a, **k):
        calls["bnl"] += int(len(a) > 16 and a[16] != 0)
        return orig(*a, **k)
    out, g = {}, None
    prev = native._BN_ON_LOAD
    try:
        native._K.conv_igemm = spy
        for on in (True, False):
            native._BN_ON_LOAD = on
            b = copy.deepcopy(blk)
            assert b.c2_bn_on_load
            xi = x.clone().requires_grad_(True)
            y = b(xi)
            if g is None:
                g = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(
                    device="cuda", dtype=y.dtype)
            y.backward(g)
            torch.cuda.synchronize()
            out[on] = (y.detach().float(), xi.grad.float(),
                       [p.grad.float() for p in b.parameters()])
            if on:
                seen = calls["bnl"]
    finally:
        native._K.conv_igemm = orig
        native._BN_ON_LOAD = prev
    assert seen == 1 and calls["bnl"] == 1
    (ya, dxa, ga), (yb, dxb, gb) = out[True], out[False]
    assert torch.equal(ya, yb)
    assert torch.equal(dxa, dxb)
    for i, (a, b) in enumerate(zip(ga, gb)):
        assert torch.equal(a, b), i


def test_training_step_frees_its_activations_without_the_cycle_collector():
    """A default training step (BN on load, lazy x3, fused BN backward) leaves no reference
    cycle holding activations: with the cyclic collector disabled, allocated memory does not
    grow over the second, third and fourth steps (the first builds per-step caches; later steps
    move by a few hundred KB as those alternate, while a leaked set of c1 outputs is ~11 MB per
    step at this batch).  (A y <-> deferred-BN-record cycle once
    kept every step's c1 outputs alive until a full collection: +2.9 GB of peak per step at
    b1984.)"""
    import gc
    torch.manual_seed(0)
    m = resnet50().cuda()
    x = torch.randn(8, 224, 224, 3, device="cuda").bfloat16()
    lab = torch.randint(0, 1000, (8,), device="cuda")
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        after = []
        for _ in range(4):
            loss = torch.nn.functional.cross_entropy(m(x).float(), lab)
            loss.backward()
            del loss
            for p in m.parameters():
                p.grad = None
            torch.cuda.synchronize()
            after.append(torch.cuda.memory_allocated())
    finally:
        if was:
            gc.enable()
    assert max(after[1:]) - min(after[1:]) < 2 * 2**20, after


def test_no_record_outlives_its_step():
    """the default ResNet-50 training step (BN on load, lazy x3, fused BN
    backward, masked residual gradients) through the optimizer, with the cyclic collector OFF:
    after every step no deferred-work record is alive (ops/records.py end_step), and the peak
    memory of step 25 equals step 2's (a record kept past its step would hold a step's
    activations: +2.9 GB per step at b1984 in round 5)."""
    import gc

    from distributedtensorflow_amd.ops import records
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import MirroredStrategy
    torch.manual_seed(0)
    with MirroredStrategy().scope():
        m = resnet50()
        opt = MomentumOptimizer(0.01, momentum=0.9, weight_decay=1e-4)
        opt.build(list(m.parameters()))
    # 224 x 224: the halo 3x3 convs (BN on load) and the stage-0 lazy x3 take their real paths
    x = torch.randn(8, 224, 224, 3, device="cuda").bfloat16()
    lab = torch.randint(0, 1000, (8,), device="cuda")
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    peaks, made = [], []
    try:
        for _ in range(25):
            torch.cuda.reset_peak_memory_stats()
            loss = ops.sparse_softmax_cross_entropy(m(x), lab)
            made.append(records.live_count())
            opt.minimize(loss)
            del loss
            torch.cuda.synchronize()
            assert records.live_count() == 0
            peaks.append(torch.cuda.max_memory_allocated())
    finally:
        if was:
            gc.enable()
    assert min(made) > 0, made                       # the step does create records
    # one leaked step's records would hold its c1 outputs and more (~11 MB per step at this
    # batch: > 250 MB over 23 steps), a GROWTH; without one the peak only jitters by a few MB
    # (per-step caches alternating, and the side-stream weight-gradient launches interleaving
    # their allocations with the main stream's differently from step to step: 1.2-3 MB on
    # fresh boxes)
    early, late = max(peaks[1:6]), max(peaks[-5:])
    assert late - early < 4 * 2**20, peaks
    assert max(peaks[1:]) - min(peaks[1:]) < 8 * 2**20, peaks
    assert abs(peaks[24] - peaks[1]) < 4 * 2**20, peaks
