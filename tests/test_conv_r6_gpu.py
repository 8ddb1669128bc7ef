"""Round-6 conv routes: the phase classes of a strided 3x3 data gradient in ONE grouped launch
(csrc/kernels/conv.hip conv_igemm_grouped_kernel, ops/native.py conv2d_dgrad): bit-identical to
the one-launch-per-class path (same kernel body, same per-output MFMA chain, same BN-sum slab
rows), and the data gradient against fp32 PyTorch; the strided 1x1 forward (projection
shortcut) on the persistent GEMM, including inputs past one 32-bit buffer descriptor."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from distributedtensorflow_amd.ops import native  # noqa: E402


def _spy():
    seen = []
    orig = native._K.conv_igemm_grouped

    def spy(*a):
        ok = orig(*a)
        seen.append(ok)
        return ok
    return orig, spy, seen


def _both(fn):
    """fn() with the grouped launch on, then off; asserts the grouped launch ran in the first."""
    orig, spy, seen = _spy()
    prev = native._DGRAD_GROUPED
    outs = []
    try:
        for grouped in (True, False):
            native._DGRAD_GROUPED = grouped
            native._K.conv_igemm_grouped = spy
            outs.append(fn())
            native._K.conv_igemm_grouped = orig
            if grouped:
                assert seen and all(seen), "the grouped launch did not run"
    finally:
        native._DGRAD_GROUPED = prev
        native._K.conv_igemm_grouped = orig
    return outs


@pytest.mark.parametrize("N,H,C,K,acc", [(2, 56, 128, 128, False), (3, 28, 64, 64, False),
                                         (2, 56, 128, 128, True), (2, 14, 96, 160, False)])
def test_grouped_strided_dgrad_bit_identical_and_vs_fp32(N, H, C, K, acc):
    torch.manual_seed(0)
    dy = torch.randn(N, H // 2, H // 2, K, device="cuda").bfloat16()
    w = (torch.randn(K, 3, 3, C, device="cuda") / (9 * C) ** 0.5).bfloat16()
    base = torch.randn(N, H, H, C, device="cuda").bfloat16()

    def run():
        out = base.clone() if acc else None
        return native.conv2d_dgrad(dy, w, (N, H, H, C), 2, 1, out=out).clone()
    g, s = _both(run)
    assert torch.equal(g, s)
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2),
                                     dy.float().permute(0, 3, 1, 2), stride=2, padding=1)
    ref = ref.permute(0, 2, 3, 1)
    if acc:
        ref = ref + base.float()
    rel = float((g.float() - ref).norm() / ref.norm())
    assert rel < 1e-2, rel


def test_grouped_dgrad_leaves_the_bn_sum_launches_split():
    """With the fused BN-backward sums the classes stay one launch each (grouped, that epilogue
    measured slower): the grouped entry refuses such a launch and launches nothing."""
    dy = torch.zeros(1, 4, 4, 32, device="cuda").bfloat16()
    dx = torch.zeros(1, 8, 8, 32, device="cuda").bfloat16()
    w = torch.zeros(32, 32, device="cuda").bfloat16()
    geom = native._fwd_geom((1, 4, 4, 32), 32, [(0, 0)], 4, 4, 1, 1, 8, 8, 2, 2, 0, 0, False)
    x = torch.zeros(1, 8, 8, 32, device="cuda").bfloat16()
    part = torch.zeros(1024, device="cuda")
    st = torch.ones(32, device="cuda")
    bnb = [x.data_ptr(), st.data_ptr(), st.data_ptr(), st.data_ptr(), st.data_ptr(), 0,
           part.data_ptr(), 2]
    assert not native._K.conv_igemm_grouped(
        dy.data_ptr(), dx.data_ptr(), geom, [w.data_ptr()] * 2, [0, 1], [0, 0], [32, 32],
        [[0], [0]], [[0], [0]], torch.cuda.current_stream().cuda_stream, bnb, [0, 1])


def _proj_stats(x, w, gemm):
    """conv2d_forward of the 1x1 stride-2 projection with its BN-statistics slab, on the GEMM
    route (gemm=True, the default) or the register kernel (conv_set_gemm(0))."""
    N, H, _, C = x.shape
    K = w.shape[0]
    P = H // 2
    geom = [N, H, H, C, P, P, 2, 2, K, C, P, P, 1, 1, 0, 0, 0]
    try:
        native._K.conv_set_gemm(1 if gemm else 0)
        rows = native._K.conv_tile_rows(geom, [0], [0], 0)
        ws = torch.zeros(native._K.bn_workspace_floats_g(rows, K), device="cuda")
        y = native.conv2d_forward(x, w, 2, 0, stats=ws)
        torch.cuda.synchronize()
    finally:
        native._K.conv_set_gemm(1)
    return y, ws[: rows * 2 * K].view(rows, 2, K).sum(0), rows


@pytest.mark.parametrize("N,H,C,K", [(4, 56, 256, 512), (3, 28, 512, 1024), (2, 14, 1024, 2048)])
def test_projection_shortcut_on_the_persistent_gemm(N, H, C, K):
    """The strided 1x1 forward (projection shortcut) on the persistent GEMM: output within one
    bf16 rounding of the register kernel's (the same k order per output), BN sums to fp32
    summation noise, and the output and its sums against fp32 PyTorch."""
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(K, 1, 1, C, device="cuda") / C ** 0.5).bfloat16()
    yg, sg, rg = _proj_stats(x, w, True)
    yr, sr, rr = _proj_stats(x, w, False)
    assert rg == (N * (H // 2) ** 2 + 255) // 256           # the GEMM route's slab rows
    print("bit-identical to the register kernel:", torch.equal(yg, yr))
    torch.testing.assert_close(yg.float(), yr.float(), rtol=1e-2, atol=1e-2)
    assert float((yg.float() - yr.float()).abs().max()) <= float(yr.float().abs().max()) * 2 ** -7
    torch.testing.assert_close(sg, sr, rtol=1e-4, atol=1e-1)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2),
                                     w.float().permute(0, 3, 1, 2), stride=2).permute(0, 2, 3, 1)
    assert float((yg.float() - ref).norm() / ref.norm()) < 1e-2
    yf = yg.float()
    torch.testing.assert_close(sg[0], yf.sum((0, 1, 2)), rtol=1e-3, atol=1.0)
    torch.testing.assert_close(sg[1], (yf * yf).sum((0, 1, 2)), rtol=1e-3, atol=1.0)


def test_projection_shortcut_input_past_2gib_runs_in_batch_parts():
    """A 2.3 GB projection input (56 x 56 x 256, 1408 images: past one 32-bit buffer descriptor)
    runs on the persistent GEMM in batch parts of whole 256-row tiles; the output equals the
    register kernel's (which rebases its descriptors per tile) to one bf16 rounding and the
    statistics slab rows continue across the parts."""
    N, H, C, K = 1408, 56, 256, 512
    assert native._K.gemm_conv_part_images(N, H, H, C, H // 2, H // 2) > 0
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(N, H, H, C, device="cuda", generator=g).bfloat16()
    w = (torch.randn(K, 1, 1, C, device="cuda", generator=g) / C ** 0.5).bfloat16()
    yg, sg, rg = _proj_stats(x, w, True)
    yr, sr, rr = _proj_stats(x, w, False)
    assert rg == N * (H // 2) ** 2 // 256
    assert float((yg.float() - yr.float()).abs().max()) <= float(yr.float().abs().max()) * 2 ** -7
    torch.testing.assert_close(sg, sr, rtol=1e-4, atol=2.0)
    # the last part's images: against fp32 PyTorch
    ref = torch.nn.functional.conv2d(x[-4:].float().permute(0, 3, 1, 2),
                                     w.float().permute(0, 3, 1, 2), stride=2).permute(0, 2, 3, 1)
    assert float((yg[-4:].float() - ref).norm() / ref.norm()) < 1e-2


@pytest.mark.parametrize("N,H,C,K,R,acc", [(2, 28, 256, 256, 3, False), (3, 14, 512, 512, 3, False),
                                           (2, 56, 256, 512, 1, True), (3, 28, 512, 1024, 1, False),
                                           (5, 14, 1024, 2048, 1, True)])
def test_strided_dgrad_phases_on_the_persistent_gemm(N, H, C, K, R, acc):
    """Stride-2 data gradients whose phase classes run on the GEMM (output channels >= 256: the
    3x3 of stages 3-4, every projection shortcut) now take the persistent kernel, output rows
    addressed through its per-wave LDS row table: bit-identical to the round-5 ping-pong kernel,
    with and without the accumulate (Cin) epilogue, and against fp32 PyTorch."""
    torch.manual_seed(0)
    dy = torch.randn(N, H // 2, H // 2, K, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5).bfloat16()
    base = torch.randn(N, H, H, C, device="cuda").bfloat16()
    pad = R // 2
    outs = []
    try:
        for on in (1, 0):
            native._K.gemm_set_pp2_strided(on)
            out = base.clone() if acc else None
            outs.append(native.conv2d_dgrad(dy, w, (N, H, H, C), 2, pad, out=out).clone())
            torch.cuda.synchronize()
    finally:
        native._K.gemm_set_pp2_strided(1)
    assert torch.equal(outs[0], outs[1])
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2),
                                     dy.float().permute(0, 3, 1, 2), stride=2,
                                     padding=pad).permute(0, 2, 3, 1)
    if acc:
        ref = ref + base.float()
    rel = float((outs[0].float() - ref).norm() / ref.norm())
    assert rel < 1e-2, rel
