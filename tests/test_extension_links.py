"""The in-tree HIP extension must load (every exported launcher resolved) even on a CPU-only
host: an unresolved symbol would otherwise only surface on the GPU box."""
import glob
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["_dtf_hip", "_dtf_native"])
def test_extension_imports(name):
    if not glob.glob(os.path.join(ROOT, "distributedtensorflow_amd", "_lib", name + "*.so")):
        pytest.skip(f"{name} not built")
    import importlib
    mod = importlib.import_module(f"distributedtensorflow_amd._lib.{name}")
    assert mod is not None


def _hip_ext():
    if not glob.glob(os.path.join(ROOT, "distributedtensorflow_amd", "_lib", "_dtf_hip*.so")):
        pytest.skip("_dtf_hip not built")
    import importlib
    return importlib.import_module("distributedtensorflow_amd._lib._dtf_hip")


def test_wgrad_strip_routes_take_exactly_their_layers():
    """Host-side routing of the strip weight-gradient kernels (no GPU needed): the stem's
    space-to-depth 4x4 VALID conv (115x115x16 -> 112x112x64) and the stage-1 3x3 (56x56x64 -> 64)
    get one fp32 slab per block (at most 256 blocks, fewer when there are fewer strips); any other
    geometry -- shifted taps, another channel count, a strided conv -- gets 0 (the tiled kernels)."""
    K = _hip_ext()
    stem_dh, stem_dw = [t // 4 for t in range(16)], [t % 4 for t in range(16)]
    # geom: N, H, W, C, P, Q, sh, sw, Kout, ldw
    assert K.conv_wgrad_halo_splits([3, 115, 115, 16, 112, 112, 1, 1, 64, 256], stem_dh, stem_dw) == 168
    assert K.conv_wgrad_halo_splits([8, 115, 115, 16, 112, 112, 1, 1, 64, 256], stem_dh, stem_dw) == 256
    assert K.conv_wgrad_halo_splits([8, 115, 115, 16, 112, 112, 1, 1, 64, 256], stem_dh,
                                    [d + 1 for d in stem_dw]) == 0
    assert K.conv_wgrad_halo_splits([8, 115, 115, 8, 112, 112, 1, 1, 64, 128], stem_dh, stem_dw) == 0
    assert K.conv_wgrad_halo_splits([8, 115, 115, 16, 112, 112, 1, 1, 128, 256], stem_dh, stem_dw) == 0
    h_dh, h_dw = [t // 3 - 1 for t in range(9)], [t % 3 - 1 for t in range(9)]
    assert K.conv_wgrad_halo_splits([8, 56, 56, 64, 56, 56, 1, 1, 64, 576], h_dh, h_dw) == 112
    assert K.conv_wgrad_halo_splits([64, 56, 56, 64, 56, 56, 1, 1, 64, 576], h_dh, h_dw) == 256
    assert K.conv_wgrad_halo_splits([8, 56, 56, 64, 28, 28, 2, 2, 64, 576], h_dh, h_dw) == 0


def test_gemm_conv_batch_parts_are_whole_tiles_under_one_descriptor():
    """Batch split of a persistent-GEMM conv whose input passes one 32-bit buffer descriptor
    (the b1984 stage-1 projection: 56x56x256 bf16 = 3.2 GB): each part is a multiple of the
    images that fill whole 256-row tiles (so the BN statistics slab rows continue across parts)
    and its input stays under 2^31 bytes; no split below that; -1 when no such part exists."""
    K = _hip_ext()
    assert K.gemm_conv_part_images(64, 56, 56, 256, 28, 28) == 0          # 103 MB: no split
    per = K.gemm_conv_part_images(1984, 56, 56, 256, 28, 28)
    assert per == 1328                                                   # 1328 + 656 images
    img = 56 * 56 * 256 * 2
    assert per * img < 2 ** 31 and (per * 28 * 28) % 256 == 0
    assert K.gemm_conv_part_images(1984, 56, 56, 256, 56, 56) > 0         # P Q = 3136: unit 16
    assert K.gemm_conv_part_images(4096, 56, 56, 256, 28, 28) == -1      # N past the packing
