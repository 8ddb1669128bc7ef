"""ResNet-50 v1.5 (stride on the 3x3 conv), NHWC / bf16 compute, fp32 master weights.

North-star model (BASELINE.json configs 2-4).  Not present in the
reference, which only trains MNIST models (``run_mnist_distributed.py:46-70``); the layer
naming follows tf.keras.applications.ResNet50 so checkpoints carry familiar keys
(``conv2_block1_1_conv/kernel``, ``conv2_block1_1_bn/gamma`` ...).

Every conv is bias-free and followed by a fused BatchNorm(+residual)(+ReLU) op, so a
bottleneck block is 3-4 conv launches + 3-4 fused BN launches forward.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .. import ops
from .layers import BatchNormalization, Conv2D, Dense, Layer, name_scope


class ConvBN(nn.Module):
    def __init__(self, cin, cout, k, stride, name, bn_momentum, bn_eps, zero_gamma=False):
        super().__init__()
        self.conv = Conv2D(cin, cout, k, strides=stride, padding=(k - 1) // 2, use_bias=False,
                           name=f"{name}_conv", init="he")
        self.bn = BatchNormalization(cout, bn_momentum, bn_eps, name=f"{name}_bn",
                                     gamma_init=0.0 if zero_gamma else 1.0)

    def forward(self, x, relu=True, residual=None, residual_to_conv=False, grad_share=None,
                defer_bn=False):
        """``defer_bn``: the output only feeds a 3x3 conv that may apply this BN + ReLU on its
        input load (ops.batch_norm(defer=True))."""
        y = ops.conv2d(x, self.conv.kernel, self.conv.strides, self.conv.padding,
                       bn_stats=self.bn.training, grad_share=grad_share)
        return self.bn(y, relu=relu, residual=residual, residual_to_conv=residual_to_conv,
                       defer=defer_bn)


class StemConvBN(ConvBN):
    """7x7/2 stem.  On the native path the conv runs as a 4x4 stride-1 conv on the
    space-to-depth image (ops.reference.space_to_depth_operands); the variable stays the TF
    [7,7,3,64] kernel (checkpoint key conv1_conv/kernel) and its gradient flows back through the
    rewrite."""

    def forward(self, x, relu=True, residual=None, residual_to_conv=False, grad_share=None,
                pool=False):
        """``pool``: also apply the 3x3/2 max-pool (fused with the BN + ReLU on the native
        path, so the 112x112x64 BN output is never stored)."""
        if not (ops._use_native(x) and self.conv.strides in (2, (2, 2)) and S2D_STEM):
            y = super().forward(x, relu, residual, residual_to_conv, grad_share)
            return ops.max_pool2d(y, 3, 2, 1) if pool else y
        from ..ops import reference
        xs, ws = reference.space_to_depth_operands(x, self.conv.kernel, 2, self.conv.padding,
                                                   want_x=x.requires_grad)
        if xs is None:   # the image: one-pass HIP layout kernel instead of pad + permute copies
            from ..ops import native
            kh, kw = self.conv.kernel.shape[1:3]
            xs = native.space_to_depth_input(x, 2, self.conv.padding, kh, kw)
        y = ops.conv2d(xs, ws, 1, 0, bn_stats=self.bn.training)
        if pool and relu and FUSE_STEM_POOL:
            bn = self.bn
            return ops.batch_norm_relu_max_pool(y, bn.gamma, bn.beta, bn.moving_mean,
                                                bn.moving_variance, bn.training, bn.momentum,
                                                bn.epsilon, 3, 2, 1)
        y = self.bn(y, relu=relu)
        return ops.max_pool2d(y, 3, 2, 1) if pool else y


S2D_STEM = True
FUSE_STEM_POOL = True
# projection blocks: shortcut BN fused into the block-output BN (ops.batch_norm_add_batch_norm)
FUSE_PROJ_BN = os.environ.get("DTF_FUSE_PROJ_BN", "1") == "1"
# bottleneck c2's BN + ReLU inside c3's GEMM (ops.batch_norm_relu_conv1x1; falls back to the two
# ops off the streaming route)
FUSE_BN_CONV = os.environ.get("DTF_FUSE_BN_CONV", "1") == "1"
# c1's BatchNorm + ReLU applied on the c2 3x3 conv's input load (ops.batch_norm(defer=True): the
# halo kernels normalise their patch in LDS and write the BN output once; other c2 shapes fall
# back to the apply pass); A/B knob, see also ops/native.py DTF_BN_ON_LOAD
BN_ON_LOAD = os.environ.get("DTF_C2_BN_ON_LOAD", "1") == "1"


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride, name, bn_momentum, bn_eps, zero_gamma=False):
        super().__init__()
        cout = width * self.expansion
        self.has_proj = stride != 1 or cin != cout
        if self.has_proj:
            self.proj = ConvBN(cin, cout, 1, stride, f"{name}_0", bn_momentum, bn_eps)
        self.c1 = ConvBN(cin, width, 1, 1, f"{name}_1", bn_momentum, bn_eps)
        self.c2 = ConvBN(width, width, 3, stride, f"{name}_2", bn_momentum, bn_eps)
        self.c3 = ConvBN(width, cout, 1, 1, f"{name}_3", bn_momentum, bn_eps, zero_gamma)
        # set by the network: this identity block's output feeds another identity block, whose
        # streamed c1 data gradient can recompute our c3 output (see _c2_c3)
        self.lazy_c3 = False
        # c1's BN + ReLU applied on c2's input load (the 3x3 halo kernels; stride-1 c2 only)
        self.c2_bn_on_load = BN_ON_LOAD and stride == 1

    def forward(self, x):
        # projection blocks: proj and c1 both read x -> one dgrad buffer, no autograd add
        share = ops.GradShare(2) if self.has_proj else None
        if self.has_proj and FUSE_PROJ_BN:
            # the shortcut's BN is applied inside the block-output BN (one pass forward, one
            # reduce + one apply pass backward for both).  (Building c1 before the projection,
            # so that c1's streamed dgrad completes d(x), measured 0.7 % slower:
            # profiles/measurements/r5_c1_last_backward_ab.jsonl)
            p, b = self.proj, self.proj.bn
            sc = ops.conv2d(x, p.conv.kernel, p.conv.strides, p.conv.padding,
                            bn_stats=b.training, grad_share=share)
            y = self._c2_c3(self.c1(x, grad_share=share, defer_bn=self.c2_bn_on_load))
            c, b3 = self.c3, self.c3.bn
            return ops.batch_norm_add_batch_norm(
                y, b3.gamma, b3.beta, b3.moving_mean, b3.moving_variance, sc, b.gamma, b.beta,
                b.moving_mean, b.moving_variance, b3.training, b3.momentum, b3.epsilon)
        y = self._c2_c3(self.c1(x, grad_share=share, defer_bn=self.c2_bn_on_load))
        sc = self.proj(x, relu=False, grad_share=share) if self.has_proj else x
        # identity shortcut: c1 (1x1, stride 1) also reads x, so its dgrad absorbs d(residual)
        return self.c3.bn(y, relu=True, residual=sc, residual_to_conv=not self.has_proj)

    def _c2_c3(self, y):
        """c2 conv -> BN + ReLU -> c3 conv (c3's output, before its BatchNorm).  Training: the
        BN + ReLU runs inside c3's GEMM (ops.batch_norm_relu_conv1x1) where that GEMM streams.
        Identity blocks followed by an identity block: c3's output only feeds the block-output
        BN, which recomputes it (``lazy_out``: never stored).  The last block of a stage feeds a
        stride-2 projection whose data gradient would have to recompute it once more (measured a
        net loss), so it stores it."""
        c2, c3 = self.c2, self.c3
        if c2.bn.training and FUSE_BN_CONV:
            y = ops.conv2d(y, c2.conv.kernel, c2.conv.strides, c2.conv.padding, bn_stats=True)
            b = c2.bn
            return ops.batch_norm_relu_conv1x1(y, b.gamma, b.beta, b.moving_mean,
                                               b.moving_variance, c3.conv.kernel, b.momentum,
                                               b.epsilon, lazy_out=self.lazy_c3)
        y = c2(y)
        return ops.conv2d(y, c3.conv.kernel, c3.conv.strides, c3.conv.padding,
                          bn_stats=c3.bn.training)


class ResNet(Layer):
    input_signature_shape = (None, 224, 224, 3)      # SavedModel serving input, NHWC

    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, in_channels=3,
                 bn_momentum=0.997, bn_eps=1e-5, zero_init_residual=False):
        super().__init__()
        with name_scope():
            self.stem = StemConvBN(in_channels, 64, 7, 2, "conv1", bn_momentum, bn_eps)
            blocks = []
            cin = 64
            for si, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
                for bi in range(n):
                    stride = 2 if (bi == 0 and si > 0) else 1
                    blocks.append(Bottleneck(cin, width, stride, f"conv{si + 2}_block{bi + 1}",
                                             bn_momentum, bn_eps, zero_init_residual))
                    cin = width * 4
            self.blocks = nn.ModuleList(blocks)
            for cur, nxt in zip(blocks, blocks[1:]):
                cur.lazy_c3 = not cur.has_proj and not nxt.has_proj
            self.fc = Dense(cin, num_classes, name="predictions")
            nn.init.normal_(self.fc.kernel.data, 0.0, 0.01)

    def forward(self, x):
        """x: [N, 224, 224, 3] NHWC (compute dtype) -> logits [N, classes] fp32."""
        y = self.stem(x, pool=True)
        for b in self.blocks:
            y = b(y)
        y = ops.global_avg_pool(y)
        return self.fc(y).float()


def resnet50(num_classes=1000, **kw) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes, **kw)


def resnet101(num_classes=1000, **kw) -> ResNet:
    return ResNet((3, 4, 23, 3), num_classes, **kw)


def resnet152(num_classes=1000, **kw) -> ResNet:
    return ResNet((3, 8, 36, 3), num_classes, **kw)


def num_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
