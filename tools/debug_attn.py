"""Per-part (dQ / dK / dV) error report of the native attention vs an fp64 reference."""
import torch

from distributedtensorflow_amd import ops
from distributedtensorflow_amd.ops import reference as R


def run(B, S, H, p, masked, seed=0):
    torch.manual_seed(seed)
    D = 64
    qkv32 = torch.randn(B * S, 3 * H * D)
    mask = torch.zeros(B, S)
    if masked:
        mask[0, S - 37:] = -10000.0
    dy = torch.randn(B * S, H * D).bfloat16()
    x = qkv32.cuda().bfloat16().requires_grad_(True)
    torch.manual_seed(11)
    y = ops.attention_qkv(x, mask.cuda() if masked else None, B, S, H, p, True)
    y.backward(dy.cuda())
    x_ = qkv32.bfloat16().double().requires_grad_(True)
    torch.manual_seed(11)
    y_ = R.attention_qkv(x_, mask.double() if masked else None, B, S, H, p, True)
    y_.backward(dy.double())
    dx, dx_ = x.grad.double().cpu(), x_.grad
    print(f"B{B} S{S} H{H} p{p} mask{masked}: y err {(y.double().cpu() - y_).abs().max():.4f}")
    for i, n in enumerate("QKV"):
        a = dx[:, i * H * D:(i + 1) * H * D]
        b = dx_[:, i * H * D:(i + 1) * H * D]
        err = (a - b).abs()
        print(f"   d{n}: max|ref| {b.abs().max():.3f}  max err {err.max():.4f}  "
              f"mean err {err.mean():.5f}  argmax {divmod(int(err.argmax()), H * D)}")


if __name__ == "__main__":
    for cfg in [(2, 128, 2, 0.0, True), (2, 128, 3, 0.1, True), (1, 512, 2, 0.0, False),
                (1, 64, 1, 0.1, False), (1, 64, 1, 0.0, False), (1, 128, 1, 0.0, False),
                (1, 128, 2, 0.0, False)]:
        run(*cfg)
