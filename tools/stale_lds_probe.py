"""Probe: does the wgrad kernel's result depend on what ran before it (stale LDS / state)?"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from distributedtensorflow_amd.ops import native, reference  # noqa: E402

K_ = native.kernels()
torch.manual_seed(0)
N, H, C, K = 1, 8, 64, 64
x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
g = torch.randn(N, H, H, K, device="cuda").to(torch.bfloat16)
ref = (g.double().reshape(-1, K).T @ x.double().reshape(-1, C)).cpu().numpy()


def mine(tr=1):
    dW = torch.full((K, C), float("nan"), device="cuda")
    K_.conv_wgrad(x.data_ptr(), g.data_ptr(), dW.data_ptr(), 0, [N, H, H, C, H, H, 1, 1, K, C],
                  [0], [0], 1, torch.cuda.current_stream().cuda_stream, tr)
    torch.cuda.synchronize()
    o = dW.cpu().numpy()
    return np.linalg.norm(o - ref) / np.linalg.norm(ref), o


def miopen():
    w = torch.randn(K, 3, 3, C, device="cuda").requires_grad_(True)
    xx = torch.randn(2, 28, 28, C, device="cuda")
    y = reference.conv2d(xx, w, 1, 1)
    y.backward(torch.randn_like(y))
    torch.cuda.synchronize()


def fill_lds_garbage():
    # a big matmul uses LDS heavily
    a = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    (a @ a).sum().item()


for label, pre in [("none", None), ("none", None), ("miopen", miopen), ("none", None),
                   ("gemm", fill_lds_garbage), ("none", None), ("miopen", miopen)]:
    if pre:
        pre()
    r, o = mine(1)
    r0, _ = mine(0)
    print(f"after {label:7s}: tr=1 rel={r:.3g}  tr=0 rel={r0:.3g}", flush=True)
    if r > 1e-4:
        Xp = np.linalg.solve(g.double().reshape(-1, K).cpu().numpy().T, o)
        diff = np.abs(Xp - x.double().reshape(-1, C).cpu().numpy()) > 1e-2
        rows, cols = np.where(diff)
        print("    wrong pixels", np.unique(rows)[:16], "channels", np.unique(cols)[:64], flush=True)

print("--- debug-style data ---", flush=True)
for trial in range(3):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    w = torch.randn(K, 1, 1, C, device="cuda")
    g = torch.randn(N, H, H, K, device="cuda").to(torch.bfloat16)
    ref = (g.double().reshape(-1, K).T @ x.double().reshape(-1, C)).cpu().numpy()
    r, o = mine(1)
    print(f"trial {trial}: rel={r:.3g}", flush=True)
    if r > 1e-4:
        Xp = np.linalg.solve(g.double().reshape(-1, K).cpu().numpy().T, o)
        diff = np.abs(Xp - x.double().reshape(-1, C).cpu().numpy()) > 1e-2
        rows, cols = np.where(diff)
        print("    wrong pixels", np.unique(rows)[:16], "channels", np.unique(cols)[:64], flush=True)
    # now exactly the debug path: ws allocated, zeros dW
    dW = torch.zeros(K, C, device="cuda")
    ws = torch.empty(K * C, device="cuda")
    K_.conv_wgrad(x.data_ptr(), g.contiguous().data_ptr(), dW.data_ptr(), ws.data_ptr(),
                  [N, H, H, C, H, H, 1, 1, K, C], [0], [0], 1,
                  torch.cuda.current_stream().cuda_stream, 1)
    torch.cuda.synchronize()
    o2 = dW.cpu().numpy()
    print(f"   debug-path rel={np.linalg.norm(o2 - ref) / np.linalg.norm(ref):.3g}", flush=True)
