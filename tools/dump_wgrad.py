"""Dump inputs/outputs of the wgrad kernel for offline analysis (gpurun_out/wgrad_dump_*.npz)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from distributedtensorflow_amd.ops import native  # noqa: E402

K_ = native.kernels()


def run(tag, N, H, C, K, tr, prefill):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    g = torch.randn(N, H, H, K, device="cuda").to(torch.bfloat16)
    outs = []
    for rep in range(3):
        dW = torch.full((K, C), prefill, device="cuda")
        geom = [N, H, H, C, H, H, 1, 1, K, C]
        K_.conv_wgrad(x.data_ptr(), g.data_ptr(), dW.data_ptr(), 0, geom, [0], [0], 1,
                      torch.cuda.current_stream().cuda_stream, tr)
        torch.cuda.synchronize()
        outs.append(dW.cpu().numpy())
    np.savez(f"gpurun_out/wgrad_dump_{tag}.npz", x=x.float().cpu().numpy(),
             g=g.float().cpu().numpy(), out=np.stack(outs))
    ref = (g.double().reshape(-1, K).T @ x.double().reshape(-1, C)).cpu().numpy()
    for i, o in enumerate(outs):
        print(tag, "rep", i, "rel", np.linalg.norm(o - ref) / np.linalg.norm(ref), flush=True)


if __name__ == "__main__":
    run("h8_tr0", 1, 8, 64, 64, 0, float("nan"))
    run("h8_tr1", 1, 8, 64, 64, 1, float("nan"))
    run("h16_tr1", 1, 16, 64, 64, 1, float("nan"))
