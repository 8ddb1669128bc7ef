#!/bin/bash
# VGPR-staged ping-pong (variant 16) vs the LDS-DMA ping-pong (8) and hipBLASLt; bit-identity
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
timeout -k 10 120 python -u - <<'PY' || exit 1
import torch
from distributedtensorflow_amd.ops import native
K = native.kernels()
g = torch.Generator(device="cuda").manual_seed(0)
for (M, N, Kd) in [(4096, 768, 768), (1000, 2304, 768), (513, 264, 200), (65536, 3072, 768)]:
    A = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
    B = (torch.randn(N, Kd, device="cuda", generator=g) / Kd ** 0.5).bfloat16()
    outs = []
    for v in (8, 16):
        K.gemm_set_variant(v)
        outs.append(native.gemm_nt(A, B))
    K.gemm_set_variant(-1)
    print("bitident", M, N, Kd, torch.equal(outs[0], outs[1]), flush=True)
PY
timeout -k 10 300 python -u tools/gemm_bench.py --variants 8,16 --dbg 0,1 \
  --only bert_qkv_fwd,bert_attnout_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_qkv_dgrad,bert_ffn1_dgrad,bert_ffn2_dgrad,bert_mlm_logits,sq4096,sq8192 \
  > gpurun_out/gemm_stg.jsonl 2> gpurun_out/gemm_stg.err
