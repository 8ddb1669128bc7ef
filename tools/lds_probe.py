import sys
import torch
sys.path.insert(0, ".")
from distributedtensorflow_amd.ops import native
K = native.kernels()
print("max shared per block attr:", K.max_dynamic_lds(0), flush=True)
for kb in (32, 60, 64, 66, 72, 80, 96, 128, 160):
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    try:
        K.lds_probe(kb * 1024, 2048, err.data_ptr(), 20000, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        print(f"{kb:4d} KiB: errors={int(err.item())}", flush=True)
    except Exception as e:
        print(f"{kb:4d} KiB: launch failed: {e}", flush=True)
