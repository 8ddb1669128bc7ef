"""One rank exercising parallel/comm.py RcclComm (launched by tests/test_rccl_comm_gpu.py under
torch.distributed.run).  Every collective is checked against the value it must produce, with
the operand written by a kernel on the compute stream right before the collective is issued and
read back on the compute stream right after ``wait()`` (the event ordering both ways)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from distributedtensorflow_amd.parallel import init_process_group_from_env
    from distributedtensorflow_amd.parallel.comm import RcclComm
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    init_process_group_from_env("nccl")
    W, r = dist.get_world_size(), dist.get_rank()
    c = RcclComm()
    out = {"version": c.version, "world": W}
    n = 1 << 22
    # all-reduce (sum) of a tensor the compute stream fills just before the issue
    x = torch.empty(n, device="cuda")
    x.fill_(float(r + 1))
    c.all_reduce(x).wait()
    out["all_reduce"] = bool(torch.all(x == W * (W + 1) / 2).item())
    # in-place reduce-scatter / all-gather on views of one flat buffer (the PS's usage)
    buf = torch.arange(W * 1024, device="cuda", dtype=torch.float32) * (r + 1)
    chunk = buf[r * 1024:(r + 1) * 1024]
    c.reduce_scatter(chunk, buf).wait()
    want = torch.arange(r * 1024, (r + 1) * 1024, device="cuda", dtype=torch.float32) * \
        (W * (W + 1) / 2)
    out["reduce_scatter"] = bool(torch.equal(chunk, want))
    chunk.add_(1.0)
    c.all_gather(buf, chunk).wait()
    out["all_gather"] = bool(torch.equal(buf[r * 1024:(r + 1) * 1024], want + 1.0))
    # bf16 broadcast and reduce
    b = torch.full((4096,), float(r), device="cuda", dtype=torch.bfloat16)
    c.broadcast(b, 0).wait()
    out["broadcast"] = bool(torch.all(b == 0).item())
    s = torch.ones(4096, device="cuda")
    c.reduce(s, 0).wait()
    out["reduce"] = bool(torch.all(s == W).item()) if r == 0 else True
    out["async_error"] = c.async_error()
    c.close()
    if r == 0:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
