"""The collectives bench.py makes over RCCL (backend "nccl"), on however many
ranks the launcher starts (one on a 1-GPU box: the calls are the same, the
ring is trivial).  Not a test of scaling; a check that the exact calls work on
this torch / ROCm:  python -m torch.distributed.run --nnodes=1 --nproc-per-node 1
--master-addr 127.0.0.1 --master-port 29561 tools/rccl_selftest.py"""
import json
import os

import torch
import torch.distributed as dist

ws, rank, local = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"]), int(os.environ["LOCAL_RANK"])
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
ids = [None] * ws
dist.all_gather_object(ids, f"rank{rank}")
dist.barrier()
t = torch.tensor([1.5 + rank], dtype=torch.float64, device="cuda")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
s = torch.tensor([1.0], dtype=torch.float64, device="cuda")
dist.all_reduce(s, op=dist.ReduceOp.SUM)
out = [torch.zeros_like(s) for _ in range(ws)]
dist.all_gather(out, s)
dist.barrier()
if rank == 0:
    print(json.dumps({"backend": dist.get_backend(), "world": ws, "ids": ids, "max": t.item(), "sum": s.item(),
                      "gather": [o.item() for o in out]}))
dist.destroy_process_group()
